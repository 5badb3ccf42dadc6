#!/usr/bin/env python3
"""bench.py's side legs alone, for the profilers: the same functions, shapes, spin-up and
launch path as the JSON line's `wire` field (datagrams and one-pass frames, RS(10,13), 100 000
groups x 1 KiB payloads), with more timed launches so that rocprofv3 averages over steady-state
launches.  Prints the leg's JSON record.

  python tools/side_legs.py [--steps 100]
  rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/side_legs.py --steps 100
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    a = ap.parse_args()
    bench._load()
    bench.torch.cuda.set_device(0)
    print(json.dumps(bench.wire_leg(0, steps=a.steps, warmup=a.warmup)), flush=True)


if __name__ == "__main__":
    main()
