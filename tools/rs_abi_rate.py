#!/usr/bin/env python3
"""bench.py's rs_abi_host leg alone: module/rs.h reed_solomon_encode + reed_solomon_reconstruct on
per-shard pointers into pageable host memory (RS(10,3) 1 KiB, config 2's shape).  For before/after
A/B of libqfec builds (tools/ab_lib.sh with QFEC_LIB / QFEC_LIB_COMPAT) and knob sweeps.

  python tools/rs_abi_rate.py [--groups 100000] [--reps 3] [--threads 0] [--chunk 0] [--zero-copy 1] [--devices 0,0]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import quicknet_amd as qa  # noqa: E402
from quicknet_amd.hoststream import rs_abi_host_leg  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--groups", type=int, default=100_000)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--threads", type=int, default=None)
    p.add_argument("--chunk", type=int, default=None)
    p.add_argument("--zero-copy", type=int, default=None)
    p.add_argument("--devices", default="", help="qfec_rs_host_devices list, e.g. 0,0 (default: the current device)")
    a = p.parse_args()
    torch.cuda.set_device(0)
    for key, v in (("host_threads", a.threads), ("host_chunk", a.chunk), ("host_zero_copy", a.zero_copy)):
        if v is not None:
            try:
                qa.tune(key, v)
            except Exception as exc:
                print(f"# {key}: {exc}", file=sys.stderr)
    if a.devices:
        print("# rs_host_devices", qa.rs_host_devices([int(x) for x in a.devices.split(",")]), file=sys.stderr)
    r = rs_abi_host_leg(G=a.groups, reps=a.reps)
    r.pop("_sample", None)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
