#!/usr/bin/env python3
"""Encode against the XOR probe of the same traffic (qfec_probe_stream) at other shapes than the
headline's: how close each encode is to what its own traffic shape streams at on this chip.
Interleaved, medians over rounds.

  python tools/probe_shape.py [--shapes "10,3,1024,100000;16,4,1400,250000;4,2,1024,100000"]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import quicknet_amd as qa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="10,3,1024,100000;16,4,1400,250000;4,2,1024,100000")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    for spec in a.shapes.split(";"):
        k, m, B, G = (int(x) for x in spec.split(","))
        pitch = (B + 15) // 16 * 16
        data = torch.empty((G, k, pitch), dtype=torch.uint8, device=dev)
        qa.synth_fill(data, 99)
        parity = torch.empty((G, m, pitch), dtype=torch.uint8, device=dev)
        code = qa.Code.cauchy(k, m)
        fns = {"encode": lambda: code.encode(data, parity, B), "probe": lambda: qa.probe_stream(data, parity, B)}
        t = {x: [] for x in fns}
        for _ in range(a.rounds):
            for name, fn in fns.items():
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.reps):
                    fn()
                e1.record(s)
                torch.cuda.synchronize()
                t[name].append(e0.elapsed_time(e1) / a.reps)
        alg = (k + m) * B * G
        enc, prb = statistics.median(t["encode"]), statistics.median(t["probe"])
        print(f"RS({k},{m}) B={B} G={G}: encode {enc * 1e3:8.1f} us {alg / enc / 1e6:7.1f} GB/s ({alg / enc / 1e6 / 8000:.3f} of 8 TB/s)"
              f" | XOR probe {prb * 1e3:8.1f} us {alg / prb / 1e6:7.1f} GB/s | encode / probe {prb / enc:.3f}", flush=True)
        del data, parity
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
