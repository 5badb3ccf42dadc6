#!/usr/bin/env python3
"""HBM rate of a plain streaming kernel at several read:write mixes (qfec_probe_stream: k rows
read, m rows written per group, XOR only), the memory-side ceiling each datagram kernel is
compared with in DESIGN 9.2: 10:3 (the encode), 1:1 (the receive: datagrams in, rows out),
10:13 (the send: payloads in, datagrams out), 1:3.  Prints GB/s of (k + m) * B * G per launch.

  python tools/mix_probe.py [--bytes 1.3e9]
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
    ap.add_argument("--bytes", type=float, default=1.3e9)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B = 1024
    s = torch.cuda.current_stream()
    for k, m in ((10, 3), (1, 1), (10, 10), (10, 13), (1, 3)):
        G = int(a.bytes // ((k + m) * B))
        data = torch.empty((G, k, B), dtype=torch.uint8, device=dev)
        qa.synth_fill(data, 7)
        par = torch.empty((G, m, B), dtype=torch.uint8, device=dev)
        for _ in range(3):
            qa.probe_stream(data, par, B)
        times = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                qa.probe_stream(data, par, B)
            e1.record(s)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / a.reps)
        ms = statistics.median(times)
        print(f"read:write {k}:{m}  G={G}  {ms:.3f} ms  {(k + m) * B * G / ms / 1e6:.0f} GB/s", flush=True)
        del data, par
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
