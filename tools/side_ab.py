#!/usr/bin/env python3
"""Interleaved A/B of reconstruct bodies through bench.py's own side_config step (encode then
reconstruct, per-kernel HIP events), for both matrix flavours.

  python tools/side_ab.py [--rounds 6] [--impls 2,3] [--k 10 --m 3 --block 1024 --groups 100000]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import quicknet_amd as qa  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=6)
    p.add_argument("--impls", default="2,3")
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--m", type=int, default=3)
    p.add_argument("--block", type=int, default=1024)
    p.add_argument("--groups", type=int, default=100_000)
    p.add_argument("--erasures", type=int, default=3)
    a = p.parse_args()
    torch.cuda.set_device(0)
    impls = [int(x) for x in a.impls.split(",")]
    res = {}
    for _ in range(a.rounds):
        for fl in ("cauchy", "vandermonde"):
            for im in impls:
                qa.tune("recon_impl", im)
                r = bench.side_config(fl, a.k, a.m, a.block, a.groups, a.erasures, 1, 0)
                assert r["verified"], r
                res.setdefault((fl, im), []).append(r["reconstruct_frac"] * bench.HBM_PEAK_GBS)
    qa.tune("recon_impl", -1)
    print(f"RS({a.k},{a.m}) B={a.block} G={a.groups}, {a.erasures} erasures: reconstruct GB/s after encode, "
          f"{a.rounds} interleaved rounds of bench.side_config")
    for (fl, im), v in sorted(res.items()):
        print(f"  {fl:12s} impl{im}  median {statistics.median(v):7.1f}  min {min(v):7.1f}  max {max(v):7.1f}")


if __name__ == "__main__":
    main()
