#!/usr/bin/env python3
"""Per-call cost of the unchanged drop-in (fec_encode / fec_decode on host packets, RS(10,3),
sz 1028) under qfec_tune knob settings, alternated in one process; medians over rounds.

  python tools/percall_ab.py [--variants "percall_resident=1;percall_resident=0" --rounds 5 --reps 2000]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
bench._load()
import quicknet_amd as qa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="percall_resident=1;percall_resident=0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=2000)
    ap.add_argument("--ref", action="store_true", help="also time the reference fec.c per-call on this CPU")
    a = ap.parse_args()
    res = {v: {"enc": [], "dec": [], "grp": []} for v in a.variants.split(";")}
    for _ in range(a.rounds):
        for v in res:
            for kv in v.split(","):
                kk, val = kv.split("=")
                qa.tune(kk, int(val))
            out = bench.per_call_leg(reps=a.reps, batched=False)
            res[v]["enc"].append(out["gpu_fec_encode_us"])
            res[v]["dec"].append(out["gpu_fec_decode_us"])
            res[v]["grp"].append(out.get("gpu_fec_encode_group_us", float("nan")))
    if a.ref:  # the reference system/fec.c on this box's CPU, same harness (oracle/_ref build)
        from oracle.oracle import RefCodec
        out = bench.per_call_leg(reps=a.reps, ref_lib=RefCodec().fec, batched=False)
        print("reference CPU:", {kk: vv for kk, vv in out.items() if kk.startswith("ref_cpu_")})
    for v, r in res.items():
        print(f"{v:28s} fec_encode {statistics.median(r['enc']):7.2f} us  fec_decode {statistics.median(r['dec']):7.2f} us"
              f"  group {statistics.median(r['grp']):7.2f} us  (min {min(r['enc']):.2f} / {min(r['dec']):.2f} / {min(r['grp']):.2f})")


if __name__ == "__main__":
    main()
