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
    p.add_argument("--lanes", type=int, default=None)
    p.add_argument("--ab", default="", help="KNOB=V1,V2,...: interleaved in-process A/B of a host knob")
    p.add_argument("--rounds", type=int, default=8)
    p.add_argument("--scattered", action="store_true", help="--ab: rows at permuted places in memory")
    p.add_argument("--devices", default="", help="qfec_rs_host_devices list, e.g. 0,0 (default: the current device)")
    a = p.parse_args()
    torch.cuda.set_device(0)
    for key, v in (("host_threads", a.threads), ("host_chunk", a.chunk), ("host_zero_copy", a.zero_copy),
                   ("host_lanes", a.lanes)):
        if v is not None:
            try:
                qa.tune(key, v)
            except Exception as exc:
                print(f"# {key}: {exc}", file=sys.stderr)
    if a.ab:
        key, vals = a.ab.split("=")
        ab(key, [int(x) for x in vals.split(",")], a.rounds, G=a.groups, scattered=a.scattered)
        return
    if a.devices:
        print("# rs_host_devices", qa.rs_host_devices([int(x) for x in a.devices.split(",")]), file=sys.stderr)
    r = rs_abi_host_leg(G=a.groups, reps=a.reps)
    r.pop("_sample", None)
    print(json.dumps(r), flush=True)



def ab(key, values, rounds, G=100_000, k=10, m=3, B=1024, E=3, scattered=False):
    """Interleaved A/B of one host knob in ONE process on the same buffers: each round runs one
    encode + reconstruct pass per value, alternating; medians per value.  scattered: every row its
    own place in memory (a permutation of the rows), as rows of a socket buffer pool would be."""
    import ctypes as C
    import time
    import numpy as np
    from quicknet_amd.synth import erasure_marks, marks_to_rs_layout, synth_bytes
    n = k + m
    data0 = synth_bytes(0x5EED0005, G * k * B).reshape(G, k, B)
    data = data0.copy()
    par = np.zeros((G, m, B), np.uint8)
    rows = np.arange(G * n, dtype=np.uint64)
    if scattered:
        rows = np.random.default_rng(1).permutation(G * n).astype(np.uint64)
    pool = np.zeros((G * n, B), np.uint8)  # scattered: rows live here at permuted places
    base = pool.ctypes.data if scattered else None
    if scattered:
        pool[rows[:G * k].astype(np.int64)] = data0.reshape(G * k, B)
        ptr = (base + rows * B).astype(np.uint64)
    else:
        ptr = np.concatenate([data.ctypes.data + np.arange(G * k, dtype=np.uint64) * B,
                              par.ctypes.data + np.arange(G * m, dtype=np.uint64) * B]).astype(np.uint64)
    ptrs = (C.c_void_p * (G * n)).from_buffer(ptr)
    gm = erasure_marks(0x5EED0005 ^ 0xD, G, n, E)
    marks = np.ascontiguousarray(marks_to_rs_layout(gm, k))
    lost_rows = np.nonzero(marks[:G * k])[0]
    rs = qa.ReedSolomon(k, m)
    L = qa.lib()
    t = {v: ([], []) for v in values}
    for r in range(rounds + 1):
        for v in values:
            qa.tune(key, v)
            t0 = time.perf_counter()
            assert L.reed_solomon_encode(rs._h, ptrs, G * n, B) == 0
            t1 = time.perf_counter()
            if scattered:
                pool[rows[lost_rows].astype(np.int64)] = 0x5A
            else:
                data.reshape(G * k, B)[lost_rows] = 0x5A
            t2 = time.perf_counter()
            assert L.reed_solomon_reconstruct(rs._h, ptrs, C.c_void_p(marks.ctypes.data), G * n, B) == 0
            t3 = time.perf_counter()
            if r:
                t[v][0].append(t1 - t0)
                t[v][1].append(t3 - t2)
    got = pool[rows[:G * k].astype(np.int64)].reshape(G, k, B) if scattered else data
    assert np.array_equal(got, data0)
    dec = int((gm[:, :k].sum(1) > 0).sum())
    for v in values:
        te, tr = float(np.median(t[v][0])), float(np.median(t[v][1]))
        print(json.dumps({"knob": key, "value": v, "scattered": scattered, "rounds": rounds,
                          "gibs": round((G + dec) * k * B / (te + tr) / 2**30, 2),
                          "encode_ms": round(te * 1e3, 2), "reconstruct_ms": round(tr * 1e3, 2)}), flush=True)
    rs.close()


if __name__ == "__main__":
    main()
