#!/usr/bin/env python3
"""Interleaved A/B of the encode (and its XOR probe) against a cap on waves per CU: a dynamic LDS
allocation per block, tuning "encode_lds" (-1 auto, 0 none, else bytes per block).  RS(10,3)
B=1024 100 000 groups, RS(16,4) B=1400 250 000 groups, other shapes ~1.3 GB; each round times
every setting back to back on the same buffers.  The reconstruct is timed beside them (round 5
measured it under caps too, profiles/r05ak: it loses with any, and has none).

  python tools/occ_ab.py [--rounds 8] [--reps 10]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import quicknet_amd as qa  # noqa: E402
from quicknet_amd.synth import erasure_marks, marks_to_rs_layout  # noqa: E402

LDS = (-1, 0, 40960, 65536)


def shape(k, m, B, G, e, seed):
    dev = torch.device("cuda:0")
    pitch = (B + 15) // 16 * 16
    code = qa.Code.cauchy(k, m)
    data = torch.empty((G, k, pitch), dtype=torch.uint8, device=dev)
    qa.synth_fill(data, seed)
    par = torch.empty((G, m, pitch), dtype=torch.uint8, device=dev)
    gm = erasure_marks(seed + 1, G, k + m, e)
    marks = torch.from_numpy(marks_to_rs_layout(gm, k)).to(dev)
    work = data.clone()
    qa.tune("encode_lds", 0)
    code.encode(data, par, B)
    qa.tune("encode_lds", -1)
    ref = par.clone()
    code.prepare_reconstruct()
    dec_groups = int((gm[:, :k].sum(1) > 0).sum())
    enc_bytes = (k + m) * B * G
    dec_bytes = (k * dec_groups + int(gm[:, :k].sum())) * B
    return dict(code=code, data=data, par=par, scratch=torch.empty_like(par), ref=ref, work=work, marks=marks, B=B, enc=enc_bytes, dec=dec_bytes)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=8)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--lds", default=",".join(map(str, LDS)))
    p.add_argument("--shapes", default="10,3,1024;16,4,1400", help="k,m,B[,groups];... (groups default: the bench's, else ~1.3 GB)")
    p.add_argument("--encode-only", action="store_true")
    p.add_argument("--probe", action="store_true", help="time the XOR probe of each shape too")
    a = p.parse_args()
    ldss = [int(x) for x in a.lds.split(",")]
    shapes = {}
    for i, sh in enumerate(a.shapes.split(";")):
        k, m, B, *g = (int(x) for x in sh.split(","))
        G = g[0] if g else 250_000 if (k, m, B) == (16, 4, 1400) else 100_000 if (k, m, B) == (10, 3, 1024) else int(1.3e9 // ((k + m) * B))
        shapes[f"RS({k},{m}) B={B} G={G}"] = shape(k, m, B, G, m, 0x5EED0002 + 16 * i)
    s = torch.cuda.current_stream()
    times = {}
    for r in range(a.rounds):
        for sname, S in shapes.items():
            kinds = ("encode",) if a.encode_only else ("encode", "reconstruct")
            for kind in kinds + (("probe",) if a.probe else ()):
                for lds in ldss if kind != "reconstruct" else (-1,):
                    qa.tune("encode_lds", lds)
                    if kind == "probe":
                        fn = lambda: qa.probe_stream(S["data"], S["scratch"], S["B"])  # noqa: E731
                    elif kind == "encode":
                        fn = lambda: S["code"].encode(S["data"], S["par"], S["B"])  # noqa: E731
                    else:
                        fn = lambda: S["code"].reconstruct(S["work"], S["par"], S["marks"], S["B"])  # noqa: E731
                    fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(a.reps):
                        fn()
                    e1.record(s)
                    torch.cuda.synchronize()
                    times.setdefault((sname, kind, lds), []).append(e0.elapsed_time(e1) / a.reps)
                qa.tune("encode_lds", -1)
    ok = True
    for sname, S in shapes.items():
        ok &= bool(torch.equal(S["par"], S["ref"])) and bool(torch.equal(S["work"], S["data"]))
    for (sname, kind, lds), t in times.items():
        S = shapes[sname]
        ms = statistics.median(t)
        nb = S["dec"] if kind == "reconstruct" else S["enc"]
        print(f"{sname} {kind:11s} lds {lds:6d}  median {ms * 1e3:7.1f} us  min {min(t) * 1e3:7.1f}  "
              f"frac {nb / (ms * 1e-3) / 8e12:.4f}", flush=True)
    print("outputs identical to the uncapped run:", ok)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
