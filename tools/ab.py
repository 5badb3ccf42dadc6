#!/usr/bin/env python3
"""Interleaved A/B timing of kernel variants in ONE process (cdna_hip_programming.md
section 5.4 rule 24): every round times each variant back to back on the same buffers, so
device-to-device and run-to-run drift does not masquerade as a kernel difference.

  python tools/ab.py [--rounds 12] [--reps 10] [--k 10 --m 3 --block 1024 --groups 100000]
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


if os.environ.get("QFEC_LIB"):  # an older build (tools/ab_lib.sh): knobs it predates are skipped
    _tune = qa.tune

    def _tune_compat(key, value):
        try:
            _tune(key, value)
        except qa.QfecError:
            pass
    qa.tune = _tune_compat


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=12)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--m", type=int, default=3)
    p.add_argument("--block", type=int, default=1024)
    p.add_argument("--groups", type=int, default=100_000)
    p.add_argument("--erasures", type=int, default=3)
    p.add_argument("--recon-only", action="store_true")
    p.add_argument("--encode-only", action="store_true")
    p.add_argument("--recon8", action="store_true", help="8-B-lane reconstruct variants only")
    p.add_argument("--only", default="", help="comma-separated variant-name prefixes ('_' for ' ')")
    p.add_argument("--patterns", type=int, default=0, help="draw each group's erasures from this many masks")
    p.add_argument("--pairs", action="store_true", help="time reconstruct right after encode, as bench.py does")
    p.add_argument("--probe-lds", default="0", help="reconstruct skeleton probe: LDS bytes per block to try")
    p.add_argument("--probe-sweep", default="", help="XOR probe block:lds pairs")
    p.add_argument("--enc-sweep", default="", help="encode block:lds[:impl] triples, e.g. 64:16384,256:65536:2")
    a = p.parse_args()
    k, m, B, G = a.k, a.m, a.block, a.groups
    dev = torch.device("cuda:0")
    pitch = (B + 15) // 16 * 16
    code = qa.Code.cauchy(k, m)
    data = torch.empty((G, k, pitch), dtype=torch.uint8, device=dev)
    qa.synth_fill(data, 0x5EED0002)
    par = torch.empty((G, m, pitch), dtype=torch.uint8, device=dev)
    gm = erasure_marks(0x5EED0003, G, k + m, a.erasures)
    if a.patterns:  # only `patterns` distinct erasure masks (their decode records stay cache-resident)
        import numpy as np
        pick = np.random.default_rng(7).integers(0, a.patterns, G)
        gm = gm[:a.patterns][pick]
    marks = torch.from_numpy(marks_to_rs_layout(gm, k)).to(dev)
    work = data.clone()
    # the erased data rows poisoned: every reconstruct variant must rebuild them (checked in round 0)
    lost = torch.from_numpy(gm[:, :k].astype(bool)).to(dev)
    damaged = data.clone()
    damaged[lost] = 0x5A
    code.encode(data, par, B)
    code.prepare_reconstruct()
    dec_groups = int((gm[:, :k].sum(1) > 0).sum())
    enc_bytes = (k + m) * B * G
    dec_bytes = (k * dec_groups + int(gm[:, :k].sum())) * B
    ref_par = par.clone()

    def enc():
        code.encode(data, par, B)

    def rec():
        code.reconstruct(work, par, marks, B)

    probe_out = torch.empty_like(par)

    def probe():  # into its own buffer: the reconstruct variants read par
        qa.probe_stream(data, probe_out, B)

    def pair_enc():  # bench.py's order: reconstruct right after an encode
        code.encode(data, par, B)

    variants = [
        ("encode auto (the library's own choice)", lambda: qa.tune("encode_impl", -1), enc, enc_bytes),
        ("encode impl0 (all rows)", lambda: qa.tune("encode_impl", 0), enc, enc_bytes),
        ("encode impl2 (inputs in halves)", lambda: qa.tune("encode_impl", 2), enc, enc_bytes),
        ("encode ldslog", lambda: (qa.tune("encode_impl", 0), qa.set_kernel_variant(1)), enc, enc_bytes),
        ("probe xor (traffic only)", lambda: None, probe, enc_bytes),
        ("recon auto (the library's own choice)", lambda: qa.tune("recon_impl", -1), rec, dec_bytes),
        ("recon impl2 (exact e rows, 16-B lanes)", lambda: qa.tune("recon_impl", 2), rec, dec_bytes),
        ("recon impl3 (exact e, 8-B lanes)", lambda: qa.tune("recon_impl", 3), rec, dec_bytes),
        ("recon impl4 (exact e, 12-B lanes)", lambda: qa.tune("recon_impl", 4), rec, dec_bytes),
        ("recon impl8 (impl3, one group per block)", lambda: qa.tune("recon_impl", 8), rec, dec_bytes),
    ]

    for spec in [x for x in a.enc_sweep.split(",") if x]:
        f = [int(v) for v in spec.split(":")]
        bs, lds, im = f[0], f[1], (f[2] if len(f) > 2 else 0)
        variants.append((f"encode bs{bs} lds{lds} impl{im}",
                         lambda bs=bs, lds=lds, im=im: (qa.tune("encode_impl", im), qa.tune("encode_block", bs),
                                                        qa.tune("encode_lds", lds)), enc, enc_bytes))
    for spec in [x for x in a.probe_sweep.split(",") if x]:
        bs, lds = (int(v) for v in spec.split(":"))
        variants.append((f"probe xor bs{bs} lds{lds}", lambda bs=bs, lds=lds: (qa.tune("encode_block", bs),
                                                                             qa.tune("encode_lds", lds)), probe, enc_bytes))
    skel = data.clone()

    # the reconstruct's memory skeleton (XOR, garbage into skel's erased rows) at LDS residency caps
    for lds in [int(x) for x in a.probe_lds.split(",")]:
        variants.append((f"probe recon lds{lds} (reconstruct skeleton)", lambda: None,
                         lambda lds=lds: qa.probe_reconstruct(skel, par, marks, B, lds), dec_bytes))
    variants.append(("recon impl8 again (drift check)", lambda: qa.tune("recon_impl", 8), rec, dec_bytes))

    if a.recon_only:
        variants = [v for v in variants if v[0].startswith(("recon impl2", "recon impl3", "recon impl4", "probe"))]
    if a.only:
        variants = [v for v in variants if v[0].startswith(tuple(x.replace("_", " ") for x in a.only.split(",")))]
    if a.recon8:
        variants = [v for v in variants if v[0].startswith(("recon impl3", "recon impl2", "recon impl4", "probe"))]
    if a.encode_only:
        variants = [v for v in variants if v[0].startswith(("encode impl0", "encode impl2", "probe"))]
    if a.pairs:
        variants = []
    times = {v[0]: [] for v in variants}
    s = torch.cuda.current_stream()
    for r in range(a.rounds):
        for name, setup, fn, _ in variants:
            qa.set_kernel_variant(0)
            qa.tune("encode_lds", -1)
            qa.tune("encode_block", -1)
            setup()
            if r == 0 and fn is rec:
                work.copy_(damaged)
            fn()
            if r == 0 and fn is rec:
                torch.cuda.synchronize()
                assert torch.equal(work[..., :B], data[..., :B]), f"{name}: wrong output"
                print(f"  {name}: output checked", flush=True)
            if r == 0 and fn is enc:
                torch.cuda.synchronize()
                assert torch.equal(par[..., :B], ref_par[..., :B]), f"{name}: wrong parity"
                print(f"  {name}: parity checked", flush=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.reps)
    if a.pairs:
        qa.tune("recon_impl", -1)
        scratch = torch.empty_like(par)

        def enc_other():  # same encode, parity into a buffer reconstruct does not read
            code.encode(data, scratch, B)

        def enc_sleep():
            code.encode(data, par, B)
            torch.cuda._sleep(100000)

        befores = [("after encode", enc), ("after encode into another buffer", enc_other),
                   ("after encode + ~50us sleep", enc_sleep),
                   ("after XOR probe (same traffic, light VALU)", lambda: qa.probe_stream(data, scratch, B)),
                   ("after 200us sleep", lambda: torch.cuda._sleep(400000)), ("after reconstruct", rec)]
        for impl in (2, 3):
            qa.tune("recon_impl", impl)
            for label, before in befores:
                tr = []
                for r in range(a.rounds * a.reps):
                    e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(2))
                    before()
                    e1.record(s)
                    rec()
                    e2.record(s)
                    torch.cuda.synchronize()
                    tr.append(e1.elapsed_time(e2))
                med = statistics.median(tr)
                print(f"  reconstruct impl{impl} {label:44s} median {med*1e3:7.1f} us -> "
                      f"{dec_bytes/(med*1e-3)/1e9:7.1f} GB/s")
        qa.tune("recon_impl", -1)
    qa.set_kernel_variant(0)
    qa.tune("encode_impl", -1)
    qa.tune("recon_impl", -1)
    qa.tune("encode_lds", -1)
    qa.tune("encode_block", -1)
    code.encode(data, par, B)
    torch.cuda.synchronize()
    assert torch.equal(par, ref_par)
    print(f"RS({k},{m}) B={B} G={G}: {a.rounds} interleaved rounds x {a.reps} launches")
    for name, _, _, nbytes in variants:
        t = times[name]
        med, mn = statistics.median(t), min(t)
        print(f"  {name:28s} median {med*1e3:8.1f} us  min {mn*1e3:8.1f} us  -> {nbytes/(med*1e-3)/1e9:7.1f} GB/s "
              f"(best {nbytes/(mn*1e-3)/1e9:7.1f})")


if __name__ == "__main__":
    main()
