#!/usr/bin/env python3
"""Interleaved A/B timing of the fused datagram send's tuning knobs (qfec_tune) in one
process, on the same buffers; every variant's wire output is checked identical.

  python tools/wire_ab.py [--k 10 --n 13 --size 1024 --groups 100000 --rounds 10 --reps 10]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import quicknet_amd as qa  # noqa: E402

KNOBS = {"wire_fused": 1, "wire_rx": 1}

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
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--n", type=int, default=13)
    p.add_argument("--size", type=int, default=1024)
    p.add_argument("--groups", type=int, default=100_000)
    p.add_argument("--rounds", type=int, default=10)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--variants", default="base;wire_fused=0")
    p.add_argument("--unpack", action="store_true", help="time qfec_unpack_datagrams (n - k losses per group)")
    p.add_argument("--align", type=int, default=16, help="shard and wire row pitches rounded to this (16 or 64)")
    p.add_argument("--wire-align", type=int, default=0, help="wire row pitch rounded to this instead (e.g. 64)")
    a = p.parse_args()
    k, n, G, S = a.k, a.n, a.groups, a.size
    dev = torch.device("cuda:0")
    code = qa.Code.vandermonde(k, n - k)
    sizes = torch.full((G * k,), S, dtype=torch.int32, device=dev)
    offs = torch.arange(G * k, dtype=torch.int64, device=dev) * S
    payload = torch.empty(G * k * S + 16, dtype=torch.uint8, device=dev)
    qa.synth_fill(payload, 77)
    seq = torch.stack([torch.arange(G, dtype=torch.int32, device=dev) * n,
                       torch.arange(G, dtype=torch.int32, device=dev) * k], 1).contiguous()
    head = 4
    A = a.align
    pitch = (S + head + A - 1) // A * A
    WA = a.wire_align or A
    wpitch = (pitch + 13 + WA - 1) // WA * WA
    row16 = (S + head + 15) // 16 * 16  # the shard bytes a row carries, for the traffic count
    shards = torch.empty((G, n, pitch), dtype=torch.uint8, device=dev)
    wire = torch.zeros((G, n, wpitch), dtype=torch.uint8, device=dev)
    wlen = torch.empty((G, n), dtype=torch.int32, device=dev)

    def pack():
        qa.lib().qfec_pack_datagrams(code._h, payload.data_ptr(), offs.data_ptr(), sizes.data_ptr(), seq.data_ptr(), G, 1,
                                     shards.data_ptr(), pitch, wire.data_ptr(), wpitch, wlen.data_ptr(), None)

    if a.unpack:
        import numpy as np
        pack()
        torch.cuda.synchronize()
        rng = np.random.default_rng(5)
        lost = np.zeros((G, n), bool)
        for g in range(G):
            lost[g, rng.choice(n, n - k, replace=False)] = True
        rx_len = torch.where(torch.from_numpy(lost).to(dev), torch.zeros_like(wlen), wlen).contiguous()
        marks = torch.empty(G * n, dtype=torch.uint8, device=dev)
        rx = torch.empty((G, n), dtype=torch.int32, device=dev)
        status = torch.empty((G, k), dtype=torch.int32, device=dev)
        psize = torch.empty((G, k), dtype=torch.int32, device=dev)
        wire_in = wire.clone()

        def pack():  # noqa: F811 -- the timed call is the receive path
            qa.lib().qfec_unpack_datagrams(code._h, wire_in.data_ptr(), wpitch, rx_len.data_ptr(), G, 1, 2068,
                                           shards.data_ptr(), pitch, marks.data_ptr(), rx.data_ptr(),
                                           status.data_ptr(), psize.data_ptr(), None)

    def setup(spec):
        for kk, v in KNOBS.items():
            qa.tune(kk, v)
        if spec != "base":
            for kv in spec.split(","):
                kk, v = kv.split("=")
                qa.tune(kk, int(v))

    variants = a.variants.split(";")
    setup("base")
    pack()
    torch.cuda.synchronize()
    out_t, len_t = (shards, status) if a.unpack else (wire, wlen)
    ref = out_t.clone()
    ref_len = len_t.clone()
    times = {v: [] for v in variants}
    s = torch.cuda.current_stream()
    for _ in range(a.rounds):
        for v in variants:
            setup(v)
            pack()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                pack()
            e1.record(s)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.reps)
            if a.unpack:
                assert torch.equal(status, ref_len), v
                assert torch.equal(shards[:, :k], ref[:, :k]), v
            else:
                L = ref_len.max().item()
                assert torch.equal(wlen, ref_len), v
                assert torch.equal(wire[..., :L], ref[..., :L]) or v.startswith("wire_fused=0"), v
    setup("base")
    nbytes = G * k * S + int(wlen.sum().item())
    if a.unpack:  # received datagrams in, data rows out
        nbytes = int(rx_len.sum().item()) + G * k * row16
    print(f"{'unpack' if a.unpack else 'pack'} RS({k},{n}) payload {S} B, G={G}, pitch {pitch} / wire {wpitch}: "
          f"{a.rounds} rounds x {a.reps}")
    for v in variants:
        t = times[v]
        med = statistics.median(t)
        print(f"  {v:36s} median {med*1e3:8.1f} us  min {min(t)*1e3:8.1f} us -> {nbytes/(med*1e-3)/1e9:7.1f} GB/s min-traffic")


if __name__ == "__main__":
    main()
