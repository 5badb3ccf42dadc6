#!/usr/bin/env python3
"""Rate of the ProtocolUdp framing kernels (qfec_frame_udp / qfec_unframe_udp) on the bench's
datagram batch: RS(10,13) x 100 000 groups of 1 KiB payloads packed at a 1088-B wire pitch,
1.3 M datagrams of 1 041 B framed (FEC cmd/protocol, no Session prefix) and unframed again,
checked to round-trip.  Minimal traffic: bytes in + bytes out per row.

  python tools/frame_bench.py [--groups 100000 --rounds 5 --reps 10 --variants "base;..."]
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
    ap.add_argument("--groups", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="base")
    ap.add_argument("--out-pitch", type=int, default=0, help="frame row pitch (0: 16-B rounding)")
    a = ap.parse_args()
    k, n, S, G = 10, 13, 1024, a.groups
    dev = torch.device("cuda:0")
    code = qa.Code.vandermonde(k, n - k)
    payload = torch.empty(G * k * S + 16, dtype=torch.uint8, device=dev)
    qa.synth_fill(payload, 5)
    offs = torch.arange(G * k, dtype=torch.int64, device=dev) * S
    sizes = torch.full((G * k,), S, dtype=torch.int32, device=dev)
    seq = torch.zeros((G, 2), dtype=torch.int32, device=dev)
    _, wire, wlen = code.pack_datagrams(payload, offs, sizes, seq, True, shard_pitch=1040, wire_pitch=1088)
    rows = wire.view(G * n, 1088)
    lens = wlen.view(-1).contiguous()
    masks = (torch.arange(G * n, device=dev) & 0xFF).to(torch.uint8)
    R = G * n
    op = a.out_pitch or None
    framed, flen = qa.frame_udp(rows, lens, masks, gmask=0x3C, out_pitch=op)
    data, dlen, status, _, _ = qa.unframe_udp(framed, flen, gmask=0x3C, out_pitch=1088)
    torch.cuda.synchronize()
    ok = bool((status == 0).all()) and torch.equal(dlen, lens)
    L = int(lens.max())
    ok = ok and torch.equal(data[:, :L] * (torch.arange(L, device=dev)[None, :] < lens[:, None]),
                            rows[:, :L] * (torch.arange(L, device=dev)[None, :] < lens[:, None]))
    s = torch.cuda.current_stream()
    fns = {"frame": lambda: qa.frame_udp(rows, lens, masks, gmask=0x3C, out_pitch=op),
           "unframe": lambda: qa.unframe_udp(framed, flen, gmask=0x3C, out_pitch=1088)}
    for spec in a.variants.split(";"):
        if spec != "base":
            for kv in spec.split(","):
                kk, v = kv.split("=")
                qa.tune(kk, int(v))
        t = {x: [] for x in fns}
        for _ in range(a.rounds):
            for name, fn in fns.items():
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.reps):
                    fn()
                e1.record(s)
                torch.cuda.synchronize()
                t[name].append(e0.elapsed_time(e1) / a.reps)
        nbytes = int(lens.sum()) * 2 + 4 * R
        for name in fns:
            ms = statistics.median(t[name])
            print(f"{spec:24s} {name:8s} {R} rows of {S + 17} B: {ms * 1e3:8.1f} us  {nbytes / ms / 1e6:7.1f} GB/s "
                  f"({nbytes / ms / 1e6 / 8000:.3f} of 8 TB/s, bytes in + out), verified {ok}", flush=True)


if __name__ == "__main__":
    main()
