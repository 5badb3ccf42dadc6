#!/usr/bin/env python3
"""Throughput of the FEC datagram batch path (qfec_pack_datagrams / qfec_unpack_datagrams):
G groups of k packets -> shards -> check shards -> n datagrams each, and back with m losses
per group.  Device-resident; reports payload GiB/s per direction and each stage's time.

  python tools/wire_bench.py [--k 10 --n 13 --size 1024 --groups 100000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import quicknet_amd as qa  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--n", type=int, default=13)
    p.add_argument("--size", type=int, default=1024, help="payload bytes per packet")
    p.add_argument("--groups", type=int, default=100_000)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--cpu-seconds", type=float, default=5.0)
    p.add_argument("--staged", action="store_true", help="force the 3-kernel send pipeline")
    a = p.parse_args()
    qa.tune("wire_fused", 0 if a.staged else 1)
    k, n, G, S = a.k, a.n, a.groups, a.size
    dev = torch.device("cuda:0")
    code = qa.Code.vandermonde(k, n - k)
    sizes = torch.full((G * k,), S, dtype=torch.int32, device=dev)
    offs = torch.arange(G * k, dtype=torch.int64, device=dev) * S
    payload = torch.empty(G * k * S + 16, dtype=torch.uint8, device=dev)
    qa.synth_fill(payload, 77)
    seq = torch.stack([torch.arange(G, dtype=torch.int32, device=dev) * n,
                       torch.arange(G, dtype=torch.int32, device=dev) * k], 1).contiguous()
    shards, wire, wlen = code.pack_datagrams(payload, offs, sizes, seq, True)
    # drop n-k datagrams of every group (data packets first: worst case for decode)
    rng = np.random.default_rng(5)
    lost = np.zeros((G, n), bool)
    for g in range(G):
        lost[g, rng.choice(n, n - k, replace=False)] = True
    rx_len = torch.where(torch.from_numpy(lost).to(dev), torch.zeros_like(wlen), wlen).contiguous()
    out = code.unpack_datagrams(wire, rx_len, True, shard_pitch=shards.shape[2])
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()

    def timed(fn):
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    t_pack = timed(lambda: code.pack_datagrams(payload, offs, sizes, seq, True))
    t_unpack = timed(lambda: code.unpack_datagrams(wire, rx_len, True, shard_pitch=shards.shape[2]))
    # correctness on the measured buffers
    sh, status, psize, rx = out
    ok = bool((status == 4).all().item())
    pl = payload[:-16].view(G, k, S)
    ok = ok and bool(torch.equal(sh[:, :k, 4:4 + S], pl))
    gib = G * k * S / float(1 << 30)
    pitch = shards.shape[2]
    wire_bytes = int(wlen.sum().item())
    cpu = None  # the reference CPU pipeline is timed by bench.py's cpu_baseline leg ("wire")
    print(json.dumps({
        "send_path": "staged" if a.staged else "fused",
        "workload": f"{G} groups x RS({k},{n}) x {S}-B payloads, checksum on, {n - k} random losses/group",
        "pack_ms": round(t_pack, 4), "pack_payload_gibs": round(gib / (t_pack * 1e-3), 1),
        "unpack_ms": round(t_unpack, 4), "unpack_payload_gibs": round(gib / (t_unpack * 1e-3), 1),
        # bytes each direction must at least move: payload in + datagrams out (pack);
        # datagrams in + recovered shards out (unpack), ignoring the scratch shard matrix
        "pack_min_bytes_gbs": round((G * k * S + wire_bytes) / (t_pack * 1e-3) / 1e9, 1),
        "shard_pitch": pitch, "verified": ok, "cpu_baseline": cpu,
    }))


if __name__ == "__main__":
    main()
