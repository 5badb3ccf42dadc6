#!/usr/bin/env python3
"""Host-to-host FEC rate: payloads start and end in host memory (the UDP socket /
PacketBuffer side of the reference), so this includes the PCIe copies (BASELINE configs[4]:
mixed (k,m) streaming batches with pinned H2D/D2H overlap on HIP streams).

Per batch: H2D of the data shards (pinned) -> encode -> D2H of the parity shards, on one of
S streams round-robin, so copies of one batch overlap the kernel of another.  The device-
resident rate is bench.py's; this number goes to DESIGN.md, never into bench's `value`.

  python tools/host_rate.py [--streams 3] [--batch-mib 64] [--total-gib 4] [--mixed]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import quicknet_amd as qa  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--streams", type=int, default=3)
    p.add_argument("--batch-mib", type=int, default=64)
    p.add_argument("--total-gib", type=float, default=4.0)
    p.add_argument("--mixed", action="store_true", help="round-robin RS(4,2), RS(10,3) B=1024 and RS(16,4) B=1400")
    p.add_argument("--verify", action="store_true")
    a = p.parse_args()
    dev = torch.device("cuda:0")
    shapes = [(10, 3, 1024)] if not a.mixed else [(4, 2, 1024), (10, 3, 1024), (16, 4, 1400)]
    codes = {(k, m): qa.Code.cauchy(k, m) for k, m, _ in shapes}
    S = a.streams
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    plan = []  # (k, m, B, pitch, groups)
    for k, m, B in shapes:
        pitch = (B + 15) // 16 * 16
        groups = max(1, (a.batch_mib << 20) // (k * pitch))
        plan.append((k, m, B, pitch, groups))
    nb = max(len(plan), int(a.total_gib * (1 << 30) // (a.batch_mib << 20)))
    # host side: one pinned input and output ring per stream, per shape
    h_in, h_out, d_in, d_out = {}, {}, {}, {}
    for s in range(S):
        for k, m, B, pitch, groups in plan:
            key = (s, k, m)
            h_in[key] = torch.empty((groups, k, pitch), dtype=torch.uint8).pin_memory()
            h_out[key] = torch.empty((groups, m, pitch), dtype=torch.uint8).pin_memory()
            d_in[key] = torch.empty((groups, k, pitch), dtype=torch.uint8, device=dev)
            d_out[key] = torch.empty((groups, m, pitch), dtype=torch.uint8, device=dev)
            h_in[key].copy_(torch.randint(0, 256, h_in[key].shape, dtype=torch.uint8))

    used = set()

    def run(n):
        data_bytes = 0
        for i in range(n):
            k, m, B, pitch, groups = plan[i % len(plan)]
            s = i % S
            key = (s, k, m)
            used.add(key)
            with torch.cuda.stream(streams[s]):
                d_in[key].copy_(h_in[key], non_blocking=True)
                codes[(k, m)].encode(d_in[key], d_out[key], B, stream=streams[s])
                h_out[key].copy_(d_out[key], non_blocking=True)
            data_bytes += groups * k * B
        torch.cuda.synchronize()
        return data_bytes

    run(len(plan) * S)  # warm-up
    t0 = time.perf_counter()
    nbytes = run(nb)
    el = time.perf_counter() - t0
    if a.verify:  # against a device-resident encode of the same batch (itself oracle-tested in tests/)
        for (s, k, m), hi in h_in.items():
            if (s, k, m) not in used:
                continue
            B = [p for p in plan if p[0] == k][0][2]
            dref = torch.zeros((hi.shape[0], m, hi.shape[2]), dtype=torch.uint8, device="cuda")
            codes[(k, m)].encode(hi.cuda(), dref, B)
            torch.cuda.synchronize()
            assert torch.equal(dref.cpu()[..., :B], h_out[(s, k, m)][..., :B])
    out = {"host_to_host_data_gibs": round(nbytes / el / (1 << 30), 2), "batches": nb, "streams": S,
           "batch_mib": a.batch_mib, "shapes": [f"RS({k},{m}) B={B}" for k, m, B in shapes],
           "seconds": round(el, 3), "verified": bool(a.verify)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
