#!/usr/bin/env python3
"""Host-to-host encode rate through the C ABI (qfec_encode_host): RS(k,m) over G groups in
host memory, pageable (numpy) and pinned (torch pin_memory) buffers; verified against a
device-resident encode of the same data.

  python tools/host_abi_rate.py [--k 10 --m 3 --block 1024 --groups 100000 --reps 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import quicknet_amd as qa  # noqa: E402

GIB = float(1 << 30)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--m", type=int, default=3)
    p.add_argument("--block", type=int, default=1024)
    p.add_argument("--groups", type=int, default=100_000)
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    k, m, B, G = a.k, a.m, a.block, a.groups
    code = qa.Code.cauchy(k, m)
    dd = torch.empty((G, k, B), dtype=torch.uint8, device="cuda:0")
    qa.synth_fill(dd, 0x5EED0002)
    dp = torch.empty((G, m, B), dtype=torch.uint8, device="cuda:0")
    code.encode(dd, dp, B)
    ref = dp.cpu().numpy()
    host = dd.cpu().numpy()
    bufs = {"pageable": (host, np.zeros((G, m, B), np.uint8)),
            "pinned": (torch.from_numpy(host).pin_memory(), torch.zeros((G, m, B), dtype=torch.uint8).pin_memory())}
    print(f"RS({k},{m}) B={B} G={G}: {G * k * B / 1e9:.3f} GB of data per call, host -> device -> host")
    for name, (hd, hp) in bufs.items():
        code.encode_host(hd, hp, B)  # warm: staging and streams
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            code.encode_host(hd, hp, B)
            ts.append(time.perf_counter() - t0)
        got = hp if isinstance(hp, np.ndarray) else hp.numpy()
        ok = np.array_equal(got, ref)
        t = min(ts)
        print(f"  {name:9s} best {t * 1e3:8.2f} ms -> {G * k * B / t / GIB:7.2f} GiB/s of data "
              f"({G * (k + m) * B / t / 1e9:6.2f} GB/s over PCIe both ways), verified={ok}")
        assert ok
    # reconstruct, pageable buffers: 3 random erasures of 13 per group (bench's seed)
    from quicknet_amd.synth import erasure_marks, marks_to_rs_layout
    gm = erasure_marks(0x5EED0003, G, k + m, 3)
    marks = np.ascontiguousarray(marks_to_rs_layout(gm, k))
    dec_groups = int((gm[:, :k].sum(1) > 0).sum())
    ts = []
    for _ in range(a.reps):
        work = host.copy()
        work.reshape(G * k, B)[marks[: G * k] == 1] = 0x5A
        t0 = time.perf_counter()
        nf = code.reconstruct_host(work, ref, marks, B)
        ts.append(time.perf_counter() - t0)
        assert nf == 0 and np.array_equal(work, host)
    t = min(ts)
    print(f"  reconstruct (pageable) best {t * 1e3:8.2f} ms -> {dec_groups * k * B / t / GIB:7.2f} GiB/s of data "
          f"decoded, verified=True")


if __name__ == "__main__":
    main()
