#!/usr/bin/env python3
"""Rate of the exact NetFecCodec layer (include/qfec_zfec.h) on one GPU: S sender sessions
packing P payloads each, one flush; their datagrams (a fraction dropped) into S receiver
sessions, one flush.  Prints payload GiB/s and packets/s for each flush and checks every
payload arrives (n - k losses per group are recoverable).

  python tools/zfec_rate.py [--sessions 64 --packets 2000 --size 1024 --k 10 --n 13 --loss 0.1]
"""
import argparse
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import quicknet_amd as qa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=64)
    ap.add_argument("--packets", type=int, default=2000)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n", type=int, default=13)
    ap.add_argument("--loss", type=float, default=0.1)
    ap.add_argument("--sorted", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--callbacks", type=int, default=0, help="1: time the receive flush with Python callbacks")
    a = ap.parse_args()
    rng = random.Random(1)
    pay = [rng.randbytes(a.size) for _ in range(257)]
    for rep in range(a.reps):
        z = qa.Zfec()
        tx = [z.session(max_pkt_size=2048, kmax=15, k=a.k, n=a.n, is_sorted=bool(a.sorted)) for _ in range(a.sessions)]
        rx = [z.session(max_pkt_size=2048, kmax=15, k=a.k, n=a.n, is_sorted=bool(a.sorted)) for _ in range(a.sessions)]
        t0 = time.perf_counter()
        for i, s in enumerate(tx):
            for p in range(a.packets):
                z.pack_input(s, pay[(i * 7 + p) % 257])
        t1 = time.perf_counter()
        sent, _ = z.flush()
        t2 = time.perf_counter()
        # drop at most n - k per group so every payload is recoverable
        per = {}
        for sess, d in sent:
            per.setdefault(sess, []).append(d)
        for i, s in enumerate(tx):
            ds = per.get(s, [])
            for g0 in range(0, len(ds), a.n):
                grp = ds[g0:g0 + a.n]
                drop = set(rng.sample(range(len(grp)), min(a.n - a.k, int(round(a.loss * len(grp))))))
                for j, d in enumerate(grp):
                    if j not in drop:
                        z.unpack_input(rx[i], d)
        t3 = time.perf_counter()
        if a.callbacks:
            _, got = z.flush()
            ndel = len(got)
        else:  # the layer alone: no callbacks, the return value counts the deliveries
            ndel = z._L.qfec_zfec_flush(z._h, None, None, None)
        t4 = time.perf_counter()
        npk = a.sessions * a.packets
        by = npk * a.size
        ok = ndel == npk
        got = range(ndel)
        print(f"rep {rep}: {a.sessions} sessions x {a.packets} x {a.size} B, RS({a.k},{a.n}), loss {a.loss}: "
              f"queue {t1 - t0:.3f}s, pack flush {t2 - t1:.3f}s ({by / (t2 - t1) / 2**30:.2f} GiB/s, "
              f"{npk / (t2 - t1) / 1e6:.2f} Mpkt/s), queue rx {t3 - t2:.3f}s, unpack flush {t4 - t3:.3f}s "
              f"({by / (t4 - t3) / 2**30:.2f} GiB/s, {npk / (t4 - t3) / 1e6:.2f} Mpkt/s), delivered {len(got)} ok={ok}",
              flush=True)
        z.close()


if __name__ == "__main__":
    main()
