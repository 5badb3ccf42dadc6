#!/usr/bin/env python3
"""Rate of the exact NetFecCodec layer (include/qfec_zfec.h) on one GPU: S sender sessions
packing P payloads each, one flush; their datagrams (a fraction dropped, at most n - k per
group so every payload is recoverable) into S receiver sessions, one flush.  Both flushes call
C callbacks (tools/zfec_sink.c: the send side copies every datagram out, as a socket layer
would; the receive side copies every delivery into an application ring and folds it into a
sum of 64-bit words), so the numbers are the layer's, not Python's.  Prints payload GiB/s and
packets/s per flush, and checks that every payload arrived (count, bytes, and the word sum of
all payloads sent).

  python tools/zfec_rate.py [--sessions 64 --packets 2000 --size 1024 --k 10 --n 13 --loss 0.1]
  --json: one JSON line with the best rep (bench.py's zfec field)
"""
import argparse
import ctypes as C
import json
import os
import random
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import quicknet_amd as qa  # noqa: E402
from quicknet_amd.codec import _PACK_OUT, _UNPACK_OUT  # noqa: E402

SINK_SRC = os.path.join(ROOT, "tools", "zfec_sink.c")
SINK_SO = os.path.join(ROOT, "tools", "_build", "libzfec_sink.so")


def load_sink():
    if not os.path.exists(SINK_SO) or os.path.getmtime(SINK_SO) < os.path.getmtime(SINK_SRC):
        os.makedirs(os.path.dirname(SINK_SO), exist_ok=True)
        subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-o", SINK_SO, SINK_SRC], check=True)
    s = C.CDLL(SINK_SO)
    s.sink_fold.argtypes = [C.c_char_p, C.c_uint]
    for f, t in (("sink_count", C.c_size_t), ("sink_buf", C.c_void_p), ("sink_offs", C.c_void_p),
                 ("sink_lens", C.c_void_p), ("sink_peers", C.c_void_p), ("sink_ndeliv", C.c_ulonglong),
                 ("sink_dbytes", C.c_ulonglong), ("sink_dsum", C.c_ulonglong), ("sink_fold", C.c_ulonglong)):
        getattr(s, f).restype = t
    return s


def run(a, sink, rep, pay):
    import numpy as np
    rng = random.Random(100 + rep)
    L = qa.lib()
    pack_cb = _PACK_OUT(C.cast(sink.sink_pack, C.c_void_p).value)
    unpack_cb = _UNPACK_OUT(C.cast(sink.sink_unpack, C.c_void_p).value)
    z = qa.Zfec()
    tx = [z.session(max_pkt_size=2048, kmax=15, k=a.k, n=a.n, is_sorted=bool(a.sorted)) for _ in range(a.sessions)]
    rx = [z.session(max_pkt_size=2048, kmax=15, k=a.k, n=a.n, is_sorted=bool(a.sorted)) for _ in range(a.sessions)]
    t0 = time.perf_counter()
    expect_sum = 0
    for i, s in enumerate(tx):
        for p in range(a.packets):
            j = (i * 7 + p) % len(pay)
            z.pack_input(s, pay[j][0])
            expect_sum += pay[j][1]
    t1 = time.perf_counter()
    sink.sink_reset()
    rc = L.qfec_zfec_flush(z._h, pack_cb, unpack_cb, None)
    t2 = time.perf_counter()
    assert rc >= 0, rc
    cnt = sink.sink_count()
    buf = C.string_at(sink.sink_buf(), int(np.ctypeslib.as_array((C.c_uint32 * cnt).from_address(sink.sink_offs()))[-1])
                      + int(np.ctypeslib.as_array((C.c_uint32 * cnt).from_address(sink.sink_lens()))[-1]))
    offs = np.ctypeslib.as_array((C.c_uint32 * cnt).from_address(sink.sink_offs())).copy()
    lens = np.ctypeslib.as_array((C.c_uint32 * cnt).from_address(sink.sink_lens())).copy()
    peers = np.ctypeslib.as_array((C.c_ssize_t * cnt).from_address(sink.sink_peers())).copy()
    per = {}
    for o, ln, pr in zip(offs, lens, peers):
        per.setdefault(int(pr) - 1, []).append(buf[int(o):int(o) + int(ln)])
    nlost = min(a.n - a.k, int(round(a.loss * a.n)))
    for i, s in enumerate(tx):
        ds = per.get(s, [])
        for g0 in range(0, len(ds), a.n):
            grp = ds[g0:g0 + a.n]
            drop = set(rng.sample(range(len(grp)), min(len(grp), nlost)))
            for j, d in enumerate(grp):
                if j not in drop:
                    z.unpack_input(rx[i], d)
    t3 = time.perf_counter()
    sink.sink_reset()
    rc = L.qfec_zfec_flush(z._h, pack_cb, unpack_cb, None)
    t4 = time.perf_counter()
    assert rc >= 0, rc
    npk = a.sessions * a.packets
    by = npk * a.size
    ok = sink.sink_ndeliv() == npk and sink.sink_dbytes() == by and sink.sink_dsum() == expect_sum % 2**64
    z.close()
    return {"sessions": a.sessions, "packets_per_session": a.packets, "payload_bytes": a.size, "k": a.k, "n": a.n,
            "loss": a.loss, "dropped_per_group": nlost, "sorted": bool(a.sorted), "datagrams": int(cnt),
            "queue_tx_s": round(t1 - t0, 4), "send_flush_s": round(t2 - t1, 4),
            "send_gibs": round(by / (t2 - t1) / 2**30, 3), "send_mpkts": round(npk / (t2 - t1) / 1e6, 3),
            "queue_rx_s": round(t3 - t2, 4), "recv_flush_s": round(t4 - t3, 4),
            "recv_gibs": round(by / (t4 - t3) / 2**30, 3), "recv_mpkts": round(npk / (t4 - t3) / 1e6, 3),
            "delivered": int(sink.sink_ndeliv()), "verified": bool(ok)}


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
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    sink = load_sink()
    r = random.Random(1)
    pay = []
    for _ in range(257):
        b = r.randbytes(a.size)
        pay.append((b, int(sink.sink_fold(b, len(b)))))
    best = None
    for rep in range(a.reps):
        res = run(a, sink, rep, pay)
        if not a.json:
            print(f"rep {rep}: {a.sessions} sessions x {a.packets} x {a.size} B, RS({a.k},{a.n}), loss {a.loss} "
                  f"({res['dropped_per_group']} of {a.n} per group): queue {res['queue_tx_s']:.3f}s, send flush "
                  f"{res['send_flush_s']:.4f}s ({res['send_gibs']:.2f} GiB/s, {res['send_mpkts']:.2f} Mpkt/s), "
                  f"queue rx {res['queue_rx_s']:.3f}s, receive flush {res['recv_flush_s']:.4f}s "
                  f"({res['recv_gibs']:.2f} GiB/s, {res['recv_mpkts']:.2f} Mpkt/s), delivered {res['delivered']} "
                  f"verified={res['verified']}", flush=True)
        if best is None or res["send_gibs"] + res["recv_gibs"] > best["send_gibs"] + best["recv_gibs"]:
            best = res
    if a.json:
        print(json.dumps(best), flush=True)


if __name__ == "__main__":
    main()
