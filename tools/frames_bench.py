#!/usr/bin/env python3
"""Payloads -> ProtocolUdp frames and back on the bench's batch, one pass against two:
RS(10,13) (fec_new matrix) x 100 000 groups of 10 x 1 KiB payloads, checksums on, 3 of 13
frames lost per group, no Session prefix (--session: the 12-byte prefix).

  send   two-pass: qfec_pack_datagrams (1088-B wire pitch) + qfec_frame_udp (1088-B frames)
         one pass: qfec_pack_frames
  recv   two-pass: qfec_unframe_udp + qfec_unpack_datagrams (+ the status fix-up launch)
         one pass: qfec_unpack_frames
Every launch goes through the C ABI on preallocated buffers (what bench.py's wire_framed leg
does).  Minimal traffic: payload in + frames out (send); frames received in + data shard rows
out (receive).  Verified: the one-pass frames equal the two-pass ones, every payload comes back.

  python tools/frames_bench.py [--groups N --rounds R --reps K --session]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import quicknet_amd as qa  # noqa: E402
from quicknet_amd.synth import erasure_marks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--session", action="store_true")
    ap.add_argument("--payload", type=int, default=1024)
    ap.add_argument("--tune", default="", help="qfec_tune settings, e.g. wire_rx=3")
    a = ap.parse_args()
    for kv in filter(None, a.tune.split(",")):
        kk, vv = kv.split("=")
        qa.tune(kk, int(vv))
    k, n, S, G = 10, 13, a.payload, a.groups
    m = n - k
    P = 12 if a.session else 4
    dev = torch.device("cuda:0")
    code = qa.Code.vandermonde(k, m)
    L = qa.lib()
    sp = (S + 4 + 15) // 16 * 16
    wp = (sp + 13 + 63) // 64 * 64
    fpitch = (sp + 13 + P + 63) // 64 * 64
    payload = torch.empty(G * k * S + 16, dtype=torch.uint8, device=dev)
    qa.synth_fill(payload, 0x77)
    offs = torch.arange(G * k, dtype=torch.int64, device=dev) * S
    sizes = torch.full((G * k,), S, dtype=torch.int32, device=dev)
    seq = torch.stack([torch.arange(G, dtype=torch.int32, device=dev) * n,
                       torch.arange(G, dtype=torch.int32, device=dev) * k], 1).contiguous()
    masks = (torch.arange(G * n, device=dev) * 7 & 0xFF).to(torch.uint8)
    ch = torch.randint(0, 2**31, (G * n, 2), dtype=torch.int32, device=dev) if a.session else None
    chp = ch.data_ptr() if ch is not None else None
    lost = torch.from_numpy(erasure_marks(0x5EED0077, G, n, m).astype(bool)).to(dev)
    shards = torch.empty((G, n, sp), dtype=torch.uint8, device=dev)
    wire = torch.empty((G, n, wp), dtype=torch.uint8, device=dev)
    wlen = torch.empty((G, n), dtype=torch.int32, device=dev)
    fr2 = torch.empty((G, n, fpitch), dtype=torch.uint8, device=dev)
    fl2 = torch.empty((G, n), dtype=torch.int32, device=dev)
    fr1 = torch.empty((G, n, fpitch), dtype=torch.uint8, device=dev)
    fl1 = torch.empty((G, n), dtype=torch.int32, device=dev)
    dgr = torch.empty((G, n, fpitch), dtype=torch.uint8, device=dev)
    dlen = torch.empty((G, n), dtype=torch.int32, device=dev)
    fst = torch.empty((G, n), dtype=torch.int32, device=dev)
    osh = torch.empty((G, n, sp), dtype=torch.uint8, device=dev)
    marks = torch.empty(G * n, dtype=torch.uint8, device=dev)
    rxs = torch.empty((G, n), dtype=torch.int32, device=dev)
    status = torch.empty((G, k), dtype=torch.int32, device=dev)
    psize = torch.empty((G, k), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def ok(rc):
        assert rc == 0, (rc, L.qfec_last_error())

    def send2():
        ok(L.qfec_pack_datagrams(code._h, payload.data_ptr(), offs.data_ptr(), sizes.data_ptr(), seq.data_ptr(), G, 1,
                                 shards.data_ptr(), sp, wire.data_ptr(), wp, wlen.data_ptr(), st))
        ok(L.qfec_frame_udp(wire.data_ptr(), wp, wlen.data_ptr(), G * n, masks.data_ptr(), chp, 0x3C, 0x11, 0xFF,
                            fr2.data_ptr(), fpitch, fl2.data_ptr(), st))

    def send1():
        ok(L.qfec_pack_frames(code._h, payload.data_ptr(), offs.data_ptr(), sizes.data_ptr(), seq.data_ptr(), G, 1,
                              shards.data_ptr(), sp, masks.data_ptr(), chp, 0x3C, 0x11, 0xFF, fr1.data_ptr(), fpitch,
                              fl1.data_ptr(), st))

    send1()
    send2()
    torch.cuda.synchronize()
    same = torch.equal(fl1, fl2) and torch.equal(fr1, fr2)
    rx_len = torch.where(lost, torch.zeros_like(fl1), fl1).contiguous()

    def recv2():
        ok(L.qfec_unframe_udp(fr1.data_ptr(), fpitch, rx_len.data_ptr(), G * n, 0x3C, int(a.session), dgr.data_ptr(),
                              fpitch, dlen.data_ptr(), fst.data_ptr(), None, None, st))
        qa.lib().qfec_tune(b"wire_rx", 1)
        ok(L.qfec_unpack_datagrams(code._h, dgr.data_ptr(), fpitch, dlen.data_ptr(), G, 1, 2068, osh.data_ptr(), sp,
                                   marks.data_ptr(), rxs.data_ptr(), status.data_ptr(), psize.data_ptr(), st))

    def recv1():
        ok(L.qfec_unpack_frames(code._h, fr1.data_ptr(), fpitch, rx_len.data_ptr(), G, 0x3C, int(a.session), 1, 2068,
                                osh.data_ptr(), sp, marks.data_ptr(), rxs.data_ptr(), status.data_ptr(),
                                psize.data_ptr(), fst.data_ptr(), None, st))

    recv1()
    torch.cuda.synchronize()
    good = bool((status == 4).all()) and torch.equal(osh[:, :k, 4:4 + S].reshape(-1), payload[:G * k * S])
    good = good and bool((fst[~lost] == 0).all())
    print(f"one-pass frames == two-pass frames: {same}; every payload back through unpack_frames: {good}", flush=True)
    s = torch.cuda.current_stream()
    fns = {"send_two_pass": send2, "send_one_pass": send1, "recv_two_pass": recv2, "recv_one_pass": recv1}
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
    pay = G * k * S
    send_bytes = pay + int(fl1.sum())
    recv_bytes = int(rx_len.sum()) + G * k * sp
    for name in fns:
        ms = statistics.median(t[name])
        nb = send_bytes if name.startswith("send") else recv_bytes
        print(f"{name:14s} {G} groups x {k} x {S} B{' +session' if a.session else ''}: {ms * 1e3:8.1f} us  "
              f"{pay / ms / 1e6 / 1.073741824:7.1f} GiB/s of payload  {nb / ms / 1e6:7.1f} GB/s min traffic "
              f"({nb / ms / 1e6 / 8000:.3f} of 8 TB/s)", flush=True)


if __name__ == "__main__":
    main()
