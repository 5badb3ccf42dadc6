#!/usr/bin/env python3
"""Zero-copy probe: the batched kernels launched directly on pinned host memory (the device
address of a hipHostMalloc'd buffer), against the staged paths, for BASELINE configs[4]-shaped
batches.  Checks the outputs equal the device-resident path's and prints host-to-host rates.

  python tools/zerocopy_probe.py [--k 10 --m 3 --block 1024 --groups 60000]
"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import quicknet_amd as qa  # noqa: E402
from quicknet_amd.synth import erasure_marks, marks_to_rs_layout  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]


def devptr(t):
    p = C.c_void_p()
    rc = hip.hipHostGetDevicePointer(C.byref(p), C.c_void_p(t.data_ptr()), 0)
    assert rc == 0, rc
    return p.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--block", type=int, default=1024)
    ap.add_argument("--groups", type=int, default=60000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    k, m, B, G = a.k, a.m, a.block, a.groups
    pitch = (B + 15) // 16 * 16
    dev = torch.device("cuda:0")
    code = qa.Code.cauchy(k, m)
    d = torch.empty((G, k, pitch), dtype=torch.uint8, device=dev)
    qa.synth_fill(d, 1234)
    p = torch.empty((G, m, pitch), dtype=torch.uint8, device=dev)
    code.encode(d, p, B)
    code.prepare_reconstruct()
    gm = erasure_marks(99, G, k + m, m)
    lost = torch.from_numpy(gm[:, :k].astype(bool))
    h_d = d.cpu().pin_memory()
    h_p = torch.zeros((G, m, pitch), dtype=torch.uint8).pin_memory()
    h_rx = d.cpu().pin_memory()
    h_rp = p.cpu().pin_memory()
    h_mk = torch.from_numpy(marks_to_rs_layout(gm, k)).pin_memory()
    print(f"RS({k},{m}) B={B} G={G}: host pointers {h_d.data_ptr():#x} -> device {devptr(h_d):#x}")
    s = torch.cuda.current_stream()
    L = qa.lib()

    def enc_zero():
        rc = L.qfec_encode(code._h, C.c_void_p(devptr(h_d)), C.c_void_p(devptr(h_p)), G, B, pitch,
                           C.c_void_p(s.cuda_stream))
        assert rc == 0, rc

    def rec_zero():
        rc = L.qfec_reconstruct(code._h, C.c_void_p(devptr(h_rx)), C.c_void_p(devptr(h_rp)),
                                C.c_void_p(devptr(h_mk)), G, B, pitch, None, C.c_void_p(s.cuda_stream))
        assert rc == 0, rc

    def enc_staged():
        code.encode_host(h_d, h_p, B)

    data_b = G * k * B
    for name, fn, reset in (("encode zero-copy", enc_zero, lambda: h_p.zero_()),
                            ("encode qfec_encode_host", enc_staged, lambda: h_p.zero_()),
                            ("reconstruct zero-copy", rec_zero, lambda: h_rx.__setitem__(lost, 0x5A))):
        ts = []
        for _ in range(a.reps):
            reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ok = torch.equal(h_p, p.cpu()) if name.startswith("encode") else torch.equal(h_rx, d.cpu())
        print(f"  {name:26s} best {min(ts)*1e3:8.3f} ms -> {data_b / min(ts) / 2**30:7.2f} GiB/s of data  ok={ok}")


if __name__ == "__main__":
    main()
