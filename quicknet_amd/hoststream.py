"""Host-to-host legs of bench.py: the FEC path starts and ends in host memory (the UDP socket /
PacketBuffer, network/FecCodecBuf.cpp), so BASELINE configs[4] is measured host -> device ->
host through the product's streaming engine (include/qfec.h qfec_pipe).

host_mixed_leg   configs[4]: (4,2), (10,3) and (16,4 @ 1400 B) batches of ~64 MiB of data
                 each, interleaved, encode AND reconstruct (m random erasures of n per
                 group), every batch in its own pinned host buffers, 3 HIP streams per GPU.
                 Runs on every rank (one GPU each) between barriers; value = all ranks' data
                 bytes / the slowest rank's time.  Verified byte for byte afterwards.
host_encode_leg  the single-shape host-inclusive encode (qfec_encode_host) of the headline
                 batch, rank 0.
Pinned batches take the zero-copy paths (the kernels read and write host memory directly);
host_mixed_leg(zero_copy=False) measures the staged H2D -> kernel -> D2H pipeline instead.

Everything here is measurement plumbing around the C ABI; the arithmetic is libqfec's.
"""
import time

import torch

from .codec import Code, Pipe, QfecError, synth_fill, tune
from .sharding import rank_seed
from .synth import SEED_DECODE, SEED_ENCODE, erasure_marks, marks_to_rs_layout

GIB = float(1 << 30)
MIXED = ((4, 2, 1024), (10, 3, 1024), (16, 4, 1400))


def _round16(x):
    return (x + 15) // 16 * 16


def make_mixed_batches(rank, dev, batch_bytes=64 << 20, per_shape=2, shapes=MIXED):
    """Pinned host batches: tx (data -> parity to compute) and rx (damaged data + parity +
    marks -> data to restore) per (shape, rep); parity and payload made on the device."""
    batches = []
    for rep in range(per_shape):
        for k, m, B in shapes:
            n, pitch = k + m, _round16(B)
            G = max(1, batch_bytes // (k * pitch))
            code = Code.cauchy(k, m)
            tag = (k << 8 | m) ^ (rep << 16)
            d = torch.empty((G, k, pitch), dtype=torch.uint8, device=dev)
            synth_fill(d, rank_seed(SEED_ENCODE ^ tag, rank))
            p = torch.empty((G, m, pitch), dtype=torch.uint8, device=dev)
            code.encode(d, p, B)
            code.prepare_reconstruct()
            gm = erasure_marks(rank_seed(SEED_DECODE ^ tag, rank), G, n, m)
            lost = torch.from_numpy(gm[:, :k].astype(bool))
            b = {"code": code, "k": k, "m": m, "B": B, "G": G,
                 "tx_data": torch.empty((G, k, pitch), dtype=torch.uint8, pin_memory=True),
                 "tx_par": torch.empty((G, m, pitch), dtype=torch.uint8, pin_memory=True),
                 "rx_data": torch.empty((G, k, pitch), dtype=torch.uint8, pin_memory=True),
                 "rx_par": torch.empty((G, m, pitch), dtype=torch.uint8, pin_memory=True),
                 "rx_marks": torch.from_numpy(marks_to_rs_layout(gm, k)).pin_memory(),
                 "lost": lost, "dec_groups": int(lost.any(1).sum()), "par_ref": p.cpu()}
            b["tx_data"].copy_(d)
            b["rx_data"].copy_(d)
            b["rx_par"].copy_(p)
            del d, p
            batches.append(b)
    torch.cuda.synchronize()
    return batches


def damage(batches):
    """Erase the marked data shards of every rx batch and clear every tx parity (untimed)."""
    for b in batches:
        b["rx_data"][b["lost"]] = 0x5A
        b["tx_par"].zero_()


def run_mixed(pipe, batches):
    """Queue every batch (encode tx, reconstruct rx, interleaved) and wait: one pass."""
    for b in batches:
        pipe.encode(b["code"], b["tx_data"], b["tx_par"], b["B"])
        pipe.reconstruct(b["code"], b["rx_data"], b["rx_par"], b["rx_marks"], b["B"])
    return pipe.wait()


def verify(batches):
    ok = True
    for b in batches:
        B = b["B"]
        ok &= bool(torch.equal(b["tx_par"][..., :B], b["par_ref"][..., :B]))
        ok &= bool(torch.equal(b["rx_data"][..., :B], b["tx_data"][..., :B]))
    return ok


def mixed_units(batches, zero_copy=True):
    """(data bytes, host->device bytes, device->host bytes) of one pass; data counted at B
    (k*B per encoded group and per decoded group), PCIe bytes at pitch.  Zero copy (the
    kernels work in the pinned buffers): encode reads k rows and writes m; reconstruct reads
    the marks, the k survivors of each group with an erased data row, and writes the e erased
    rows.  Staged: every row goes in (data + parity + marks) and all k data rows come back."""
    data = h2d = d2h = 0
    for b in batches:
        k, m, B, G = b["k"], b["m"], b["B"], b["G"]
        pitch = b["tx_data"].shape[2]
        data += G * k * B + b["dec_groups"] * k * B
        if zero_copy:
            h2d += G * k * pitch + b["dec_groups"] * k * pitch + G * (k + m)
            d2h += G * m * pitch + int(b["lost"].sum()) * pitch
        else:
            h2d += G * k * pitch + G * (k + m) * pitch + G * (k + m)
            d2h += G * m * pitch + G * k * pitch
    return data, h2d, d2h


def host_mixed_leg(rank, world, barrier, all_max, all_sum, all_gather, passes=3, streams=3, zero_copy=True,
                   sample_groups=0):
    dev = torch.device("cuda", torch.cuda.current_device())
    tune("host_zero_copy", int(zero_copy))
    try:
        batches = make_mixed_batches(rank, dev)
        pipe = Pipe(devices=[dev.index], streams=streams)
        damage(batches)
        nf = run_mixed(pipe, batches)  # warm-up pass (restores rx, computes tx)
        damage(batches)
        err = None
    except (QfecError, RuntimeError) as exc:  # report, never fake (the collectives below still run)
        err, nf = repr(exc), -1
    barrier(world)
    t0 = time.perf_counter()
    if err is None:
        for _ in range(passes):
            nf += run_mixed(pipe, batches)
    t1 = time.perf_counter()
    barrier(world)
    el = all_max(t1 - t0, world)
    ok = err is None and nf == 0 and verify(batches)
    ok = all_sum(0.0 if ok else 1.0, world) == 0.0
    data, h2d, d2h = mixed_units(batches, zero_copy) if err is None else (0, 0, 0)
    total = all_sum(float(data * passes), world)
    per_rank = all_gather((t1 - t0) * 1e3 / passes, world, rank)
    out = {"value": round(total / el / GIB, 2) if el > 0 else None, "unit": "GiB/s", "verified": ok,
           "verified_against": "the pipe's own device-resident encode (parity) and the undamaged data (restored rows); "
                               "bench.py's cpu_baseline leg re-checks a sample against the reference rs.c at N=1",
           "what": "BASELINE configs[4]: (4,2), (10,3) 1 KiB and (16,4) 1400 B batches of ~64 MiB data, interleaved, "
                   "encode + reconstruct (m random erasures of n per group), pinned host buffers per batch, "
                   f"qfec_pipe with {streams} HIP streams per GPU, "
                   + ("zero copy: the kernels read and write the pinned host buffers over PCIe, only the marks staged"
                      if zero_copy else "staged: H2D -> kernel -> D2H through device buffers"),
           "zero_copy": bool(zero_copy),
           "passes": passes, "ms_per_pass": round(el / passes * 1e3, 3),
           "per_rank_ms_per_pass": [round(x, 3) for x in per_rank],
           "pcie_gbs_per_rank": round((h2d + d2h) * passes / (t1 - t0) / 1e9, 2) if err is None else None,
           "h2d_gbs_per_rank": round(h2d * passes / (t1 - t0) / 1e9, 2) if err is None else None,
           "d2h_gbs_per_rank": round(d2h * passes / (t1 - t0) / 1e9, 2) if err is None else None,
           "batches_per_rank": len(batches) if err is None else 0}
    if err is not None:
        out["error"] = err
    if err is None:
        pipe.close()
        if sample_groups:
            out["_sample"] = sample_batches(batches, sample_groups, rank)
    tune("host_zero_copy", 1)
    del batches
    return out


def sample_batches(batches, per_batch, rank):
    """Copies of `per_batch` seeded random groups of every batch after the timed passes, as
    numpy arrays, for an independent CPU check: the tx data and the parity the pipe wrote,
    and the rx marks (rs.c layout) with the rows the pipe restored."""
    import numpy as np
    rng = np.random.default_rng(0x5A3F1E + rank)
    out = []
    for b in batches:
        k, m, B, G = b["k"], b["m"], b["B"], b["G"]
        idx = np.sort(rng.choice(G, size=min(per_batch, G), replace=False))
        ti = torch.from_numpy(idx)
        gm = b["rx_marks"].numpy()
        dm, pm = gm[:G * k].reshape(G, k), gm[G * k:].reshape(G, m)
        out.append({"k": k, "m": m, "B": B, "idx": idx,
                    "data": b["tx_data"][ti, :, :B].numpy().copy(), "parity": b["tx_par"][ti, :, :B].numpy().copy(),
                    "marks_data": dm[idx].copy(), "marks_parity": pm[idx].copy(),
                    "restored": b["rx_data"][ti, :, :B].numpy().copy()})
    return out


def host_encode_leg(code, data, parity, B):
    """qfec_encode_host over the headline batch from pinned host buffers, best of 3 after one
    warm-up call; parity verified against the device-resident encode."""
    try:
        h_data = data.cpu().pin_memory()
        h_par = torch.empty(parity.shape, dtype=torch.uint8).pin_memory()
        ts = []
        for _ in range(4):
            t = time.perf_counter()
            code.encode_host(h_data, h_par, B)
            ts.append(time.perf_counter() - t)
        G, k = data.shape[0], data.shape[1]
        ok = bool(torch.equal(h_par, parity.cpu()))
        return {"value": round(G * k * B / min(ts[1:]) / GIB, 2), "unit": "GiB/s", "verified": ok,
                "what": "qfec_encode_host, pinned host buffers: zero copy (one launch reads the data and writes the "
                        "parity in host memory over PCIe)"}
    except Exception as exc:  # report, never fake
        return {"value": None, "verified": False, "error": repr(exc)}


def rs_abi_host_leg(G=100_000, k=10, m=3, B=1024, E=3, reps=3, sample_groups=384, seed=0x5EED0005):
    """module/rs.h unchanged on host memory: reed_solomon_encode then reed_solomon_reconstruct
    (E random erasures per group) through libqfec.so on arrays of per-shard pointers into pageable
    numpy buffers (rs.c's own calling convention, module/rs.c:574-643), the config-2 shape.  The
    same metric as cpu_baseline (data GiB/s of encode + decode).  Verified in full afterwards (the
    restored rows equal the originals; the parity equals the device encode's); `_sample` carries
    groups for the cpu_baseline leg's reference rs.c check."""
    import ctypes as C

    import numpy as np

    from .codec import ReedSolomon, lib
    n = k + m
    dev = torch.device("cuda", torch.cuda.current_device())
    d = torch.empty((G, k, B), dtype=torch.uint8, device=dev)
    synth_fill(d, seed)
    p = torch.empty((G, m, B), dtype=torch.uint8, device=dev)
    Code.cauchy(k, m).encode(d, p)
    data0 = d.cpu().numpy()
    par_want = p.cpu().numpy()
    del d, p
    data = data0.copy()                      # pageable, as a socket buffer pool would be
    par = np.zeros((G, m, B), np.uint8)
    ptr = np.concatenate([data.ctypes.data + np.arange(G * k, dtype=np.uint64) * B,
                          par.ctypes.data + np.arange(G * m, dtype=np.uint64) * B]).astype(np.uint64)
    ptrs = (C.c_void_p * (G * n)).from_buffer(ptr)
    gm = erasure_marks(seed ^ 0xD, G, n, E)
    marks = np.ascontiguousarray(marks_to_rs_layout(gm, k))
    lost = gm[:, :k].astype(bool)
    dec_groups = int(lost.any(1).sum())
    rs = ReedSolomon(k, m)
    L = lib()
    enc_s, rec_s = [], []
    rc_enc = rc_rec = 0
    for rep in range(reps + 1):  # the first pass warms the pool, the pinned slots and the tables
        t0 = time.perf_counter()
        rc_enc |= L.reed_solomon_encode(rs._h, ptrs, G * n, B)
        t1 = time.perf_counter()
        data[lost] = 0x5A                    # the erased rows as the receive buffers hold them
        t2 = time.perf_counter()
        rc_rec |= L.reed_solomon_reconstruct(rs._h, ptrs, C.c_void_p(marks.ctypes.data), G * n, B)
        t3 = time.perf_counter()
        if rep:
            enc_s.append(t1 - t0)
            rec_s.append(t3 - t2)
    ok = rc_enc == 0 and rc_rec == 0 and np.array_equal(par, par_want) and np.array_equal(data, data0)
    te, tr = float(np.median(enc_s)), float(np.median(rec_s))
    idx = np.linspace(0, G - 1, sample_groups).astype(np.int64)
    out = {"what": f"reed_solomon_encode + reed_solomon_reconstruct ({E} random erasures/group) on per-shard "
                   f"pointers into pageable host memory, RS({k},{m}) B={B}, {G:,} groups (config 2's shape), "
                   f"median of {reps} passes after one warm pass",
           "value": round((G + dec_groups) * k * B / (te + tr) / GIB, 3), "unit": "GiB/s",
           "encode_gibs": round(G * k * B / te / GIB, 3), "reconstruct_gibs": round(dec_groups * k * B / tr / GIB, 3),
           "encode_ms": round(te * 1e3, 2), "reconstruct_ms": round(tr * 1e3, 2),
           "host_threads": _tune_get("host_threads"), "verified": bool(ok),
           "_sample": {"k": k, "m": m, "B": B, "data": data0[idx].copy(), "par": par[idx].copy(),
                       "marks_gn": gm[idx].copy(), "restored": data[idx].copy()}}
    rs.close()
    del data, par, data0, par_want
    return out


def _tune_get(key):
    from .codec import tune_get
    try:
        return tune_get(key)
    except Exception:  # an older build (QFEC_LIB_COMPAT A/B) without the knob
        return None
