"""module/rs.h on arrays of caller shard pointers (reed_solomon_encode / reed_solomon_reconstruct,
module/rs.c:574-643) through libqfec.so: the pipelined host path over many chunks, arrays that mix
host and device shards, and shards scattered in memory -- all against the CPU oracle, return code
for return code (unrecoverable groups included).
"""
import ctypes as C

import numpy as np
import pytest

import quicknet_amd as qa
from quicknet_amd.synth import erasure_marks, marks_to_rs_layout, synth_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")


@pytest.fixture
def knobs():
    """Set knobs for one test and put back what was there before (qfec_tune_get)."""
    saved = {}

    def set_(key, value):
        if key not in saved:
            saved[key] = qa.tune_get(key)
        qa.tune(key, value)

    yield set_
    for key, value in saved.items():
        qa.tune(key, value)


def scattered_rows(G, n, B, seed):
    """G * n separately allocated host rows of B bytes (not one contiguous batch), in a random order
    in memory; returns (rows, keepalive)."""
    rng = np.random.default_rng(seed)
    pool = np.zeros((G * n + 8, B + 24), np.uint8)
    order = rng.permutation(G * n)
    rows = [pool[order[i], 8 + (i % 3) * 8:8 + (i % 3) * 8 + B] for i in range(G * n)]
    return rows, pool


def ptr_array(rows):
    return (C.c_void_p * len(rows))(*[r.ctypes.data if isinstance(r, np.ndarray) else r.data_ptr() for r in rows])


def mixed_marks(G, k, m, seed):
    """Per group 0..m+1 erasures: some groups lose nothing, some more than the parity can cover."""
    rng = np.random.default_rng(seed)
    gm = np.zeros((G, k + m), np.uint8)
    for g in range(G):
        e = int(rng.integers(0, m + 2))
        gm[g, rng.choice(k + m, e, replace=False)] = 1
    gm[0, :] = 0  # nothing erased
    gm[1, :m + 1] = 1  # m + 1 data rows erased: unrecoverable
    return gm


@pytest.mark.parametrize("k,m,B", [(10, 3, 1000), (4, 2, 1024), (16, 4, 1400)])
@pytest.mark.parametrize("chunk,threads,lanes", [(7, 4, 2), (0, 0, 4), (1, 1, 8)])
def test_rs_host_encode_pipeline_vs_oracle(oracle, knobs, k, m, B, chunk, threads, lanes):
    """reed_solomon_encode on host pointers: many pipelined chunks (host_chunk groups each, two slots
    alternating), 1 to 4 copy threads; shard rows scattered in memory.  The encode leg always stages
    each chunk through the slot's device buffer (reading the pinned slot in place over PCIe measured
    slower, profiles/r05af), so host_zero_copy does not apply to it and is not varied here.  2, 4 or 8
    chunks in flight (host_lanes)."""
    knobs("host_lanes", lanes)
    knobs("host_chunk", chunk)
    knobs("host_threads", threads)
    G, n = 61, k + m
    rows, _keep = scattered_rows(G, n, B, 5)
    data0 = synth_bytes(0xA11CE + k, G * k * B).reshape(G, k, B)
    for i in range(G * k):
        rows[i][:] = data0.reshape(G * k, B)[i]
    for i in range(G * k, G * n):
        rows[i][:] = 0x33
    rs = qa.ReedSolomon(k, m)
    assert qa.lib().reed_solomon_encode(rs._h, ptr_array(rows), G * n, B) == 0
    want = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(oracle.cauchy(k, m), data0, want, B)
    assert np.array_equal(np.stack(rows[G * k:]).reshape(G, m, B), want)
    rs.close()


@pytest.mark.parametrize("k,m,B", [(10, 3, 1000), (4, 2, 1024), (16, 4, 1400)])
@pytest.mark.parametrize("zero_copy", [1, 0])
@pytest.mark.parametrize("chunk,threads,lanes", [(7, 4, 8), (0, 0, 4), (1, 1, 2)])
def test_rs_host_reconstruct_pipeline_vs_oracle(oracle, knobs, k, m, B, zero_copy, chunk, threads, lanes):
    """reed_solomon_reconstruct on host pointers: many pipelined chunks, 1 to 4 copy threads, the
    kernel reading the survivors and writing the erased rows in the pinned slot in place (zero copy)
    or through the slot's device buffer; inconsistent parity (pins the survivor rule byte for byte),
    erased rows pre-filled with 0x5A, unrecoverable groups; 2, 4 or 8 chunks in flight."""
    knobs("host_lanes", lanes)
    knobs("host_zero_copy", zero_copy)
    knobs("host_chunk", chunk)
    knobs("host_threads", threads)
    G, n = 61, k + m
    rows, _keep = scattered_rows(G, n, B, 5)
    data0 = synth_bytes(0xA11CE + k, G * k * B).reshape(G, k, B)
    rs = qa.ReedSolomon(k, m)
    L = qa.lib()
    ptrs = ptr_array(rows)
    par = synth_bytes(0xBEEF + k, G * m * B).reshape(G, m, B)
    gm = mixed_marks(G, k, m, 11 + k)
    marks = marks_to_rs_layout(gm, k)
    d = data0.copy()
    d.reshape(G * k, B)[marks[:G * k] == 1] = 0x5A
    for i in range(G * k):
        rows[i][:] = d.reshape(G * k, B)[i]
    for i in range(G * m):
        rows[G * k + i][:] = par.reshape(G * m, B)[i]
    rc = L.reed_solomon_reconstruct(rs._h, ptrs, C.c_void_p(marks.ctypes.data), G * n, B)
    exp = d.copy()
    rc_o = oracle.rs_reconstruct(oracle.cauchy(k, m), exp, par.copy(), marks, B)
    assert rc == rc_o == -1
    assert np.array_equal(np.stack(rows[:G * k]).reshape(G, k, B), exp)
    assert np.array_equal(np.stack(rows[G * k:]).reshape(G, m, B), par)  # parity never written
    rs.close()


@pytest.mark.parametrize("B", [40, 1000, 1400])
@pytest.mark.parametrize("layout", ["contiguous", "scattered"])
@pytest.mark.parametrize("nt", [0, 1, 2])
def test_rs_host_streaming_rows_vs_oracle(oracle, knobs, B, layout, nt):
    """The slot gathers with streaming stores (host_nt 1: every row; 2, the default: rows that start
    where the previous row of the run ended; 0: none), over rows that follow one another in memory
    (data and parity each one batch at pitch B, so mode 2 streams them) and rows scattered at
    misaligned places; B = 40 takes the short-row copy, 1000 a tail after the 64-B steps.  Encode,
    then reconstruct, both equal to the oracle."""
    knobs("host_nt", nt)
    knobs("host_chunk", 13)
    k, m, G = 10, 3, 97
    n = k + m
    if layout == "contiguous":
        dbuf = np.zeros((G * k, B), np.uint8)
        pbuf = np.zeros((G * m, B), np.uint8)
        rows = list(dbuf) + list(pbuf)
    else:
        rows, _keep = scattered_rows(G, n, B, 9)
    data0 = synth_bytes(0x57EA + B, G * k * B).reshape(G, k, B)
    for i in range(G * k):
        rows[i][:] = data0.reshape(G * k, B)[i]
    ptrs = ptr_array(rows)
    rs = qa.ReedSolomon(k, m)
    L = qa.lib()
    assert L.reed_solomon_encode(rs._h, ptrs, G * n, B) == 0
    par = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(oracle.cauchy(k, m), data0, par, B)
    assert np.array_equal(np.stack(rows[G * k:]).reshape(G, m, B), par)
    gm = mixed_marks(G, k, m, 23)
    marks = marks_to_rs_layout(gm, k)
    d = data0.copy()
    d.reshape(G * k, B)[marks[:G * k] == 1] = 0x5A
    for i in range(G * k):
        rows[i][:] = d.reshape(G * k, B)[i]
    rc = L.reed_solomon_reconstruct(rs._h, ptrs, C.c_void_p(marks.ctypes.data), G * n, B)
    exp = d.copy()
    rc_o = oracle.rs_reconstruct(oracle.cauchy(k, m), exp, par.copy(), marks, B)
    assert rc == rc_o == -1
    assert np.array_equal(np.stack(rows[:G * k]).reshape(G, k, B), exp)
    rs.close()


@pytest.mark.parametrize("layout", ["host", "mixed"])
def test_rs_wide_code_host_pointers(oracle, capfd, monkeypatch, layout):
    """n = k + m > 24 (no pattern LUT: per-chunk decode records) on host shard pointers.
    Host rows go through the pinned stage with one DMA per chunk, device rows one copy each; both
    calls equal the oracle, return code included, and the reconstruct of 3 000 RS(20,10) groups
    (90 000 pointers) finishes in well under a second (it had taken one pageable copy per row)."""
    import time
    k, m, B, G = 20, 10, 1024, 3000
    n = k + m
    rows, _keep = scattered_rows(G, n, B, 21)
    dev = []
    if layout == "mixed":  # every 7th row in device memory
        for i in range(0, G * n, 7):
            t = torch.zeros(B, dtype=torch.uint8, device=DEV)
            dev.append(t)
            rows[i] = t
    data0 = synth_bytes(0x20 + len(dev), G * k * B).reshape(G, k, B)

    def put(i, a):
        if isinstance(rows[i], np.ndarray):
            rows[i][:] = a
        else:
            rows[i].copy_(torch.from_numpy(np.ascontiguousarray(a)).to(DEV))

    def get_all(lo, hi):
        return np.stack([rows[i].copy() if isinstance(rows[i], np.ndarray) else rows[i].cpu().numpy()
                         for i in range(lo, hi)])
    for i in range(G * k):
        put(i, data0.reshape(G * k, B)[i])
    torch.cuda.synchronize()
    rs = qa.ReedSolomon(k, m)
    L = qa.lib()
    ptrs = ptr_array(rows)
    assert L.reed_solomon_encode(rs._h, ptrs, G * n, B) == 0
    want = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(oracle.cauchy(k, m), data0, want, B)
    assert np.array_equal(get_all(G * k, G * n).reshape(G, m, B), want)
    gm = mixed_marks(G, k, m, 31)
    marks = marks_to_rs_layout(gm, k)
    d = data0.copy()
    d.reshape(G * k, B)[marks[:G * k] == 1] = 0x5A
    for i in range(G * k):
        put(i, d.reshape(G * k, B)[i])
    torch.cuda.synchronize()
    monkeypatch.setenv("QFEC_RS_TRACE", "1")
    t0 = time.perf_counter()
    rc = L.reed_solomon_reconstruct(rs._h, ptrs, C.c_void_p(marks.ctypes.data), G * n, B)
    el = time.perf_counter() - t0
    monkeypatch.delenv("QFEC_RS_TRACE")
    exp = d.copy()
    rc_o = oracle.rs_reconstruct(oracle.cauchy(k, m), exp, want.copy(), marks, B)
    assert rc == rc_o == -1
    assert np.array_equal(get_all(0, G * k).reshape(G, k, B), exp)
    print(capfd.readouterr().err)
    if layout == "host":
        assert el < 1.0, el
    rs.close()


def test_rs_many_device_allocations_classify_fast(oracle, capfd, monkeypatch):
    """every device row in its own hipMalloc (40 000 allocations): the classifier keeps
    the allocation ranges ordered (binary search), so classifying the array costs milliseconds, not
    a scan of every range per pointer (QFEC_RS_TRACE reports the classify time); the encode equals
    the oracle's."""
    import re
    hip = C.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipFree.argtypes = [C.c_void_p]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    k, m, B = 10, 3, 512
    G = 40000 // (k + m)
    n = k + m
    ptrs = []
    try:
        for _ in range(G * n):
            p = C.c_void_p()
            assert hip.hipMalloc(C.byref(p), 65536) == 0
            ptrs.append(p.value)
        data0 = synth_bytes(0x77, G * k * B).reshape(G, k, B)
        flat = np.ascontiguousarray(data0.reshape(G * k, B))
        for i in range(G * k):
            assert hip.hipMemcpy(ptrs[i], flat[i].ctypes.data, B, 1) == 0  # hipMemcpyHostToDevice
        rs = qa.ReedSolomon(k, m)
        arr = (C.c_void_p * len(ptrs))(*ptrs)
        monkeypatch.setenv("QFEC_RS_TRACE", "1")
        assert qa.lib().reed_solomon_encode(rs._h, arr, G * n, B) == 0
        monkeypatch.delenv("QFEC_RS_TRACE")
        err = capfd.readouterr().err
        cls = re.search(r"reed_solomon_encode \(staged\).*classify ([0-9.]+) ms", err)
        assert cls, err[-2000:]
        assert float(cls.group(1)) < 500.0, err[-500:]
        got = np.zeros((G * m, B), np.uint8)
        for i in range(G * m):
            assert hip.hipMemcpy(got[i].ctypes.data, ptrs[G * k + i], B, 2) == 0  # hipMemcpyDeviceToHost
        want = np.zeros((G, m, B), np.uint8)
        oracle.rs_encode(oracle.cauchy(k, m), data0, want, B)
        assert np.array_equal(got.reshape(G, m, B), want)
        rs.close()
    finally:
        for p in ptrs:
            hip.hipFree(p)


def test_rs_host_pipeline_recoverable_rc0(oracle, knobs):
    """Every group recoverable -> 0; many chunks."""
    knobs("host_chunk", 5)
    k, m, B, G = 10, 3, 1024, 40
    data0 = synth_bytes(7, G * k * B).reshape(G, k, B)
    par = np.zeros((G, m, B), np.uint8)
    rs = qa.ReedSolomon(k, m)
    assert rs.encode(data0, par, B) == 0
    gm = erasure_marks(9, G, k + m, 3)
    marks = marks_to_rs_layout(gm, k)
    d = data0.copy()
    d.reshape(G * k, B)[marks[:G * k] == 1] = 0
    assert rs.reconstruct(d, par, marks, B) == 0
    assert np.array_equal(d, data0)
    rs.close()


@pytest.mark.parametrize("pattern", ["alternate", "data_dev", "parity_dev", "one_dev"])
def test_rs_mixed_host_device_pointers(oracle, pattern):
    """A pointer array mixing host and device shards (module/rs.h promises either kind per shard):
    every pointer is classified, and the mixed array takes a copy per row of whatever kind."""
    k, m, B, G = 10, 3, 1000, 12
    n = k + m
    data0 = synth_bytes(0x31337, G * k * B).reshape(G, k, B)
    host_rows, _keep = scattered_rows(G, n, B, 3)
    dev_rows = [torch.zeros(B, dtype=torch.uint8, device=DEV) for _ in range(G * n)]

    def on_dev(i):
        if pattern == "alternate":
            return i % 2 == 0
        if pattern == "data_dev":
            return i < G * k
        if pattern == "parity_dev":
            return i >= G * k
        return i == 5

    rows = [dev_rows[i] if on_dev(i) else host_rows[i] for i in range(G * n)]

    def put(i, a):
        if isinstance(rows[i], np.ndarray):
            rows[i][:] = a
        else:
            rows[i].copy_(torch.from_numpy(np.ascontiguousarray(a)).to(DEV))

    def get(i):
        return rows[i].copy() if isinstance(rows[i], np.ndarray) else rows[i].cpu().numpy()

    for i in range(G * k):
        put(i, data0.reshape(G * k, B)[i])
    torch.cuda.synchronize()
    rs = qa.ReedSolomon(k, m)
    L = qa.lib()
    ptrs = ptr_array(rows)
    assert L.reed_solomon_encode(rs._h, ptrs, G * n, B) == 0
    torch.cuda.synchronize()
    want = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(oracle.cauchy(k, m), data0, want, B)
    assert np.array_equal(np.stack([get(G * k + i) for i in range(G * m)]).reshape(G, m, B), want)
    par = synth_bytes(0x5150, G * m * B).reshape(G, m, B)
    gm = mixed_marks(G, k, m, 4)
    marks = marks_to_rs_layout(gm, k)
    d = data0.copy()
    d.reshape(G * k, B)[marks[:G * k] == 1] = 0x5A
    for i in range(G * k):
        put(i, d.reshape(G * k, B)[i])
    for i in range(G * m):
        put(G * k + i, par.reshape(G * m, B)[i])
    torch.cuda.synchronize()
    rc = L.reed_solomon_reconstruct(rs._h, ptrs, C.c_void_p(marks.ctypes.data), G * n, B)
    torch.cuda.synchronize()
    exp = d.copy()
    rc_o = oracle.rs_reconstruct(oracle.cauchy(k, m), exp, par.copy(), marks, B)
    assert rc == rc_o
    assert np.array_equal(np.stack([get(i) for i in range(G * k)]).reshape(G, k, B), exp)
    rs.close()


def test_rs_host_while_tuning(oracle):
    """Encodes and reconstructs on host pointers from two threads while a third flips the host
    knobs (chunking, copy threads, zero copy, lanes, streaming stores): every result still equals the oracle's."""
    import threading
    keys = ("host_chunk", "host_threads", "host_zero_copy", "host_lanes", "host_nt")
    before = {k: qa.tune_get(k) for k in keys}
    stop = threading.Event()
    errors = []

    def tuner():
        i = 0
        while not stop.is_set():
            qa.tune("host_chunk", (0, 3, 17)[i % 3])
            qa.tune("host_threads", (0, 1, 3)[i % 3])
            qa.tune("host_zero_copy", i & 1)
            qa.tune("host_lanes", (2, 4, 8)[i % 3])
            qa.tune("host_nt", (2, 0, 1, 2)[i % 4])
            i += 1

    def coder(seed):
        k, m, B, G = 10, 3, 512, 23
        rs = qa.ReedSolomon(k, m)
        want_p = None
        for it in range(6):
            data0 = synth_bytes(seed * 100 + it, G * k * B).reshape(G, k, B)
            par = np.zeros((G, m, B), np.uint8)
            if rs.encode(data0, par, B) != 0:
                errors.append("encode rc")
            want_p = np.zeros((G, m, B), np.uint8)
            oracle.rs_encode(oracle.cauchy(k, m), data0, want_p, B)
            if not np.array_equal(par, want_p):
                errors.append(("encode", seed, it))
            marks = marks_to_rs_layout(erasure_marks(seed + it, G, k + m, 3), k)
            d = data0.copy()
            d.reshape(G * k, B)[marks[:G * k] == 1] = 0
            if rs.reconstruct(d, par, marks, B) != 0 or not np.array_equal(d, data0):
                errors.append(("reconstruct", seed, it))
        rs.close()

    t = threading.Thread(target=tuner)
    coders = [threading.Thread(target=coder, args=(s,)) for s in (1, 2)]
    t.start()
    for c in coders:
        c.start()
    for c in coders:
        c.join()
    stop.set()
    t.join()
    for k, v in before.items():
        qa.tune(k, v)
    assert not errors, errors[:5]


@pytest.mark.parametrize("G", [9, 330])
@pytest.mark.parametrize("kind", ["pinned", "shm", "file", "pinned_dev_mix"])
def test_rs_host_memory_kinds(oracle, tmp_path, kind, G):
    """Shards in the other kinds of system memory the pointer classifier meets (pinned host
    tensors, /dev/shm and regular-file mappings), alone and mixed with device rows: encode and
    reconstruct equal the oracle's.  9 groups (117 pointers) are classified by runtime probes,
    330 groups (4 290 pointers, past kMapsMinPointers) by the process's mappings."""
    import mmap
    k, m, B = 10, 3, 1000
    n = k + m
    nbytes = G * n * B
    keep = []
    if kind in ("pinned", "pinned_dev_mix"):
        t = torch.zeros(nbytes, dtype=torch.uint8).pin_memory()
        keep.append(t)
        base = t.numpy()
    else:
        path = f"/dev/shm/qfec_test_{__import__('os').getpid()}" if kind == "shm" else str(tmp_path / "rows.bin")
        with open(path, "wb") as f:
            f.write(b"\0" * nbytes)
        f = open(path, "r+b")
        mm = mmap.mmap(f.fileno(), nbytes)
        keep += [f, mm]
        base = np.frombuffer(mm, dtype=np.uint8)
        if kind == "shm":
            __import__("os").unlink(path)
    rows = [base[i * B:(i + 1) * B] for i in range(G * n)]
    if kind == "pinned_dev_mix":
        rows = [torch.zeros(B, dtype=torch.uint8, device=DEV) if i % 5 == 1 else r for i, r in enumerate(rows)]

    def put(i, a):
        if isinstance(rows[i], np.ndarray):
            rows[i][:] = a
        else:
            rows[i].copy_(torch.from_numpy(np.ascontiguousarray(a)).to(DEV))

    def get(i):
        return rows[i].copy() if isinstance(rows[i], np.ndarray) else rows[i].cpu().numpy()

    data0 = synth_bytes(0xC0DE, G * k * B).reshape(G, k, B)
    for i in range(G * k):
        put(i, data0.reshape(G * k, B)[i])
    torch.cuda.synchronize()
    rs = qa.ReedSolomon(k, m)
    L = qa.lib()
    ptrs = ptr_array(rows)
    assert L.reed_solomon_encode(rs._h, ptrs, G * n, B) == 0
    torch.cuda.synchronize()
    want = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(oracle.cauchy(k, m), data0, want, B)
    assert np.array_equal(np.stack([get(G * k + i) for i in range(G * m)]).reshape(G, m, B), want)
    gm = mixed_marks(G, k, m, 21)
    marks = marks_to_rs_layout(gm, k)
    d = data0.copy()
    d.reshape(G * k, B)[marks[:G * k] == 1] = 0x5A
    for i in range(G * k):
        put(i, d.reshape(G * k, B)[i])
    torch.cuda.synchronize()
    rc = L.reed_solomon_reconstruct(rs._h, ptrs, C.c_void_p(marks.ctypes.data), G * n, B)
    torch.cuda.synchronize()
    exp = d.copy()
    rc_o = oracle.rs_reconstruct(oracle.cauchy(k, m), exp, want.copy(), marks, B)
    assert rc == rc_o == -1
    assert np.array_equal(np.stack([get(i) for i in range(G * k)]).reshape(G, k, B), exp)
    rs.close()
    del rows, base


@pytest.mark.parametrize("zero_copy", [1, 0])
def test_rs_host_pipeline_quirk_edits(oracle, knobs, zero_copy):
    """Edited public matrices through the pipelined host path over many chunks: a zero
    coefficient in column 0 of `rs->parity` leaves that parity row's old bytes in place
    (rs.c:116-117: the pipeline then stages the parity rows too), and `rs->m` edited so the
    reconstruct decodes with the edited rows (rs.c:505, 536-556) -- both against the oracle."""
    knobs("host_zero_copy", zero_copy)
    knobs("host_chunk", 4)
    k, m, B, G = 10, 3, 600, 23
    rs = qa.ReedSolomon(k, m)
    rows = rs.parity.copy()
    rows[1, 0] = 0  # parity row 1 keeps its old bytes where column 0 contributes
    rs.parity[:] = rows
    data0 = synth_bytes(0xED17, G * k * B).reshape(G, k, B)
    par0 = synth_bytes(0x0DD, G * m * B).reshape(G, m, B)  # stale parity the quirk keeps
    par = par0.copy()
    assert rs.encode(data0, par, B) == 0
    want = par0.copy()
    oracle.rs_encode(rows, data0, want, B)
    assert np.array_equal(par, want)
    full = rs.m_matrix.copy()
    full[k + 2, 3] ^= 0x21  # a parity row of the decode matrix edited (the reconstruct reads rs->m)
    rs.m_matrix[:] = full
    gm = mixed_marks(G, k, m, 77)
    marks = marks_to_rs_layout(gm, k)
    d = data0.copy()
    d.reshape(G * k, B)[marks[:G * k] == 1] = 0x5A
    exp = d.copy()
    rc_o = oracle.rs_reconstruct_full(full, exp, want.copy(), marks, B)
    rc = rs.reconstruct(d, want.copy(), marks, B)
    assert rc == rc_o
    assert np.array_equal(d, exp)
    rs.close()


def _ref_codec():
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle.oracle import RefCodec
    if not RefCodec.available():
        pytest.skip("reference libraries not built (make -C oracle ref)")
    return RefCodec()


@pytest.fixture
def devlist():
    """Set qfec_rs_host_devices for one test, back to the current device afterwards."""
    yield qa.rs_host_devices
    qa.rs_host_devices(None)


@pytest.mark.parametrize("devices", [None, [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("k,m,B,G,edit", [(10, 3, 1000, 61, False), (10, 3, 1024, 40, True), (16, 4, 1400, 37, True),
                                          (4, 2, 37, 200, True), (20, 5, 256, 50, False), (3, 2, 33, 90, True)])
def test_rs_host_pipeline_vs_reference_rs(knobs, devlist, k, m, B, G, edit, devices):
    """The pipelined host path against the reference's own module/rs.c (oracle/_ref, compiled from
    /root/reference) on identical scattered rows: the same public-matrix edits on both handles
    (a zero column-0 coefficient, an edited row of rs->m), encode, then reconstruct with 0..m+1
    erasures per group (unrecoverable groups included) -- bytes and return codes equal.  Chunks on
    the current device's two slots, or spread over qfec_rs_host_devices' lanes (device 0 listed two
    or three times: four or six chunks in flight, the multi-GPU path's control flow on one GPU)."""
    ref = _ref_codec()
    knobs("host_chunk", 9)
    assert devlist(devices) == (devices or [])
    n = k + m
    rng = np.random.default_rng(k * 1000 + B)
    rows, _keep = scattered_rows(G, n, B, k + B)
    rrows, _rkeep = scattered_rows(G, n, B, k + B + 1)
    data0 = synth_bytes(0xC0FFEE + k + B, G * k * B).reshape(G * k, B)
    par0 = synth_bytes(0xFACADE + m + B, G * m * B).reshape(G * m, B)
    for i in range(G * k):
        rows[i][:] = data0[i]
        rrows[i][:] = data0[i]
    for i in range(G * m):
        rows[G * k + i][:] = par0[i]
        rrows[G * k + i][:] = par0[i]
    rs = qa.ReedSolomon(k, m)
    h = ref.rs.reed_solomon_new(k, m)
    try:
        if edit:
            par_ref = np.ctypeslib.as_array(h.contents.parity, shape=(m, k))
            m_ref = np.ctypeslib.as_array(h.contents.m, shape=(n, k))
            r = int(rng.integers(0, m))
            rs.parity[r, 0] = 0
            par_ref[r, 0] = 0
            j, c, v = int(rng.integers(0, n)), int(rng.integers(0, k)), int(rng.integers(1, 256))
            rs.m_matrix[j, c] ^= v
            m_ref[j, c] ^= v
        L = qa.lib()
        ptrs, rptrs = ptr_array(rows), ptr_array(rrows)
        assert L.reed_solomon_encode(rs._h, ptrs, G * n, B) == ref.rs_encode(h, rptrs, G * n, B) == 0
        assert all(np.array_equal(rows[i], rrows[i]) for i in range(G * n))
        gm = mixed_marks(G, k, m, k + m + B)
        marks = marks_to_rs_layout(gm, k)
        for i in range(G * k):
            if marks[i]:
                rows[i][:] = 0x5A
                rrows[i][:] = 0x5A
        rc = L.reed_solomon_reconstruct(rs._h, ptrs, C.c_void_p(marks.ctypes.data), G * n, B)
        rc_ref = ref.rs_reconstruct(h, rptrs, marks, G * n, B)
        assert rc == rc_ref == -1
        bad = [i for i in range(G * n) if not np.array_equal(rows[i], rrows[i])]
        assert not bad, bad[:10]
    finally:
        ref.rs.reed_solomon_release(h)
        rs.close()
