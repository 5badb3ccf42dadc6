"""GPU: the host-memory paths against the oracle.

* qfec_pipe (BASELINE configs[4]): interleaved (4,2) / (10,3) / (16,4 @ 1400 B) batches,
  encode AND reconstruct, from pinned host buffers over 3 streams per device, and over a
  two-entry device list (the multi-device slot rotation; the box has one GPU, so the list
  names it twice).  Byte-checked against the oracle (module/rs.c restatement, pinned).
* reed_solomon_reconstruct on host pointer arrays spanning several staging chunks.
* The Python face rejects tensors the C ABI would misread (dtype) or cannot reach (host).
* A product multi-rank run: two gloo ranks share cuda:0, each runs libqfec on its
  shard_range slice; the gathered result equals the single-rank oracle output.
"""
import os
import socket

import numpy as np
import pytest

import quicknet_amd as qa
from quicknet_amd.sharding import shard_range
from quicknet_amd.synth import marks_to_rs_layout, synth_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")
MIXED = [(4, 2, 1024, 301), (10, 3, 1024, 257), (16, 4, 1400, 129)]


def round16(x):
    return (x + 15) // 16 * 16


def random_marks(rng, G, k, m, unrecoverable=True):
    gm = np.zeros((G, k + m), np.uint8)
    hi = m + 2 if unrecoverable else m + 1
    for g in range(G):
        gm[g, rng.choice(k + m, size=int(rng.integers(0, hi)), replace=False)] = 1
    return gm


def make_case(oracle, k, m, B, G, seed):
    """Pinned host buffers for one encode batch and one reconstruct batch + oracle answers."""
    pitch = round16(B)
    rng = np.random.default_rng(seed)
    code = qa.Code.cauchy(k, m)
    data = synth_bytes(seed, G * k * B).reshape(G, k, B)
    par_ref = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(code.rows, data, par_ref, B)
    # reconstruct with INCONSISTENT parity: pins the survivor rule byte for byte (rs.c:620-629)
    rx_par = synth_bytes(seed + 1, G * m * B).reshape(G, m, B)
    gm = random_marks(rng, G, k, m)
    marks = marks_to_rs_layout(gm, k)
    damaged = data.copy()
    damaged.reshape(G * k, B)[marks[: G * k] == 1] = 0x5A
    rx_ref = damaged.copy()
    oracle.rs_reconstruct(code.rows, rx_ref, rx_par.copy(), marks, B)
    nfail = int(((gm[:, :k].sum(1) > 0) & (gm.sum(1) > m)).sum())

    def pin(a, pad=0xC3):
        out = np.full(a.shape[:-1] + (pitch,), pad, np.uint8)
        out[..., :B] = a
        return torch.from_numpy(out).pin_memory()

    return {"code": code, "B": B, "tx_data": pin(data), "tx_par": torch.full((G, m, pitch), 0x5A, dtype=torch.uint8)
            .pin_memory(), "par_ref": par_ref, "rx_data": pin(damaged), "rx_par": pin(rx_par),
            "rx_marks": torch.from_numpy(marks).pin_memory(), "rx_ref": rx_ref, "nfail": nfail}


@pytest.mark.parametrize("zero_copy", [1, 0])
@pytest.mark.parametrize("devices,streams,slot", [([0], 3, 1 << 20), ([0, 0], 3, 1 << 20), ([0], 1, 64 << 20),
                                                  (None, 4, 256 << 10)])
def test_pipe_mixed_vs_oracle(oracle, devices, streams, slot, zero_copy):
    """zero_copy 1: each piece's kernel reads and writes the pinned batches in place (only the
    marks are staged); 0: H2D -> kernel -> D2H through the slot's device staging."""
    qa.tune("host_zero_copy", zero_copy)
    try:
        _pipe_mixed(oracle, devices, streams, slot)
    finally:
        qa.tune("host_zero_copy", 1)


def _pipe_mixed(oracle, devices, streams, slot):
    pipe = qa.Pipe(devices=devices, streams=streams, slot_bytes=slot)
    assert pipe.slots == streams * (len(devices) if devices else torch.cuda.device_count())
    cases = [make_case(oracle, k, m, B, G, 1000 + 7 * k + B) for k, m, B, G in MIXED]
    for c in cases:  # interleaved: encode one shape, reconstruct it, then the next shape
        pipe.encode(c["code"], c["tx_data"], c["tx_par"], c["B"])
        pipe.reconstruct(c["code"], c["rx_data"], c["rx_par"], c["rx_marks"], c["B"])
    nf = pipe.wait()
    for c in cases:
        B = c["B"]
        assert np.array_equal(c["tx_par"].numpy()[..., :B], c["par_ref"])
        assert np.array_equal(c["rx_data"].numpy()[..., :B], c["rx_ref"])
    assert nf == sum(c["nfail"] for c in cases)
    # a second round on the same pipe: the failed counters were reset by wait()
    c = cases[1]
    pipe.reconstruct(c["code"], c["rx_data"], c["rx_par"], c["rx_marks"], c["B"])
    assert pipe.wait() == c["nfail"]
    pipe.close()


def test_pipe_rejects_pageable_and_oversize(oracle):
    pipe = qa.Pipe(devices=[0], streams=2, slot_bytes=1 << 16)
    code = qa.Code.cauchy(10, 3)
    with pytest.raises(qa.QfecError, match="pinned"):
        pipe.encode(code, np.zeros((4, 10, 1024), np.uint8), np.zeros((4, 3, 1024), np.uint8))
    big = torch.zeros((2, 10, 8192), dtype=torch.uint8).pin_memory()
    with pytest.raises(qa.QfecError, match="exceeds"):
        pipe.encode(code, big, torch.zeros((2, 3, 8192), dtype=torch.uint8).pin_memory())
    assert pipe.wait() == 0
    pipe.close()


def test_codec_rejects_misread_tensors():
    """tensors with another element type would be read as bytes; host tensors
    cannot be launched on."""
    code = qa.Code.cauchy(4, 2)
    d = torch.zeros((8, 4, 64), dtype=torch.uint8, device=DEV)
    p = torch.zeros((8, 2, 64), dtype=torch.uint8, device=DEV)
    with pytest.raises(qa.QfecError, match="dtype"):
        code.encode(d.to(torch.int32), p)
    with pytest.raises(qa.QfecError, match="device tensor"):
        code.encode(d.cpu(), p)
    marks = torch.zeros(8 * 6, dtype=torch.uint8, device=DEV)
    with pytest.raises(qa.QfecError, match="dtype"):
        code.reconstruct(d, p, marks, failed=torch.zeros(1, dtype=torch.float32, device=DEV))
    code.encode(d, p)  # the well-typed call still works
    torch.cuda.synchronize()


@pytest.mark.parametrize("chunk", [7, 0])
def test_rs_reconstruct_host_chunks(oracle, chunk):
    """reed_solomon_reconstruct over host pointer arrays, staged in chunks of `chunk` groups
    (0: the 256 MiB default) with per-chunk decode records; unrecoverable groups -> -1."""
    k, m, B, G = 10, 3, 1000, 53
    rs = qa.ReedSolomon(k, m)
    rng = np.random.default_rng(5)
    data = synth_bytes(77, G * k * B).reshape(G, k, B)
    par = synth_bytes(78, G * m * B).reshape(G, m, B)
    gm = random_marks(rng, G, k, m)
    marks = marks_to_rs_layout(gm, k)
    work = data.copy()
    work.reshape(G * k, B)[marks[: G * k] == 1] = 0x5A
    expect = work.copy()
    oracle.rs_reconstruct(rs.parity.copy(), expect, par.copy(), marks, B)
    qa.tune("host_chunk", chunk)
    try:
        rc = rs.reconstruct(work, par.copy(), marks, B)
    finally:
        qa.tune("host_chunk", 0)
    assert np.array_equal(work, expect)
    assert rc == (-1 if ((gm[:, :k].sum(1) > 0) & (gm.sum(1) > m)).any() else 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, G, k, m, B, q):
    """One rank: libqfec encode + reconstruct of its contiguous slice on cuda:0 (ranks share
    the one GPU of the box), results gathered over gloo for the check only."""
    import torch.distributed as dist
    from quicknet_amd.synth import erasure_marks
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    a, b = shard_range(G, rank, world)
    code = qa.Code.cauchy(k, m)
    data = synth_bytes(4242, G * k * B).reshape(G, k, B)[a:b]
    gm = erasure_marks(4343, G, k + m, m)[a:b]
    d = torch.from_numpy(np.ascontiguousarray(data)).to("cuda:0")
    p = torch.empty((b - a, m, B), dtype=torch.uint8, device="cuda:0")
    code.encode(d, p)
    w = d.clone()
    w[torch.from_numpy(gm[:, :k].astype(bool)).to("cuda:0")] = 0x5A
    code.reconstruct(w, p, torch.from_numpy(marks_to_rs_layout(gm, k)).to("cuda:0"))
    torch.cuda.synchronize()
    out = [None] * world
    dist.all_gather_object(out, (p.cpu().numpy().tobytes(), bool(torch.equal(w, d))))
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


def test_two_ranks_share_gpu_match_single(oracle):
    import torch.multiprocessing as mp
    G, k, m, B, world = 1001, 10, 3, 1024, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, G, k, m, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=90)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = synth_bytes(4242, G * k * B).reshape(G, k, B)
    ref = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(qa.Code.cauchy(k, m).rows, data, ref, B)
    assert b"".join(x[0] for x in out) == ref.tobytes()
    assert all(x[1] for x in out)  # every rank's reconstruct restored its slice


@pytest.mark.parametrize("fast,resident", [(1, 1), (1, 0), (0, 0)])
@pytest.mark.parametrize("k,n,sz", [(10, 13, 1028), (4, 6, 37), (3, 5, 2052), (16, 20, 1400), (3, 5, 4096),
                                    (3, 5, 8200), (1, 161, 64), (160, 161, 100), (13, 18, 1028), (17, 19, 200),
                                    (7, 12, 300), (2, 3, 1028), (12, 16, 1028)])
def test_per_packet_paths_vs_oracle(oracle, fast, resident, k, n, sz):
    """fec_encode / fec_decode on host packets through the resident server (percall_resident 1:
    rows and tables stored into device memory, a request word polled by one resident wave),
    the per-call kernel (percall_fast 1: mapped pinned staging, tables in the kernel arguments,
    one launch, the caller waiting on the kernel's completion word up to 4 KiB, on the stream
    above) and the staged DMA path (percall_fast 0), against the oracle's fec.c restatement.
    sz 4096 is the server's largest packet; sz 8200 needs a multi-block launch, which is always
    waited for on the stream; (1, 161) and (160, 161) are the 160-coefficient limit's two ends;
    the server takes k <= 16 and k * e <= 64 ((16, 20) decodes 64 coefficients, (13, 18) 65 and
    (17, 19) k = 17 go to the one-launch kernel).  The server's straight-line bodies: k == 10 / 4 /
    16 (exact) and k = 7, 2, 12 (padded), one to four rows per chunk, (7, 12) five rows in two
    chunks."""
    rng = np.random.default_rng(k * 100 + sz)
    fp = qa.FecParms(k, n)
    full = fp.matrix
    data = rng.integers(0, 256, (k, sz), dtype=np.uint8)
    qa.tune("percall_fast", fast)
    qa.tune("percall_resident", resident)
    before = qa.percall_stats()
    try:
        for idx in range(k, n):
            dst = np.zeros(sz, np.uint8)
            fp.encode(data, dst, idx, sz)
            exp = np.zeros(sz, np.uint8)
            for c in range(k):
                exp ^= _gf_row(oracle, int(full[idx, c]), data[c])
            assert np.array_equal(dst, exp)
        # decode: the first min(n - k, k) data packets lost, the first k valid ones in group order
        coded = np.concatenate([data, np.zeros((n - k, sz), np.uint8)])
        for idx in range(k, n):
            fp.encode(data, coded[idx], idx, sz)
        keep = sorted(set(range(n)) - set(range(min(n - k, k))))[:k]
        rc, pk, ix = fp.decode(coded[keep], keep, sz)
        rc2, pk2, ix2 = oracle.fec_decode(k, n, full, coded[keep], keep)
        assert rc == rc2 == 0
        assert np.array_equal(pk, pk2) and np.array_equal(ix, ix2)
        assert np.array_equal(pk, data)
        after = qa.percall_stats()
        served = after["calls"] - before["calls"]
        if fast and resident and sz <= 4096 and after["usable"] > 0:
            lost = min(n - k, k)
            # percall_group: one request computes a group's n - k rows, and both encode loops use
            # the same inputs, so every later index is served from the handle's group copy
            grouped = n - k > 1 and k <= 16 and k * (n - k) <= 64
            enc = 1 if grouped else (n - k) * 2 * (k <= 16)
            want = enc + (1 if lost and k <= 16 and k * lost <= 64 else 0)
            assert served == want, served  # every encode (checker + decode input) + the decode
        else:
            assert served == 0
    finally:
        qa.tune("percall_fast", 1)
        qa.tune("percall_resident", 1)


def _encode_checker(oracle, fp, k, n):
    full = fp.matrix
    coefs = sorted(set(full[k:].ravel().tolist()))
    mul = np.array([[oracle.mul(a, b) for b in range(256)] for a in coefs], np.uint8)
    row_of = {c: i for i, c in enumerate(coefs)}

    def expect(data, idx):
        exp = np.zeros(data.shape[1], np.uint8)
        for c in range(k):
            exp ^= mul[row_of[int(full[idx, c])]][data[c]]
        return exp
    return expect


@pytest.mark.parametrize("resident", [1, 0])
def test_per_packet_spin_back_to_back(oracle, resident):
    """2 000 back-to-back fec_encode calls on fresh data each, through the resident server (1)
    or one launch per call waited for on its completion word (0): every output is the oracle's
    (a stale completion word, rows read before the CPU's stores landed, or an output read before
    it landed would show up as a mismatch).  Back to back, the server is launched about once."""
    k, n, sz = 10, 13, 1028
    fp = qa.FecParms(k, n)
    expect = _encode_checker(oracle, fp, k, n)
    rng = np.random.default_rng(2024)
    qa.tune("percall_resident", resident)
    try:
        before = qa.percall_stats()
        for call in range(2000):
            data = rng.integers(0, 256, (k, sz), dtype=np.uint8)
            idx = k + call % (n - k)
            dst = np.zeros(sz, np.uint8)
            fp.encode(data, dst, idx, sz)
            assert np.array_equal(dst, expect(data, idx)), call
        st = qa.percall_stats()
        if resident and st["usable"] > 0:
            assert st["calls"] - before["calls"] == 2000
            # the Python loop between calls (fresh data, the oracle check) stays well under 1 ms
            assert st["launches"] - before["launches"] <= 20, st
        else:
            assert st["calls"] == before["calls"]
    finally:
        qa.tune("percall_resident", 1)


def test_per_packet_threads(oracle):
    """fec_encode / fec_decode from four host threads at once (ctypes drops the GIL, so the calls
    really overlap), each on its own handle and fresh packets: every call is served by the one
    resident server of the device, one request at a time, and every output is the oracle's."""
    import threading
    k, n, sz = 10, 13, 1028
    fps = [qa.FecParms(k, n) for _ in range(4)]
    expect = _encode_checker(oracle, fps[0], k, n)
    full = fps[0].matrix
    errors = []
    qa.tune("percall_resident", 1)
    before = qa.percall_stats()

    def worker(t):
        rng = np.random.default_rng(900 + t)
        fp = fps[t]
        try:
            for call in range(150):
                data = rng.integers(0, 256, (k, sz), dtype=np.uint8)
                idx = k + call % (n - k)
                dst = np.zeros(sz, np.uint8)
                fp.encode(data, dst, idx, sz)
                if not np.array_equal(dst, expect(data, idx)):
                    errors.append(("encode", t, call))
                if call % 10 == 0:  # a decode with the first 3 data packets lost
                    coded = np.concatenate([data, np.zeros((n - k, sz), np.uint8)])
                    for j in range(k, n):
                        coded[j] = expect(data, j)
                    keep = list(range(3, n))
                    rc, pk, ix = fp.decode(coded[keep], keep, sz)
                    if rc != 0 or not np.array_equal(pk, data):
                        errors.append(("decode", t, call))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(("raised", t, repr(e)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:5]
    st = qa.percall_stats()
    if st["usable"] > 0:
        assert st["calls"] - before["calls"] == 4 * (150 + 15)
    assert full is not None


def test_percall_server_idle_exit_and_relaunch(oracle):
    """The resident server exits by itself 1 ms after its last request (so no block outlives an
    idle caller, and a device synchronise never waits on it for long), a call after an idle gap
    relaunches it, calls spaced around the 1 ms idle limit (where a request can meet a server on
    its way out) are all served correctly, and percall_resident 0 stops it at once."""
    import time

    import torch
    k, n, sz = 10, 13, 1028
    fp = qa.FecParms(k, n)
    expect = _encode_checker(oracle, fp, k, n)
    rng = np.random.default_rng(77)

    def call(i):
        data = rng.integers(0, 256, (k, sz), dtype=np.uint8)
        idx = k + i % (n - k)
        dst = np.zeros(sz, np.uint8)
        fp.encode(data, dst, idx, sz)
        assert np.array_equal(dst, expect(data, idx)), i

    qa.tune("percall_resident", 1)
    call(0)
    st = qa.percall_stats()
    if st["usable"] < 0:
        pytest.skip("device memory not CPU-mapped on this box: the launch-per-call path serves")
    assert st["usable"] == 1 and st["calls"] >= 1
    time.sleep(0.02)
    assert not qa.percall_stats()["running"]  # exited within 20 ms (its limit is 1 ms idle)
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 0.5
    l0 = qa.percall_stats()["launches"]
    call(1)
    st = qa.percall_stats()
    assert st["launches"] == l0 + 1 and st["running"]
    # gaps from 0.5 to 1.5 ms: some requests find the server alive, some find it gone, some
    # arrive as it leaves
    for i in range(300):
        t = time.perf_counter() + (0.5 + (i % 11) * 0.1) * 1e-3
        while time.perf_counter() < t:
            pass
        call(2 + i)
    st = qa.percall_stats()
    assert st["launches"] > l0 + 1  # the longer gaps did meet an exited server
    qa.tune("percall_resident", 0)
    assert not qa.percall_stats()["running"]
    qa.tune("percall_resident", 1)
    call(400)


def test_fec_encode_group_cache(oracle):
    """fec_encode's group cache (percall_group 1): the n - k calls of one group (the way
    get_fec_encoded_pkt asks for them, network/NetFecCodec.cpp:133-166) cost one request; inputs
    mutated between the calls, reused pointers with new contents, another sz and interleaved
    handles all get the rows of the bytes they pass, checked against the oracle every time."""
    k, n, sz = 10, 13, 1028
    fa, fb = qa.FecParms(k, n), qa.FecParms(k, n)
    expect = _encode_checker(oracle, fa, k, n)
    rng = np.random.default_rng(31)

    def enc(fp, data, idx, size=sz):
        dst = np.full(size, 0xEE, np.uint8)
        fp.encode(data, dst, idx, size)
        assert np.array_equal(dst, expect(data[:, :size], idx)), (idx, size)

    def counters():
        c = qa.percall_counters()
        return c["group_hits"], c["group_misses"]

    h0, m0 = counters()
    data = rng.integers(0, 256, (k, sz), dtype=np.uint8)
    for idx in range(k, n):
        enc(fa, data, idx)
    h1, m1 = counters()
    assert (h1 - h0, m1 - m0) == (n - k - 1, 1)
    # a byte of one input changed between two calls of the group: recomputed
    data[3, 500] ^= 0x5A
    enc(fa, data, k + 1)
    # the same buffers, wholly new contents (the pointers repeat): recomputed
    data[:] = rng.integers(0, 256, (k, sz), dtype=np.uint8)
    enc(fa, data, k + 2)
    enc(fa, data, k)
    # a shorter sz over the same pointers: recomputed
    enc(fa, data, k + 1, size=700)
    enc(fa, data, k + 2, size=700)
    h2, m2 = counters()
    assert (h2 - h1, m2 - m1) == (2, 3)
    # two handles interleaved, each with its own group
    da = rng.integers(0, 256, (k, sz), dtype=np.uint8)
    db = rng.integers(0, 256, (k, sz), dtype=np.uint8)
    for idx in range(k, n):
        enc(fa, da, idx)
        enc(fb, db, idx)
    h3, m3 = counters()
    assert (h3 - h2, m3 - m2) == (2 * (n - k - 1), 2)
    # the index < k copy and the index >= n no-op stay as the reference has them
    dst = np.zeros(sz, np.uint8)
    fa.encode(da, dst, 4, sz)
    assert np.array_equal(dst, da[4])
    dst[:] = 0x33
    fa.encode(da, dst, n, sz)
    assert (dst == 0x33).all()
    # percall_group 0: one request per index, same bytes
    qa.tune("percall_group", 0)
    try:
        for idx in range(k, n):
            enc(fa, da, idx)
        assert counters() == (h3, m3)
    finally:
        qa.tune("percall_group", 1)


def test_fec_encode_group_cache_threads(oracle):
    """Four threads encoding groups through ONE handle: each group is computed under the handle's
    group lock, so a thread never receives rows of another thread's inputs."""
    import threading
    k, n, sz = 10, 13, 1028
    fp = qa.FecParms(k, n)
    expect = _encode_checker(oracle, fp, k, n)
    errors = []

    def worker(t):
        rng = np.random.default_rng(4100 + t)
        try:
            for g in range(60):
                data = rng.integers(0, 256, (k, sz), dtype=np.uint8)
                for idx in range(k, n):
                    dst = np.zeros(sz, np.uint8)
                    fp.encode(data, dst, idx, sz)
                    if not np.array_equal(dst, expect(data, idx)):
                        errors.append((t, g, idx))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(("raised", t, repr(e)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:5]


def test_percall_timeout_branch(oracle):
    """a request the server does not serve within percall_timeout_us is not lost.  With
    the limit at 0 every call stops the server and waits for it (it serves the pending request on
    its way out); with percall_fault 1 no server ever takes the request, and the call runs it through
    one launch.  Every output is the oracle's, encodes and decodes alike."""
    k, n, sz = 10, 13, 1028
    fp = qa.FecParms(k, n)
    full = fp.matrix
    expect = _encode_checker(oracle, fp, k, n)
    rng = np.random.default_rng(55)
    qa.tune("percall_resident", 1)
    qa.tune("percall_group", 0)
    c0 = qa.percall_counters()
    if c0["usable"] < 0:
        pytest.skip("device memory not CPU-mapped on this box: the launch-per-call path serves")
    try:
        for fault in (0, 1):
            qa.tune("percall_timeout_us", 0)
            qa.tune("percall_fault", fault)
            before = qa.percall_counters()
            for call in range(60):
                data = rng.integers(0, 256, (k, sz), dtype=np.uint8)
                idx = k + call % (n - k)
                dst = np.zeros(sz, np.uint8)
                fp.encode(data, dst, idx, sz)
                assert np.array_equal(dst, expect(data, idx)), (fault, call)
                if call % 10 == 0:
                    coded = np.concatenate([data, np.stack([expect(data, j) for j in range(k, n)])])
                    keep = list(range(3, n))
                    rc, pk, ix = fp.decode(coded[keep], keep, sz)
                    rc2, pk2, _ = oracle.fec_decode(k, n, full, coded[keep], keep)
                    assert rc == rc2 == 0 and np.array_equal(pk, pk2) and np.array_equal(pk, data)
            after = qa.percall_counters()
            assert after["timeouts"] - before["timeouts"] >= (66 if fault else 1), after
            if fault:
                assert after["calls"] == before["calls"]  # no server ever served one
    finally:
        qa.tune("percall_fault", 0)
        qa.tune("percall_timeout_us", 2000000)
        qa.tune("percall_group", 1)
    data = rng.integers(0, 256, (k, sz), dtype=np.uint8)
    dst = np.zeros(sz, np.uint8)
    fp.encode(data, dst, k, sz)  # and the server serves again
    assert np.array_equal(dst, expect(data, k))


def test_percall_abandon_branch(oracle, capfd):
    """the wait for a stopped server is bounded by percall_stop_us.  With percall_fault
    2 (no server takes the request, and the stopped block counts as not done within percall_stop_us)
    fec_encode prints to stderr and leaves dst as it was, fec_decode returns 1, and the device's
    server is abandoned (usable -2): later calls run through one launch, oracle-exact, and
    percall_resident 1 sets up a fresh server.  No real CU starvation is needed."""
    import time
    k, n, sz = 10, 13, 1028
    fp = qa.FecParms(k, n)
    full = fp.matrix
    expect = _encode_checker(oracle, fp, k, n)
    rng = np.random.default_rng(57)
    qa.tune("percall_resident", 1)
    qa.tune("percall_group", 0)
    c0 = qa.percall_counters()
    if c0["usable"] == -1:
        pytest.skip("device memory not CPU-mapped on this box: the launch-per-call path serves")
    data = rng.integers(0, 256, (k, sz), dtype=np.uint8)
    coded = np.concatenate([data, np.stack([expect(data, j) for j in range(k, n)])])
    keep = list(range(3, n))
    try:
        qa.tune("percall_timeout_us", 0)
        qa.tune("percall_fault", 2)
        dst = np.full(sz, 0xA5, np.uint8)
        t0 = time.perf_counter()
        fp.encode(data, dst, k, sz)
        assert time.perf_counter() - t0 < 1.0
        assert (dst == 0xA5).all()  # left as it was
        assert "[qfec] fec_encode:" in capfd.readouterr().err
        c1 = qa.percall_counters()
        assert c1["usable"] == -2 and c1["abandoned"] == c0["abandoned"] + 1, c1
        qa.tune("percall_fault", 0)
        fp.encode(data, dst, k, sz)  # the one-launch path while the server is abandoned
        assert np.array_equal(dst, expect(data, k))
        assert qa.percall_counters()["usable"] == -2
        qa.tune("percall_resident", 1)  # retry: a fresh server at the next call
        qa.tune("percall_fault", 2)
        rc, _, _ = fp.decode(coded[keep], keep, sz)
        assert rc == 1
        assert qa.percall_counters()["abandoned"] == c0["abandoned"] + 2
    finally:
        qa.tune("percall_fault", 0)
        qa.tune("percall_timeout_us", 2000000)
        qa.tune("percall_group", 1)
        qa.tune("percall_resident", 1)
    rc, pk, _ = fp.decode(coded[keep], keep, sz)
    rc2, pk2, _ = oracle.fec_decode(k, n, full, coded[keep], keep)
    assert rc == rc2 == 0 and np.array_equal(pk, pk2)
    dst = np.zeros(sz, np.uint8)
    fp.encode(data, dst, k + 1, sz)
    assert np.array_equal(dst, expect(data, k + 1))
    assert qa.percall_counters()["usable"] == 1  # served by a fresh server again


def test_percall_idle_knob_bounds_device_sync(oracle):
    """The resident block's footprint (qfec.h): a hipDeviceSynchronize issued
    right after a call waits for the block's idle exit, at most percall_idle_us (1 ms by default) --
    measured here at <= 2 ms -- and percall_idle_us 0 makes the block exit right after each call."""
    import time

    import torch
    k, n, sz = 10, 13, 1028
    fp = qa.FecParms(k, n)
    expect = _encode_checker(oracle, fp, k, n)
    rng = np.random.default_rng(808)
    qa.tune("percall_resident", 1)

    def call():
        data = rng.integers(0, 256, (k, sz), dtype=np.uint8)
        dst = np.zeros(sz, np.uint8)
        fp.encode(data, dst, k, sz)
        assert np.array_equal(dst, expect(data, k))

    call()
    if qa.percall_counters()["usable"] < 0:
        pytest.skip("device memory not CPU-mapped on this box: the launch-per-call path serves")
    torch.cuda.synchronize()
    waits = []
    for _ in range(7):
        call()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        waits.append(time.perf_counter() - t0)
    assert qa.percall_counters()["idle_us"] == 1000
    assert sorted(waits)[3] <= 2e-3, waits
    qa.tune("percall_idle_us", 0)
    try:
        l0 = qa.percall_counters()["launches"]
        zero = []
        for _ in range(7):
            call()
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            zero.append(time.perf_counter() - t0)
        c = qa.percall_counters()
        assert c["idle_us"] == 0 and c["launches"] - l0 >= 6  # a launch per call
        assert sorted(zero)[3] <= 0.5e-3, zero
    finally:
        qa.tune("percall_idle_us", 1000)
    call()


def _gf_row(oracle, c, row):
    """c * row over GF(2^8) via the oracle's multiplication table (256 products, then a gather)."""
    t = np.array([oracle.mul(c, b) for b in range(256)], np.uint8)
    return t[row]


@pytest.mark.parametrize("k,n,sz", [(10, 13, 1028), (4, 6, 100), (16, 20, 4096), (7, 12, 333), (1, 2, 64),
                                    (128, 256, 96), (200, 255, 40)])
def test_fec_packets_vs_reference_fec(k, n, sz):
    """fec_encode / fec_decode of libqfec against the reference's own system/fec.c
    (oracle/_ref/libref_fec.so) on the same packets: every parity index encoded by both, then
    decodes from random k-subsets handed over in random order (fec_decode's shuffle moves them
    into place) -- output packets, index arrays and return codes equal."""
    import ctypes as C
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle.oracle import RefCodec
    if not RefCodec.available():
        pytest.skip("reference libraries not built (make -C oracle ref)")
    ref = RefCodec()
    L = qa.lib()
    rng = np.random.default_rng(k * 7 + n + sz)
    data = rng.integers(0, 256, (k, sz), dtype=np.uint8)
    h, hr = L.fec_new(k, n), ref.fec.fec_new(k, n)
    try:
        src = (C.c_void_p * k)(*[data[i].ctypes.data for i in range(k)])
        coded = np.zeros((n, sz), np.uint8)
        coded[:k] = data
        for idx in range(k, n):
            out, outr = np.zeros(sz, np.uint8), np.zeros(sz, np.uint8)
            L.fec_encode(h, src, out.ctypes.data, idx, sz)
            ref.fec.fec_encode(hr, src, outr.ctypes.data, idx, sz)
            assert np.array_equal(out, outr), idx
            coded[idx] = out
        for trial in range(6):
            keep = rng.choice(n, size=k, replace=False)
            if trial % 2:
                keep = np.sort(keep)
            bufs = [coded[keep].copy(), coded[keep].copy()]
            idxs = [np.ascontiguousarray(keep, dtype=np.int32), np.ascontiguousarray(keep, dtype=np.int32)]
            rcs = []
            for (b, ix, fn, hh) in ((bufs[0], idxs[0], L.fec_decode, h), (bufs[1], idxs[1], ref.fec.fec_decode, hr)):
                pk = (C.c_void_p * k)(*[b[i].ctypes.data for i in range(k)])
                rcs.append(fn(hh, pk, ix.ctypes.data_as(C.POINTER(C.c_int)), sz))
            assert rcs[0] == rcs[1] == 0
            assert np.array_equal(idxs[0], idxs[1])
            assert np.array_equal(bufs[0], bufs[1])
    finally:
        L.fec_free(h)
        ref.fec.fec_free(hr)
