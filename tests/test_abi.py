"""CPU tests of libqfec: it loads, exports every symbol include/*.h declares, and its host
logic (matrix builders, decode-matrix selection, handle bookkeeping) matches the golden
vectors the reference produced.  No kernel is launched here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT

import quicknet_amd as qa
from quicknet_amd._lib import EXPORTS, lib


def header_functions(path):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"^typedef .*?;", "", txt, flags=re.S | re.M)   # callback types
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b([a-z_][a-z0-9_]*)\s*\(", txt, flags=re.M)
    return sorted(set(n for n in names if n not in ("defined",)))


@pytest.mark.parametrize("header", ["qfec.h", "qfec_fec.h", "qfec_rs.h", "qfec_net.h", "qfec_zfec.h"])
def test_exports_match_headers(header):
    L = lib()
    declared = header_functions(os.path.join(ROOT, "include", header))
    assert declared, header
    assert sorted(EXPORTS[header]) == declared
    for name in declared:
        assert hasattr(L, name), f"{name} not exported"


def test_version():
    assert lib().qfec_version().decode().startswith("qfec")


def test_matrices_vs_golden(golden):
    z = golden("matrices.npz")
    for key in z.files:
        if key.startswith("rs_") and key != "rs_errors":
            k, m = map(int, key.split("_")[1:])
            assert np.array_equal(qa.Code.cauchy(k, m).rows, z[key]), key
        elif key.startswith("fec_") and key != "fec_errors":
            k, n = map(int, key.split("_")[1:])
            if n > k:
                assert np.array_equal(qa.Code.vandermonde(k, n - k).rows, z[key][k:]), key
            f = qa.FecParms(k, n)
            assert np.array_equal(f.matrix, z[key]), key


def test_reed_solomon_handle_vs_golden(golden):
    """reed_solomon_new exposes the same public struct contents as module/rs.c."""
    z = golden("matrices.npz")
    L = lib()
    for k, m in [(1, 1), (4, 2), (10, 3), (16, 4), (200, 55), (1, 254)]:
        rs = qa.ReedSolomon(k, m)
        h = rs._h.contents
        assert (h.data_shards, h.parity_shards, h.shards) == (k, m, k + m)
        full = np.ctypeslib.as_array(h.m, shape=(k + m, k))
        assert np.array_equal(full, z[f"rsfull_{k}_{m}"])
        assert np.array_equal(rs.parity, z[f"rs_{k}_{m}"])
        assert L.reed_solomon_error() == 0
    for k, m, err in z["rs_errors"]:
        assert not L.reed_solomon_new(int(k), int(m))
        assert L.reed_solomon_error() == err


def test_fec_new_rejects_like_reference(golden):
    z = golden("matrices.npz")
    for k, n, ok in z["fec_errors"]:
        assert not lib().fec_new(int(k), int(n))


def test_decode_rows_host(oracle):
    """Decode-matrix selection (module/rs.c:620-629) + GF inversion on the host."""
    rng = np.random.default_rng(5)
    for flavour in ("cauchy", "vandermonde"):
        for k, m in [(4, 2), (10, 3), (16, 4), (5, 3)]:
            code = getattr(qa.Code, flavour)(k, m)
            P = code.rows
            for _ in range(40):
                marks = (rng.random(k + m) < 0.25).astype(np.uint8)
                e, rows, surv, lost = code.decode_rows(marks)
                lost_ref = [i for i in range(k) if marks[i]]
                avail = [j for j in range(m) if not marks[k + j]]
                if not lost_ref:
                    assert e == 0
                    continue
                if len(avail) < len(lost_ref):
                    assert e == -1
                    continue
                chosen = avail[: len(lost_ref)]
                surv_ref = [i for i in range(k) if not marks[i]] + [k + j for j in chosen]
                assert e == len(lost_ref) and list(lost) == lost_ref and list(surv) == surv_ref
                D = np.zeros((k, k), dtype=np.uint8)
                for r, s in enumerate(surv_ref):
                    if s < k:
                        D[r, s] = 1
                    else:
                        D[r] = P[s - k]
                inv = oracle.invert(D)
                assert np.array_equal(rows, inv[lost_ref])


def test_no_gpu_fails_loudly():
    """Without a device every compute entry point errors (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    L = lib()
    assert L.qfec_device_count() == 0
    rc = L.qfec_synth_fill(C.c_void_p(64), 16, 1, None)
    assert rc == -2 and "no HIP device" in L.qfec_last_error().decode()
    code = qa.Code.cauchy(4, 2)
    rc = L.qfec_encode(code._h, C.c_void_p(64), C.c_void_p(128), 1, 16, 16, None)
    assert rc == -2
    rs = qa.ReedSolomon(4, 2)
    data = np.zeros((1, 4, 16), np.uint8)
    par = np.zeros((1, 2, 16), np.uint8)
    assert rs.encode(data, par, 16) != 0
    arr = (C.c_int * 2)(0, 0)
    assert L.qfec_rs_host_devices(arr, 2) == -2  # no device to list


def test_net_layer_host_side():
    """qfec_net (include/qfec_net.h): argument checks and session numbering run on the host;
    a flush without a device fails loudly (QFEC_ENODEV), it does not fall back."""
    import ctypes as C
    L = qa.lib()
    assert not L.qfec_net_new(4, 16, 1400, 1)      # n > 15: the header's 4-bit field
    assert not L.qfec_net_new(4, 4, 1400, 1)       # no check packets
    h = L.qfec_net_new(4, 6, 1400, 1)
    assert h
    s0, s1 = L.qfec_net_session(h, None), L.qfec_net_session(h, None)
    assert (s0, s1) == (0, 1)
    assert L.qfec_net_pack_input(h, 0, b"x" * 1401, 1401) < 0     # > max_pkt_size
    assert L.qfec_net_pack_input(h, 7, b"x", 1) < 0               # no such session
    for i in range(4):
        assert L.qfec_net_pack_input(h, s1, bytes([i]) * 10, 10) == 0
    # dropped on the host: empty, a header no codec fits (k >= n), ik >= n
    assert L.qfec_net_unpack_input(h, 0, b"", 0) == 0
    bad = bytes([0xED]) + bytes(8) + bytes([5 | 7 << 4, 0]) + bytes(20)
    assert L.qfec_net_unpack_input(h, 0, bad, len(bad)) == 0
    bad = bytes([0xED]) + bytes(8) + bytes([5 | 3 << 4, 9]) + bytes(20)
    assert L.qfec_net_unpack_input(h, 0, bad, len(bad)) == 0
    # queued: another (k, n) (decoded with its own code), and non-FEC / short datagrams
    other = bytes([0xED]) + bytes(8) + bytes([5 | 3 << 4, 0]) + bytes(20)
    assert L.qfec_net_unpack_input(h, 0, other, len(other)) == 1
    assert L.qfec_net_unpack_input(h, 0, b"\xed" * 5, 5) == 1
    st = (C.c_longlong * 8)()
    assert L.qfec_net_stats(h, st) == 0 and st[6] == 3
    assert L.qfec_net_enable(h, 9, 0) < 0
    if L.qfec_device_count() <= 0:
        assert L.qfec_net_flush_pack(h, None, None) == -2   # QFEC_ENODEV
    L.qfec_net_free(h)


def test_net_layer_fec_off_host_side():
    """FEC off at a session (enable_zfec): [0x13][payload] datagrams, no numbering advance;
    non-FEC datagrams received are handed over minus their tag, source index 0.  Neither
    needs the device, so this runs anywhere (byte-pinned to the reference in
    tests/test_reference_callers.py)."""
    net = qa.NetFec(4, 6, max_pkt_size=1400)
    s = net.session()
    net.enable(s, False)
    net.pack_input(s, b"abc")
    net.pack_input(s, b"")
    assert net.flush_pack() == [(s, b"\x13abc"), (s, b"\x13")]
    rx = qa.NetFec(4, 6)
    r = rx.session()
    assert rx.unpack_input(r, b"\x13abc") == 1
    assert rx.unpack_input(r, b"\xed" * 5) == 1   # an FEC tag but under 11 bytes: plain too
    assert rx.flush_unpack() == [(r, b"abc", 0), (r, b"\xed" * 4, 0)]
    assert rx.stats()["delivered"] == 2


def test_tune_keys_documented_and_accepted():
    """Every qfec_tune key that include/qfec.h documents is accepted with its documented first
    value (host state only: no device is touched), and an unknown key or value is refused."""
    text = open(os.path.join(ROOT, "include", "qfec.h")).read()
    block = text[text.index("int qfec_tune(") - 6000:text.index("int qfec_tune(")]
    keys = re.findall(r'^ \*   "(\w+)"\s+(-?\d+)?', block, re.M)
    assert len(keys) >= 13, keys
    # the A/B switches retired in round 5 (bodies the auto choice never picks) are refused
    for gone in ("recon_compact", "recon_full_lines", "wire_store_nt", "wire_line", "wire_chunk", "wire_send_wave",
                 "frame_rows", "wire_fused_rx", "wire_rx_split", "wire_rx_lds", "wire_rx_skip_lost", "percall_in",
                 "percall_spin"):
        assert lib().qfec_tune(gone.encode(), 0) != 0, gone
    L = lib()
    before = {key: qa.tune_get(key) for key, _ in keys}
    try:
        for key, first in keys:
            value = int(first) if first else 0
            assert L.qfec_tune(key.encode(), value) == 0, (key, value)
            assert qa.tune_get(key) == value
        assert L.qfec_tune(b"no_such_knob", 1) != 0
        assert L.qfec_tune(b"percall_in", 7) != 0
        assert L.qfec_tune(b"recon_impl", 99) != 0
        v = C.c_int(0)
        assert L.qfec_tune_get(b"no_such_knob", C.byref(v)) != 0
    finally:
        # back to the values the rest of this process runs with
        for key, value in before.items():
            assert L.qfec_tune(key.encode(), value) == 0
    assert {key: qa.tune_get(key) for key, _ in keys} == before


def test_tune_while_encoding_threads():
    """qfec_tune / qfec_tune_get from one thread while others call the codec (knobs are atomics
    read per launch decision, SURVEY 8(b) threading).  Without a device the codec calls fail with
    QFEC_ENODEV every time; on a GPU box they run (tests/test_gpu_rs_host.py checks the bytes)."""
    import threading
    L = lib()
    keys = ("host_chunk", "host_threads", "host_zero_copy", "recon_impl", "encode_impl")
    before = {k: qa.tune_get(k) for k in keys}
    stop = threading.Event()
    errors = []

    def tuner():
        i = 0
        while not stop.is_set():
            for k, vals in (("host_chunk", (0, 3, 17)), ("host_threads", (0, 1, 2)), ("host_zero_copy", (0, 1)),
                            ("recon_impl", (-1, 3)), ("encode_impl", (-1, 0))):
                if L.qfec_tune(k.encode(), vals[i % len(vals)]) != 0:
                    errors.append(k)
                qa.tune_get(k)
            i += 1

    def coder(seed):
        rs = qa.ReedSolomon(4, 2)
        data = np.zeros((3, 4, 64), np.uint8)
        par = np.zeros((3, 2, 64), np.uint8)
        marks = np.zeros(18, np.uint8)
        for _ in range(200):
            rc = rs.encode(data, par, 64)
            if rc not in (0, -2):
                errors.append(("encode", rc))
            if rs.reconstruct(data, par, marks, 64) != 0:  # nothing erased: 0 with or without a device
                errors.append("reconstruct")
        rs.close()

    t = threading.Thread(target=tuner)
    coders = [threading.Thread(target=coder, args=(i,)) for i in range(3)]
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


def test_fec_decode_shuffle_and_pattern_cache(oracle):
    """fec_decode's host part on CPU (sz = 0: no bytes move, so no device is touched): the
    shuffle's permutation of pkt[] and index[], and the return code for valid, conflicting,
    invalid and duplicate index lists, equal the oracle's restatement of fec.c:738-862 over
    6 000 random calls -- more distinct loss patterns than the per-handle decode cache holds
    (4 096), so the cache is cleared and refilled on the way, and every repeat of a pattern
    is served from it."""
    L = lib()
    k, n = 10, 20
    h = C.c_void_p(L.fec_new(k, n))
    full = np.zeros((n, k), np.uint8)
    assert L.qfec_fec_matrix(h, full.ctypes.data_as(C.c_void_p)) == 0
    rng = np.random.default_rng(77)
    bufs = np.zeros((n, 4), np.uint8)
    base = bufs.ctypes.data
    prev = None
    for call in range(6000):
        if call % 7 == 0 and prev is not None:  # a repeat: served from the cache
            idx = list(prev)
        elif call % 50 == 49:  # now and then an invalid or conflicting list
            idx = list(rng.choice(n, k, replace=False))
            if call % 100 == 49:
                idx[int(rng.integers(0, k))] = n + 3  # invalid index
            else:
                idx[1] = idx[0] if idx[0] < k else int(rng.integers(0, k))  # duplicate / conflict
        else:
            idx = sorted(rng.choice(n, k, replace=False)) if call % 3 else list(rng.choice(n, k, replace=False))
        idx = [int(x) for x in idx]
        prev = idx
        ptrs = (C.c_void_p * k)(*[base + 4 * i for i in range(k)])
        ia = (C.c_int * k)(*idx)
        rc = L.fec_decode(h, ptrs, ia, 0)
        rc2, _, ix2 = oracle.fec_decode(k, n, full, bufs[:k], idx)
        assert rc == rc2, (call, idx, rc, rc2)
        if rc == 0:
            assert list(ia) == list(ix2), (call, idx)
            # the pointers moved with their indices: slot s holds the buffer the caller gave for index[s]
            where = {v: i for i, v in enumerate(idx)}
            assert [((p - base) // 4) for p in ptrs] == [where[v] for v in ia], (call, idx)
    L.fec_free(h)


@pytest.mark.parametrize("name", ["p42", "m42", "s42", "s103", "m103w", "m164w"])
def test_rs_edits_decode_rows_host(oracle, golden, name):
    """The host half of reed_solomon_reconstruct on a handle whose public `m` / `parity` were
    edited (rs_edits.npz, produced by the reference's rs.c): qfec_rs_code picks the edits up, and
    every pattern's decode rows are rows `lost` of rs.c's invert_mat over rs->m's survivor rows
    -- the partial elimination state when the sub-matrix is singular (rs.c:505-556).  CPU only:
    the kernels that apply these rows are held to the fixture's bytes in test_gpu_parity.py."""
    z = golden("rs_edits.npz")
    k, m, B = (int(x) for x in z[f"shape_{name}"])
    rs = qa.ReedSolomon(k, m)
    rs.parity[:] = z[f"parity_{name}"]
    rs.m_matrix[:] = z[f"m_{name}"]
    code = rs.code()
    assert np.array_equal(code.rows, z[f"parity_{name}"])
    full = z[f"m_{name}"]
    singular = 0
    for mask in np.unique(z[f"marks_{name}"], axis=0)[:600]:
        e, rows, surv, lost = code.decode_rows(mask)
        lost_ref = [i for i in range(k) if mask[i]]
        avail = [k + j for j in range(m) if not mask[k + j]]
        if not lost_ref:
            assert e == 0
            continue
        if len(avail) < len(lost_ref):
            assert e == -1
            continue
        surv_ref = [i for i in range(k) if not mask[i]] + avail[:len(lost_ref)]
        assert e == len(lost_ref) and list(surv) == surv_ref and list(lost) == lost_ref
        rc, inv = oracle.invert_partial(full[surv_ref])
        singular += rc != 0
        assert np.array_equal(rows, inv[lost_ref]), mask
    assert singular > 0 or name in ("p42", "m42")  # every other case has singular patterns by design
    rs.close()
