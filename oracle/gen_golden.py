#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ by running the REFERENCE itself.

TEST INFRASTRUCTURE.  Runs only in the build container, where /root/reference exists:
`make -C oracle ref` compiles the reference's own module/rs.c and system/fec.c (read in
place, never copied) into oracle/_ref/, and this script drives those libraries through
ctypes on seeded synthetic inputs (quicknet_amd/synth.py).  The outputs are committed as
small .npz fixtures; the tests then pin both the CPU restatement (oracle/liboracle.so)
and the HIP product path against them on the GPU box, where the reference is absent.

    python oracle/gen_golden.py            # rewrites tests/golden/*.npz

Reference entry points driven (file:line in /root/reference):
  reed_solomon_init/new/encode/reconstruct/error   module/rs.c:382,387,574,598,649
  fec_new/fec_encode/fec_decode/fec_free           system/fec.c:653,714,821,639
"""
import ctypes as C
import hashlib
import itertools
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from quicknet_amd.synth import synth_bytes  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


class RS(C.Structure):  # module/rs.h:7-13
    _fields_ = [("data_shards", C.c_int), ("parity_shards", C.c_int), ("shards", C.c_int),
                ("m", C.POINTER(C.c_ubyte)), ("parity", C.POINTER(C.c_ubyte))]


class FecParms(C.Structure):  # module/fec.c:633-636
    _fields_ = [("k", C.c_int), ("n", C.c_int), ("enc_matrix", C.POINTER(C.c_ubyte))]


def load_ref():
    rs = C.CDLL(os.path.join(HERE, "_ref", "libref_rs.so"))
    fec = C.CDLL(os.path.join(HERE, "_ref", "libref_fec.so"))
    rs.reed_solomon_new.restype = C.POINTER(RS)
    rs.reed_solomon_new.argtypes = [C.c_int, C.c_int]
    rs.reed_solomon_release.argtypes = [C.POINTER(RS)]
    rs.reed_solomon_encode.argtypes = [C.POINTER(RS), C.POINTER(C.c_void_p), C.c_int, C.c_int]
    rs.reed_solomon_reconstruct.argtypes = [C.POINTER(RS), C.POINTER(C.c_void_p), C.c_void_p, C.c_int, C.c_int]
    fec.fec_new.restype = C.POINTER(FecParms)
    fec.fec_new.argtypes = [C.c_int, C.c_int]
    fec.fec_free.argtypes = [C.POINTER(FecParms)]
    fec.fec_encode.argtypes = [C.POINTER(FecParms), C.POINTER(C.c_void_p), C.c_void_p, C.c_int, C.c_int]
    fec.fec_decode.argtypes = [C.POINTER(FecParms), C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.c_int]
    rs.reed_solomon_init()
    return rs, fec


def ptr(a, off=0):
    return a.ctypes.data + off


def rs_matrix(rs, k, m):
    h = rs.reed_solomon_new(k, m)
    if not h:
        return None, rs.reed_solomon_error()
    p = np.ctypeslib.as_array(h.contents.parity, shape=(m * k,)).copy()
    full = np.ctypeslib.as_array(h.contents.m, shape=((k + m) * k,)).copy()
    rs.reed_solomon_release(h)
    return (p.reshape(m, k), full.reshape(k + m, k)), 0


def fec_matrix(fec, k, n):
    h = fec.fec_new(k, n)
    if not h:
        return None
    full = np.ctypeslib.as_array(h.contents.enc_matrix, shape=(n * k,)).copy().reshape(n, k)
    fec.fec_free(h)
    return full


def gen_matrices(rs, fec):
    out = {}
    rs_shapes = [(1, 1), (2, 1), (3, 2), (4, 2), (7, 1), (10, 3), (16, 4), (32, 8), (64, 32),
                 (128, 127), (200, 55), (254, 1), (1, 254)]
    for k, m in rs_shapes:
        (p, full), err = rs_matrix(rs, k, m)
        assert err == 0
        out[f"rs_{k}_{m}"] = p
        out[f"rsfull_{k}_{m}"] = full
    errs = []
    for k, m in [(0, 1), (1, 0), (200, 56), (-1, 3), (255, 1)]:
        res, err = rs_matrix(rs, k, m)
        assert res is None
        errs.append((k, m, err))
    out["rs_errors"] = np.array(errs, dtype=np.int32)
    fec_shapes = [(1, 1), (1, 2), (2, 4), (3, 5), (5, 8), (4, 6), (3, 4), (4, 5), (5, 6), (7, 8),
                  (10, 13), (16, 20), (4, 4), (32, 40), (100, 150), (128, 256), (200, 255),
                  (256, 256), (255, 256), (1, 256), (2, 3)]
    for k, n in fec_shapes:
        full = fec_matrix(fec, k, n)
        assert full is not None
        out[f"fec_{k}_{n}"] = full
    bad = []
    for k, n in [(257, 257), (5, 4), (3, 257)]:
        bad.append((k, n, 0 if fec_matrix(fec, k, n) is None else 1))
    out["fec_errors"] = np.array(bad, dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, "matrices.npz"), **out)
    return out


ENC_CASES = [(2, 1), (4, 2), (10, 3), (16, 4), (7, 1), (3, 2)]
ENC_LENS = [1, 8, 1024, 1400, 37]
ENC_GROUPS = 4


def gen_encode(rs, fec):
    out = {}
    seed = 0xE0C0DE00
    for (k, m), B in itertools.product(ENC_CASES, ENC_LENS):
        n = k + m
        seed += 1
        G = ENC_GROUPS
        data = synth_bytes(seed, G * k * B).reshape(G * k, B)
        # rs.c: batched encode over the pointer layout (rs.c:574-588)
        par = np.full((G * m, B), 0x5A, dtype=np.uint8)
        h = rs.reed_solomon_new(k, m)
        ptrs = (C.c_void_p * (G * n))(*([ptr(data, i * B) for i in range(G * k)] +
                                         [ptr(par, i * B) for i in range(G * m)]))
        assert rs.reed_solomon_encode(h, ptrs, G * n, B) == 0
        rs.reed_solomon_release(h)
        # fec.c: one fec_encode per parity index (the get_fec_encoded_pkt pattern,
        # network/FecCodecBuf.cpp:151)
        fpar = np.full((G * m, B), 0xA5, dtype=np.uint8)
        fh = fec.fec_new(k, n)
        for g in range(G):
            src = (C.c_void_p * k)(*[ptr(data, (g * k + i) * B) for i in range(k)])
            for j in range(m):
                fec.fec_encode(fh, src, C.c_void_p(ptr(fpar, (g * m + j) * B)), k + j, B)
        # index < k is a copy; index >= n leaves dst untouched
        cp = np.zeros(B, dtype=np.uint8)
        src = (C.c_void_p * k)(*[ptr(data, i * B) for i in range(k)])
        fec.fec_encode(fh, src, C.c_void_p(ptr(cp)), k - 1, B)
        untouched = np.full(B, 0x33, dtype=np.uint8)
        fec.fec_encode(fh, src, C.c_void_p(ptr(untouched)), n, B)
        fec.fec_free(fh)
        key = f"{k}_{m}_{B}"
        out[f"seed_{key}"] = np.array([seed], dtype=np.uint64)
        out[f"rs_{key}"] = par
        out[f"fec_{key}"] = fpar
        out[f"fcopy_{key}"] = cp
        out[f"fbad_{key}"] = untouched
    # the rs.c column-0 zero-coefficient quirk: mul() with c == 0 leaves dst stale
    # (rs.c:116-117).  Poke a zero into the public parity matrix and encode over 0x5A.
    k, m, B, G = 4, 2, 16, 2
    data = synth_bytes(0xE0C0DEFF, G * k * B).reshape(G * k, B)
    par = np.full((G * m, B), 0x5A, dtype=np.uint8)
    h = rs.reed_solomon_new(k, m)
    h.contents.parity[0 * k + 0] = 0
    h.contents.parity[1 * k + 2] = 0
    pm = np.ctypeslib.as_array(h.contents.parity, shape=(m * k,)).copy()
    ptrs = (C.c_void_p * (G * (k + m)))(*([ptr(data, i * B) for i in range(G * k)] +
                                         [ptr(par, i * B) for i in range(G * m)]))
    rs.reed_solomon_encode(h, ptrs, G * (k + m), B)
    rs.reed_solomon_release(h)
    out["quirk_seed"] = np.array([0xE0C0DEFF], dtype=np.uint64)
    out["quirk_matrix"] = pm.reshape(m, k)
    out["quirk_parity"] = par
    # survey KAT: data[i][b] = (8 i + b) & 255, B = 8
    for k, m in [(10, 3), (4, 2)]:
        B = 8
        data = np.array([[(8 * i + b) & 255 for b in range(B)] for i in range(k)], dtype=np.uint8)
        par = np.zeros((m, B), dtype=np.uint8)
        h = rs.reed_solomon_new(k, m)
        ptrs = (C.c_void_p * (k + m))(*([ptr(data, i * B) for i in range(k)] + [ptr(par, i * B) for i in range(m)]))
        rs.reed_solomon_encode(h, ptrs, k + m, B)
        rs.reed_solomon_release(h)
        fh = fec.fec_new(k, k + m)
        fpar = np.zeros((m, B), dtype=np.uint8)
        src = (C.c_void_p * k)(*[ptr(data, i * B) for i in range(k)])
        for j in range(m):
            fec.fec_encode(fh, src, C.c_void_p(ptr(fpar, j * B)), k + j, B)
        fec.fec_free(fh)
        out[f"kat_rs_{k}_{m}"] = par
        out[f"kat_fec_{k}_{m}"] = fpar
    np.savez_compressed(os.path.join(OUT, "encode.npz"), **out)


def rs_reconstruct_batch(rs, k, m, data, par, marks, B):
    """Run the reference reconstruct on a contiguous batch (modified in place)."""
    G = data.shape[0] // k
    n = k + m
    h = rs.reed_solomon_new(k, m)
    ptrs = (C.c_void_p * (G * n))(*([ptr(data, i * B) for i in range(G * k)] +
                                     [ptr(par, i * B) for i in range(G * m)]))
    rc = rs.reed_solomon_reconstruct(h, ptrs, C.c_void_p(ptr(marks)), G * n, B)
    rs.reed_solomon_release(h)
    return rc


def all_masks(n):
    return np.array([[(mask >> i) & 1 for i in range(n)] for mask in range(1 << n)], dtype=np.uint8)


def gen_reconstruct(rs):
    """rs.c reconstruct, exhaustive over every erasure mask for (4,2) and (10,3), sampled
    for (16,4).  Two payload kinds: 'cons' (parity = encode(data)) and 'incons' (random
    parity) -- the latter pins the survivor-selection rule (rs.c:620-629) bit for bit.
    Erased data buffers are pre-filled with 0x5A so an unwritten output shows."""
    out = {}
    cases = [(4, 2, 16, None), (10, 3, 8, None), (16, 4, 8, 2000), (2, 1, 5, None), (3, 2, 33, None)]
    for k, m, B, sample in cases:
        n = k + m
        if sample is None:
            gmarks = all_masks(n)
        else:
            gen = np.random.default_rng(0x5EED + k)
            gmarks = (gen.random((sample, n)) < 0.2).astype(np.uint8)
        G = gmarks.shape[0]
        seed = 0x7EC0 + 31 * k + m
        data0 = synth_bytes(seed, G * k * B).reshape(G * k, B)
        # consistent parity via the reference encoder
        par_c = np.zeros((G * m, B), dtype=np.uint8)
        h = rs.reed_solomon_new(k, m)
        ptrs = (C.c_void_p * (G * n))(*([ptr(data0, i * B) for i in range(G * k)] +
                                         [ptr(par_c, i * B) for i in range(G * m)]))
        rs.reed_solomon_encode(h, ptrs, G * n, B)
        rs.reed_solomon_release(h)
        par_i = synth_bytes(seed ^ 0xFFFF, G * m * B).reshape(G * m, B)
        marks = np.concatenate([gmarks[:, :k].reshape(-1), gmarks[:, k:].reshape(-1)]).astype(np.uint8)
        key = f"{k}_{m}_{B}"
        for kind, par in (("cons", par_c), ("incons", par_i)):
            d = data0.copy()
            d[marks[:G * k] == 1] = 0x5A
            p = par.copy()
            rc = rs_reconstruct_batch(rs, k, m, d, p, marks, B)
            assert np.array_equal(p, par)  # parity is never regenerated
            if kind == "cons":  # recovered == original where recoverable: a digest suffices
                out[f"{kind}_{key}"] = np.frombuffer(hashlib.sha256(d.tobytes()).digest(), dtype=np.uint8)
            else:
                out[f"{kind}_{key}"] = d
            out[f"rc_{kind}_{key}"] = np.array([rc], dtype=np.int32)
        out[f"seed_{key}"] = np.array([seed], dtype=np.uint64)
        out[f"marks_{key}"] = gmarks
        out[f"parc_{key}"] = np.frombuffer(hashlib.sha256(par_c.tobytes()).digest(), dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "reconstruct.npz"), **out)


def gen_reconstruct_large(rs):
    """rs.c reconstruct at the bench block sizes (B = 1024 / 1400), where the GPU's 8-, 12- and
    16-byte-lane bodies and the multi-wave-per-group split engage: sampled masks with 0..m+1
    erasures (so unrecoverable groups too), consistent and inconsistent parity, erased
    buffers pre-filled with 0x5A.  Stored as sha256 digests of the whole reconstructed data
    region plus rc (the fixtures stay small); tests regenerate inputs from the seeds."""
    out = {}
    cases = [(10, 3, 1024, 600), (16, 4, 1400, 400), (10, 3, 1400, 300), (4, 2, 1024, 300), (16, 4, 1024, 300),
             (12, 4, 1400, 200)]
    for k, m, B, sample in cases:
        n = k + m
        gen = np.random.default_rng(0xB16B + 13 * k + B)
        gmarks = np.zeros((sample, n), np.uint8)
        for g in range(sample):
            gmarks[g, gen.choice(n, size=int(gen.integers(0, m + 2)), replace=False)] = 1
        seed = 0x1A2E + 31 * k + m + B
        data0 = synth_bytes(seed, sample * k * B).reshape(sample * k, B)
        par_c = np.zeros((sample * m, B), dtype=np.uint8)
        h = rs.reed_solomon_new(k, m)
        ptrs = (C.c_void_p * (sample * n))(*([ptr(data0, i * B) for i in range(sample * k)] +
                                              [ptr(par_c, i * B) for i in range(sample * m)]))
        rs.reed_solomon_encode(h, ptrs, sample * n, B)
        rs.reed_solomon_release(h)
        par_i = synth_bytes(seed ^ 0xFFFF, sample * m * B).reshape(sample * m, B)
        marks = np.concatenate([gmarks[:, :k].reshape(-1), gmarks[:, k:].reshape(-1)]).astype(np.uint8)
        key = f"{k}_{m}_{B}"
        for kind, par in (("cons", par_c), ("incons", par_i)):
            d = data0.copy()
            d[marks[:sample * k] == 1] = 0x5A
            p = par.copy()
            rc = rs_reconstruct_batch(rs, k, m, d, p, marks, B)
            assert np.array_equal(p, par)
            out[f"{kind}_{key}"] = np.frombuffer(hashlib.sha256(d.tobytes()).digest(), dtype=np.uint8)
            out[f"rc_{kind}_{key}"] = np.array([rc], dtype=np.int32)
        out[f"seed_{key}"] = np.array([seed], dtype=np.uint64)
        out[f"marks_{key}"] = gmarks
    np.savez_compressed(os.path.join(OUT, "reconstruct_large.npz"), **out)


# reed_solomon handles whose public matrices the caller edits (rs.h:7-13 exposes both):
# encode reads rs->parity (rs.c:583), reconstruct builds its sub-matrix from rs->m, data rows
# included (rs.c:505, 536-548), and ignores invert_mat's failure (rs.c:556).
#   name: (k, m, B, groups or None = every mask, edits of parity, edits of m, stored in full?)
# an edit is (row, col, value); a row edit (row, None, values) replaces the whole row
RS_EDITS = {
    # (i) parity edited (a zero in column 0 among them): encode, then reconstruct from the
    # untouched m over the parity that encode produced
    "p42": (4, 2, 16, None, [(0, 0, 0), (1, 3, 0x77), (0, 2, 0x11)], [], True),
    # (ii) rows of m edited: a data row and a parity row (column 0 zeroed)
    "m42": (4, 2, 16, None, [], [(1, None, [3, 1, 0, 9]), (5, None, [0, 0xC4, 0x21, 0x90])], True),
    # (iii) singular sub-matrices: parity row 0 == data row 0, parity row 1 all zero
    "s42": (4, 2, 16, None, [], [(4, None, [1, 0, 0, 0]), (5, None, [0, 0, 0, 0])], True),
    "s103": (10, 3, 8, None, [(2, 0, 0)], [(4, None, list(range(1, 11))), (11, None, [0, 0, 0, 0, 0, 0, 0, 1, 0, 0]),
                                           (12, None, [0] * 10)], False),
    # bench block sizes, where the wide-lane kernel bodies run
    "m103w": (10, 3, 1024, 300, [], [(4, None, [7, 0, 3, 1, 0x99, 2, 5, 0, 1, 0xFE]), (11, 0, 0),
                                    (12, None, [0, 0, 0, 0, 0, 0, 0, 1, 0, 0])], False),
    "m164w": (16, 4, 1400, 200, [(3, 0, 0)], [(0, None, [(5 * i + 1) & 255 for i in range(16)]),
                                             (16, None, [(11 * i + 7) & 255 for i in range(16)]),
                                             (18, None, [0] * 16), (19, 0, 0)], False),
}


def _apply_edits(arr, k, edits):
    for r, c, v in edits:
        if c is None:
            for i, x in enumerate(v):
                arr[r * k + i] = x
        else:
            arr[r * k + c] = v


def gen_rs_edits(rs):
    """reed_solomon_encode / reconstruct on handles whose public `parity` / `m` were edited,
    including edits that make some erasure pattern's sub-matrix singular (rs.c then decodes
    with invert_mat's partial state and keeps err unchanged).  Erased data buffers are
    pre-filled with 0x5A; parity is random ('incons') unless the case encodes first."""
    out = {}
    for name, (k, m, B, sample, pedits, medits, store) in RS_EDITS.items():
        n = k + m
        if sample is None:
            gmarks = all_masks(n)
        else:
            gen = np.random.default_rng(0xED17 + 7 * k + B)
            gmarks = np.zeros((sample, n), np.uint8)
            for g in range(sample):
                gmarks[g, gen.choice(n, size=int(gen.integers(1, m + 2)), replace=False)] = 1
        G = gmarks.shape[0]
        seed = 0xED170000 + 131 * k + m + B
        data0 = synth_bytes(seed, G * k * B).reshape(G * k, B)
        h = rs.reed_solomon_new(k, m)
        _apply_edits(h.contents.parity, k, pedits)
        _apply_edits(h.contents.m, k, medits)
        pm = np.ctypeslib.as_array(h.contents.parity, shape=(m * k,)).copy().reshape(m, k)
        full = np.ctypeslib.as_array(h.contents.m, shape=(n * k,)).copy().reshape(n, k)
        if pedits:  # encode with the edited parity rows over 0x5A (stale bytes show)
            par = np.full((G * m, B), 0x5A, dtype=np.uint8)
            ptrs = (C.c_void_p * (G * n))(*([ptr(data0, i * B) for i in range(G * k)] +
                                             [ptr(par, i * B) for i in range(G * m)]))
            rs.reed_solomon_encode(h, ptrs, G * n, B)
            enc = par.copy()
        else:
            par = synth_bytes(seed ^ 0xFFFF, G * m * B).reshape(G * m, B)
            enc = None
        marks = np.concatenate([gmarks[:, :k].reshape(-1), gmarks[:, k:].reshape(-1)]).astype(np.uint8)
        d = data0.copy()
        d[marks[:G * k] == 1] = 0x5A
        p = par.copy()
        ptrs = (C.c_void_p * (G * n))(*([ptr(d, i * B) for i in range(G * k)] + [ptr(p, i * B) for i in range(G * m)]))
        rc = rs.reed_solomon_reconstruct(h, ptrs, C.c_void_p(ptr(marks)), G * n, B)
        rs.reed_solomon_release(h)
        assert np.array_equal(p, par)
        out[f"seed_{name}"] = np.array([seed], dtype=np.uint64)
        out[f"shape_{name}"] = np.array([k, m, B], dtype=np.int32)
        out[f"marks_{name}"] = gmarks
        out[f"parity_{name}"] = pm
        out[f"m_{name}"] = full
        out[f"rc_{name}"] = np.array([rc], dtype=np.int32)
        if enc is not None:  # whole for the small cases, else a digest (tests re-encode and compare)
            out[f"enc_{name}"] = enc if store else np.frombuffer(hashlib.sha256(enc.tobytes()).digest(), np.uint8)
        if store:
            out[f"out_{name}"] = d
        else:
            out[f"out_{name}"] = np.frombuffer(hashlib.sha256(d.tobytes()).digest(), dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "rs_edits.npz"), **out)


def gen_fec_decode(fec):
    """fec.c fec_decode on k received packets: NetFecCodec order (first k valid in group
    order), random arrival order (exercises shuffle, fec.c:738-771), and error cases
    (duplicate data index -> conflict, index >= n -> invalid)."""
    out = {}
    gen = np.random.default_rng(0xDEC0DE)
    cases = [(2, 4), (3, 5), (5, 8), (4, 6), (3, 4), (4, 5), (5, 6), (7, 8), (10, 13), (16, 20), (1, 3)]
    B = 32
    for k, n in cases:
        fh = fec.fec_new(k, n)
        full = np.ctypeslib.as_array(fh.contents.enc_matrix, shape=(n * k,)).copy().reshape(n, k)
        T = 24
        seed = 0xFEC0 + 97 * k + n
        data = synth_bytes(seed, T * k * B).reshape(T, k, B)
        par_rand = synth_bytes(seed ^ 0xABCD, T * (n - k) * B).reshape(T, n - k, B)
        idx_in, idx_out, pk_in, pk_out, rcs = [], [], [], [], []
        for t in range(T):
            # full packet set of this trial: data + (consistent for even t, random for odd t) parity
            pkts = np.zeros((n, B), dtype=np.uint8)
            pkts[:k] = data[t]
            if t % 2 == 0:
                src = (C.c_void_p * k)(*[ptr(data[t], i * B) for i in range(k)])
                for j in range(k, n):
                    fec.fec_encode(fh, src, C.c_void_p(ptr(pkts, j * B)), j, B)
            else:
                pkts[k:] = par_rand[t]
            mode = t % 4
            if mode in (0, 1):       # NetFecCodec order: first k valid in group order
                lost = gen.choice(n, size=min(n - k, gen.integers(0, n - k + 1)), replace=False)
                valid = [i for i in range(n) if i not in set(lost.tolist())][:k]
            elif mode == 2:          # arbitrary arrival order
                valid = gen.choice(n, size=k, replace=False).tolist()
            else:                    # error cases
                valid = list(range(k))
                if k >= 2 and t % 8 == 3:
                    valid[1] = valid[0]          # duplicate data index -> shuffle conflict
                else:
                    valid[-1] = n + 1            # invalid index -> build_decode_matrix fails
            idx = np.array(valid, dtype=np.int32)
            buf = np.zeros((k, B), dtype=np.uint8)
            for s, i in enumerate(valid):
                buf[s] = pkts[i] if 0 <= i < n else 0xEE
            bptrs = (C.c_void_p * k)(*[ptr(buf, s * B) for s in range(k)])
            ia = (C.c_int * k)(*idx.tolist())
            before = buf.copy()
            rc = fec.fec_decode(fh, bptrs, ia, B)
            # read back the (possibly permuted) pointer array: which original slot each now points to
            perm = [(bptrs[s] - ptr(buf)) // B for s in range(k)]
            after = np.stack([buf[p] for p in perm])
            idx_in.append(idx)
            idx_out.append(np.array(list(ia), dtype=np.int32))
            pk_in.append(before)
            pk_out.append(after)
            rcs.append(rc)
        fec.fec_free(fh)
        key = f"{k}_{n}"
        out[f"matrix_{key}"] = full
        out[f"idx_in_{key}"] = np.stack(idx_in)
        out[f"idx_out_{key}"] = np.stack(idx_out)
        out[f"pk_in_{key}"] = np.stack(pk_in)
        out[f"pk_out_{key}"] = np.stack(pk_out)
        out[f"rc_{key}"] = np.array(rcs, dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, "fec_decode.npz"), **out)


WIRE_CASES = [(4, 5), (4, 6), (3, 5), (5, 8), (7, 8), (10, 13), (2, 4), (3, 4), (14, 15), (1, 2)]


def gen_wire():
    """The FEC wire format, produced by the reference's own network/FecCodecBuf.cpp (built
    unchanged into oracle/_ref/libref_feccodec_ref.so with system/fec.c): full groups sent
    the way zfec_pack_input does (NetFecCodec.cpp:96-172), then every datagram -- and a
    corrupted copy -- parsed by unpack_fec_head, source shards by dec_src_pkt_info, and one
    lossy group decoded by fec_decode_pkts."""
    sys.path.insert(0, ROOT)
    from oracle.oracle import FecCodecBufS, FecCodecHead, load_callers
    L = load_callers(os.path.join(HERE, "_ref", "libref_feccodec_ref.so"))
    L.fec_new.restype = C.c_void_p
    L.fec_new.argtypes = [C.c_int, C.c_int]
    L.fec_free.argtypes = [C.c_void_p]
    out = {}
    gen = np.random.default_rng(0x31BE)
    for (k, n), checksum in itertools.product(WIRE_CASES, (1, 0)):
        G = 3
        S = FecCodecBufS()
        L.init_fec_buf(C.byref(S), 2048, 16)
        S.is_send_checksum = bool(checksum)
        codec = L.fec_new(k, n)
        sizes = gen.integers(0, 2049, size=G * k).astype(np.int32)
        if k > 1:
            sizes[0] = 0  # an empty payload
            sizes[1] = 2048  # the largest the default init allows
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
        payload = gen.integers(0, 256, size=int(sizes.sum()) + 1, dtype=np.uint8)
        sent0 = np.array([0xFFFFFFF0 + 0, 7, 123456], dtype=np.uint32)[:G]  # incl. u32 wrap
        src0 = np.array([0xFFFFFFFA, 5, 99999], dtype=np.uint32)[:G]
        pitch = 2048 + 4 + 13 + 3
        dgrams = np.zeros((G, n, pitch), dtype=np.uint8)
        dlen = np.zeros((G, n), dtype=np.int32)
        gmax = np.zeros(G, dtype=np.int32)
        for g in range(G):
            en = C.c_int()
            for ik in range(k):
                i = g * k + ik
                pl = payload[offs[i]:offs[i] + sizes[i]]
                pp = L.set_fec_enc_buf(C.byref(S), ik, C.c_void_p(pl.ctypes.data if sizes[i] else payload.ctypes.data),
                                       int(sizes[i]), C.byref(en))
                gmax[g] = en.value if ik == 0 else max(gmax[g], en.value)
                h = FecCodecHead(int(sent0[g]) + ik & 0xFFFFFFFF, int(src0[g]) + ik & 0xFFFFFFFF, n, k, ik)
                ol = C.c_int()
                q = L.pack_fec_head(C.byref(S), C.byref(h), pp, en.value, C.byref(ol))
                dgrams[g, ik, :ol.value] = np.frombuffer(C.string_at(q, ol.value), dtype=np.uint8)
                dlen[g, ik] = ol.value
            for ik in range(k, n):
                pp = L.get_fec_encoded_pkt(C.byref(S), codec, ik, int(gmax[g]), C.byref(en))
                h = FecCodecHead(int(sent0[g]) + ik & 0xFFFFFFFF, int(src0[g]) + k - 1 & 0xFFFFFFFF, n, k, ik)
                ol = C.c_int()
                q = L.pack_fec_head(C.byref(S), C.byref(h), pp, en.value, C.byref(ol))
                dgrams[g, ik, :ol.value] = np.frombuffer(C.string_at(q, ol.value), dtype=np.uint8)
                dlen[g, ik] = ol.value
        # receive side: parse every datagram and a corrupted copy of it
        R = FecCodecBufS()
        L.init_fec_buf(C.byref(R), 2048, 16)
        parsed = np.zeros((G, n, 2, 8), dtype=np.int64)  # ok, sent, src, n, k, ik, unpacked_len, is_checksum
        shards = np.zeros((G, n, pitch), dtype=np.uint8)
        srcinfo = np.full((G, k, 2), -1, dtype=np.int64)  # (payload offset in shard or -1, size)
        for g in range(G):
            for ik in range(n):
                for var in range(2):
                    d = dgrams[g, ik, :dlen[g, ik]].copy()
                    if var == 1 and dlen[g, ik] > 14:
                        d[14] ^= 0x40  # a payload byte: caught by the shard checksum when present
                    h = FecCodecHead()
                    un = C.c_int()
                    q = L.unpack_fec_head(C.byref(R), C.byref(h), C.c_void_p(d.ctypes.data), len(d), C.byref(un))
                    parsed[g, ik, var] = [1 if q else 0, h.sent_pkt_index, h.src_pkt_index, h.codec_n, h.codec_k, h.ik,
                                          un.value, int(R.is_checksum)]
                    if q and var == 0:
                        shards[g, ik, :un.value] = np.frombuffer(C.string_at(q, un.value), dtype=np.uint8)
                        if ik < k:
                            sz = C.c_uint16()
                            sp = L.dec_src_pkt_info(q, C.byref(R), C.byref(sz))
                            srcinfo[g, ik] = [(sp - q) if sp else -1, sz.value]
        L.fec_free(codec)
        L.release_fec_buf(C.byref(S))
        L.release_fec_buf(C.byref(R))
        key = f"{k}_{n}_{checksum}"
        out[f"sizes_{key}"] = sizes
        out[f"payload_{key}"] = payload
        out[f"seq_{key}"] = np.stack([sent0, src0], axis=1)
        out[f"dgrams_{key}"] = dgrams
        out[f"dlen_{key}"] = dlen
        out[f"gmax_{key}"] = gmax
        out[f"parsed_{key}"] = parsed
        out[f"shards_{key}"] = shards
        out[f"srcinfo_{key}"] = srcinfo
    np.savez_compressed(os.path.join(OUT, "wire.npz"), **out)


def main():
    """python oracle/gen_golden.py [name ...]  (default: every fixture file)"""
    os.makedirs(OUT, exist_ok=True)
    rs, fec = load_ref()
    gens = {"matrices": lambda: gen_matrices(rs, fec), "encode": lambda: gen_encode(rs, fec),
            "reconstruct": lambda: gen_reconstruct(rs), "reconstruct_large": lambda: gen_reconstruct_large(rs),
            "fec_decode": lambda: gen_fec_decode(fec), "wire": gen_wire, "rs_edits": lambda: gen_rs_edits(rs)}
    for name in (sys.argv[1:] or list(gens)):
        gens[name]()
    manifest = {
        "generator": "oracle/gen_golden.py",
        "reference": "skywind3000/QuickNet @ 2024-10-08, module/rs.c + system/fec.c compiled by oracle/Makefile",
        "files": sorted(f for f in os.listdir(OUT) if f.endswith(".npz")),
    }
    with open(os.path.join(OUT, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", manifest["files"])


if __name__ == "__main__":
    main()
