"""Edges of the reference's API surface on the GPU path: empty batches, one-byte shards, and
the largest shapes each codec admits (module/rs.c n <= 255, rs.h:5, rs.c:404; system/fec.c
n <= 256, fec.c:664) against the oracle (oracle/qfec_oracle.c, pinned by tests/golden) on the
reference's own matrices for those shapes (tests/golden/matrices.npz), including the batched
device reconstruct above the device LUT's reach (k + m > 24)."""
import numpy as np
import pytest
import torch

import quicknet_amd as qa
from quicknet_amd.synth import marks_to_rs_layout, synth_bytes

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
EDGE_RS = [(128, 127), (254, 1), (1, 254), (200, 55), (32, 8)]   # matrices.npz has each
EDGE_FEC = [(128, 256), (1, 256), (255, 256), (200, 255)]


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def test_empty_batches():
    """G = 0 everywhere is a no-op that succeeds (rs.c:581 and :616 loop zero times)."""
    code = qa.Code.cauchy(10, 3)
    d = torch.empty((0, 10, 1024), dtype=torch.uint8, device=DEV)
    p = torch.empty((0, 3, 1024), dtype=torch.uint8, device=DEV)
    code.encode(d, p)
    code.reconstruct(d, p, torch.empty(0, dtype=torch.uint8, device=DEV))
    rs = qa.ReedSolomon(10, 3)
    assert rs.encode(np.zeros((0, 10, 8), np.uint8), np.zeros((0, 3, 8), np.uint8), 8) == 0
    assert rs.reconstruct(np.zeros((0, 10, 8), np.uint8), np.zeros((0, 3, 8), np.uint8), np.zeros(0, np.uint8), 8) == 0
    big = qa.Code.cauchy(30, 10)  # host-record path with nothing to do
    big.reconstruct(torch.empty((0, 30, 64), dtype=torch.uint8, device=DEV),
                    torch.empty((0, 10, 64), dtype=torch.uint8, device=DEV),
                    torch.empty(0, dtype=torch.uint8, device=DEV))
    torch.cuda.synchronize()


def test_one_byte_shards_batched(oracle):
    """B = 1 through the batched API (byte-granular kernels: pitch 1 is not 16-B aligned)."""
    k, m, G = 10, 3, 257
    code = qa.Code.vandermonde(k, m)
    data = synth_bytes(11, G * k).reshape(G, k, 1)
    par = to_dev(np.zeros((G, m, 1), np.uint8))
    code.encode(to_dev(data), par, 1)
    ref = np.zeros((G, m, 1), np.uint8)
    oracle.fec_encode(code.rows, data, ref, 1)
    torch.cuda.synchronize()
    assert np.array_equal(par.cpu().numpy(), ref)


@pytest.mark.parametrize("k,m", EDGE_RS)
def test_rs_largest_shapes_vs_oracle(oracle, golden, k, m):
    """reed_solomon_* and the batched API at n = 255: encode, then reconstruct with random
    (inconsistent) parity and 0..m+1 erasures per group, erased buffers pre-filled 0x5A."""
    rows = golden("matrices.npz")[f"rs_{k}_{m}"]  # the reference's own matrix
    assert np.array_equal(oracle.cauchy(k, m), rows)
    G, B, pitch = 3, 37, 48
    data = synth_bytes(k * 3 + m, G * k * B).reshape(G, k, B)
    ref = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(rows, data, ref, B)
    rs = qa.ReedSolomon(k, m)
    par = np.zeros((G, m, B), np.uint8)
    assert rs.encode(data, par, B) == 0
    assert np.array_equal(par, ref)
    code = qa.Code.cauchy(k, m)
    ddat = np.zeros((G, k, pitch), np.uint8)
    ddat[..., :B] = data
    dpar = to_dev(np.zeros((G, m, pitch), np.uint8))
    code.encode(to_dev(ddat), dpar, B)
    torch.cuda.synchronize()
    assert np.array_equal(dpar.cpu().numpy()[..., :B], ref)

    rng = np.random.default_rng(k * 1000 + m)
    gm = np.zeros((G, k + m), np.uint8)
    for g in range(1, G):  # 0..m+1 erasures anywhere
        e = int(rng.integers(0, m + 2))
        gm[g, rng.choice(k + m, size=min(e, k + m), replace=False)] = 1
    gm[0, rng.choice(k, size=min(m, k), replace=False)] = 1  # group 0: data erasures only
    marks = marks_to_rs_layout(gm, k)
    rpar = synth_bytes(k + 5 * m, G * m * B).reshape(G, m, B)
    damaged = data.copy()
    damaged.reshape(G * k, B)[marks[: G * k] == 1] = 0x5A
    expect = damaged.copy()
    rc_ref = oracle.rs_reconstruct(rows, expect, rpar.copy(), marks, B)
    got = damaged.copy()
    assert rs.reconstruct(got, rpar.copy(), marks, B) == rc_ref
    assert np.array_equal(got, expect)
    dd = np.zeros((G, k, pitch), np.uint8)
    dd[..., :B] = damaged
    dd = to_dev(dd)
    dp = np.zeros((G, m, pitch), np.uint8)
    dp[..., :B] = rpar
    failed = torch.zeros(1, dtype=torch.int32, device=DEV)
    code.reconstruct(dd, to_dev(dp), to_dev(marks), B, failed)
    torch.cuda.synchronize()
    assert np.array_equal(dd.cpu().numpy()[..., :B], expect)
    under = int(((gm[:, :k].sum(1) > 0) & (gm.sum(1) > m)).sum())
    assert int(failed.item()) == under
    assert (under > 0) == (rc_ref == -1)


@pytest.mark.parametrize("k,n", EDGE_FEC)
def test_fec_largest_shapes_vs_oracle(oracle, golden, k, n):
    """fec_encode for copy / parity / out-of-range indices (fec.c:714-733: no write) and
    fec_decode of a random k-subset in arbitrary order (fec.c:821-862, the permuted pkt[] and
    index[] included) at n = 256."""
    full = golden("matrices.npz")[f"fec_{k}_{n}"]  # the reference's own n x k matrix
    sz = 33
    f = qa.FecParms(k, n)
    assert np.array_equal(f.matrix, full)
    src = synth_bytes(k + n, k * sz).reshape(k, sz)
    par = np.zeros((1, n - k, sz), np.uint8)
    oracle.fec_encode(full[k:], src[None], par, sz)
    for index in sorted({0, k - 1, k, (k + n) // 2, n - 1, n}):
        dst = np.full(sz, 0xA5, np.uint8)
        f.encode(src, dst, index, sz)
        want = src[index] if index < k else par[0, index - k] if index < n else np.full(sz, 0xA5, np.uint8)
        assert np.array_equal(dst, want), index
    idx = np.random.default_rng(n * 7 + k).choice(n, size=k, replace=False).astype(np.int32)
    pk = np.concatenate([src, par[0]], 0)[idx]
    rc, after, ia = f.decode(pk, idx, sz)
    rc_o, after_o, ia_o = oracle.fec_decode(k, n, full, pk, idx)
    assert rc == rc_o == 0
    assert np.array_equal(ia, ia_o)
    assert np.array_equal(after, after_o)
    assert np.array_equal(after, src)
