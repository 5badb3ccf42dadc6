"""GPU parity: the HIP path (libqfec.so kernels, called through the C ABI) against the golden
vectors the reference produced and against the CPU oracle.  Bit-exact (integer work).

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import hashlib
import itertools

import numpy as np
import pytest

import quicknet_amd as qa
from quicknet_amd.synth import erasure_marks, marks_to_rs_layout, synth_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")
ENC_CASES = [(2, 1), (4, 2), (10, 3), (16, 4), (7, 1), (3, 2)]
ENC_LENS = [1, 8, 1024, 1400, 37]


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def padded(a, pitch, fill=0):
    """[..., B] -> [..., pitch] with pad bytes = fill."""
    out = np.full(a.shape[:-1] + (pitch,), fill, dtype=np.uint8)
    out[..., : a.shape[-1]] = a
    return out


def round16(x):
    return (x + 15) // 16 * 16


@pytest.fixture(autouse=True)
def _variant_reset():
    qa.set_kernel_variant(qa._lib.QFEC_VARIANT_PERM)
    yield
    qa.set_kernel_variant(qa._lib.QFEC_VARIANT_PERM)


def test_synth_fill_matches_host():
    for n, seed in [(1, 3), (7, 5), (4096, 0x5EED0002), (100003, 9)]:
        t = torch.empty(n, dtype=torch.uint8, device=DEV)
        qa.synth_fill(t, seed)
        assert np.array_equal(t.cpu().numpy(), synth_bytes(seed, n))


@pytest.mark.parametrize("km,B", list(itertools.product(ENC_CASES, ENC_LENS)))
@pytest.mark.parametrize("variant", [0, 1])
def test_encode_batched_vs_golden(golden, km, B, variant):
    """qfec_encode on device buffers, fast (pitch = round16) and byte (pitch = B) paths."""
    qa.set_kernel_variant(variant)
    z = golden("encode.npz")
    k, m = km
    key = f"{k}_{m}_{B}"
    G = 4
    data = synth_bytes(int(z[f"seed_{key}"][0]), G * k * B).reshape(G, k, B)
    for pitch in sorted({round16(B), B}):
        for flavour, gold, ctor in (("rs", z[f"rs_{key}"], qa.Code.cauchy), ("fec", z[f"fec_{key}"], qa.Code.vandermonde)):
            code = ctor(k, m)
            d = to_dev(padded(data, pitch, 0xC3))
            p = to_dev(np.full((G, m, pitch), 0x5A, np.uint8))
            code.encode(d, p, B)
            torch.cuda.synchronize()
            got = p.cpu().numpy()[..., :B].reshape(G * m, B)
            assert np.array_equal(got, gold), (flavour, pitch)


@pytest.mark.parametrize("km,B", list(itertools.product(ENC_CASES, [8, 1400])))
def test_encode_abi_vs_golden(golden, km, B):
    """reed_solomon_encode (host pointer arrays) and per-packet fec_encode."""
    z = golden("encode.npz")
    k, m = km
    key = f"{k}_{m}_{B}"
    G = 4
    data = synth_bytes(int(z[f"seed_{key}"][0]), G * k * B).reshape(G, k, B)
    rs = qa.ReedSolomon(k, m)
    par = np.full((G, m, B), 0x5A, np.uint8)
    assert rs.encode(data, par, B) == 0
    assert np.array_equal(par.reshape(G * m, B), z[f"rs_{key}"])
    f = qa.FecParms(k, k + m)
    fpar = np.full((G, m, B), 0xA5, np.uint8)
    for g in range(G):
        for j in range(m):
            f.encode(list(data[g]), fpar[g, j], k + j, B)
    assert np.array_equal(fpar.reshape(G * m, B), z[f"fec_{key}"])
    cp = np.zeros(B, np.uint8)
    f.encode(list(data[0]), cp, k - 1, B)
    assert np.array_equal(cp, z[f"fcopy_{key}"])
    bad = np.full(B, 0x33, np.uint8)
    f.encode(list(data[0]), bad, k + m, B)
    assert np.array_equal(bad, z[f"fbad_{key}"])


def test_encode_rs_quirk(golden):
    """A zero in column 0 of the public parity matrix leaves dst stale (rs.c:116-117)."""
    z = golden("encode.npz")
    k, m, B, G = 4, 2, 16, 2
    data = synth_bytes(int(z["quirk_seed"][0]), G * k * B).reshape(G, k, B)
    rs = qa.ReedSolomon(k, m)
    rs.parity[:] = z["quirk_matrix"]
    par = np.full((G, m, B), 0x5A, np.uint8)
    rs.encode(data, par, B)
    assert np.array_equal(par.reshape(G * m, B), z["quirk_parity"])
    # same through the batched API with the quirk flag
    code = qa.Code.from_rows(z["quirk_matrix"], rs_stale_quirk=True)
    d = to_dev(data)
    p = to_dev(np.full((G, m, B), 0x5A, np.uint8))
    code.encode(d, p, B)
    torch.cuda.synchronize()
    assert np.array_equal(p.cpu().numpy().reshape(G * m, B), z["quirk_parity"])


RECON = [(4, 2, 16), (10, 3, 8), (16, 4, 8), (2, 1, 5), (3, 2, 33)]


@pytest.mark.parametrize("k,m,B", RECON)
@pytest.mark.parametrize("path", ["device", "abi"])
def test_reconstruct_vs_golden(golden, oracle, k, m, B, path):
    z = golden("reconstruct.npz")
    key = f"{k}_{m}_{B}"
    gm = z[f"marks_{key}"]
    G = gm.shape[0]
    seed = int(z[f"seed_{key}"][0])
    data0 = synth_bytes(seed, G * k * B).reshape(G, k, B)
    par_c = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(oracle.cauchy(k, m), data0, par_c, B)
    par_i = synth_bytes(seed ^ 0xFFFF, G * m * B).reshape(G, m, B)
    marks = marks_to_rs_layout(gm, k)
    for kind, par in (("cons", par_c), ("incons", par_i)):
        d = data0.copy()
        d.reshape(G * k, B)[marks[: G * k] == 1] = 0x5A
        if path == "abi":
            rs = qa.ReedSolomon(k, m)
            rc = rs.reconstruct(d, par.copy(), marks, B)
            assert rc == z[f"rc_{kind}_{key}"][0]
            out = d
        else:
            code = qa.Code.cauchy(k, m)
            pitch = round16(B)
            dd = to_dev(padded(d, pitch))
            pp = to_dev(padded(par, pitch))
            failed = torch.zeros(1, dtype=torch.int32, device=DEV)
            code.reconstruct(dd, pp, to_dev(marks), B, failed)
            torch.cuda.synchronize()
            out = dd.cpu().numpy()[..., :B]
            nfail = int(failed.item())
            assert (nfail > 0) == (z[f"rc_{kind}_{key}"][0] == -1)
        if kind == "cons":
            assert hashlib.sha256(np.ascontiguousarray(out).tobytes()).digest() == z[f"cons_{key}"].tobytes()
        else:
            assert np.array_equal(out.reshape(G * k, B), z[f"incons_{key}"])


RECON_LARGE = [(10, 3, 1024), (16, 4, 1400), (10, 3, 1400), (4, 2, 1024), (16, 4, 1024), (12, 4, 1400)]


@pytest.mark.parametrize("impl", [-1, 2, 3, 4, 8, "abi"])
@pytest.mark.parametrize("k,m,B", RECON_LARGE)
def test_reconstruct_large_vs_golden(golden, oracle, k, m, B, impl):
    """Every reconstruct body (-1 auto; exact-e rows on 2 16-, 3 8- and 4 12-B lanes, 8 the 8-B
    body one group per block) and the reed_solomon_reconstruct ABI against bytes the reference's own rs.c
    produced at the bench block sizes (digests in reconstruct_large.npz): the wide-lane bodies
    and the multi-wave-per-group split are pinned to the reference directly."""
    from test_oracle_golden import large_case
    z = golden("reconstruct_large.npz")
    key, gm, data0, par_i, marks = large_case(z, k, m, B)
    G = gm.shape[0]
    par_c = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(oracle.cauchy(k, m), data0, par_c, B)
    for kind, par in (("cons", par_c), ("incons", par_i)):
        d = data0.copy()
        d.reshape(G * k, B)[marks[: G * k] == 1] = 0x5A
        if impl == "abi":
            rc = qa.ReedSolomon(k, m).reconstruct(d, par.copy(), marks, B)
            assert rc == z[f"rc_{kind}_{key}"][0]
            out = d
        else:
            pitch = round16(B)
            dd = to_dev(padded(d, pitch))
            failed = torch.zeros(1, dtype=torch.int32, device=DEV)
            qa.tune("recon_impl", impl)
            try:
                qa.Code.cauchy(k, m).reconstruct(dd, to_dev(padded(par, pitch)), to_dev(marks), B, failed)
                torch.cuda.synchronize()
            finally:
                qa.tune("recon_impl", -1)
            out = dd.cpu().numpy()[..., :B]
            assert (int(failed.item()) > 0) == (z[f"rc_{kind}_{key}"][0] == -1)
        assert hashlib.sha256(np.ascontiguousarray(out).tobytes()).digest() == z[f"{kind}_{key}"].tobytes()


FEC_DEC = [(2, 4), (3, 5), (5, 8), (4, 6), (3, 4), (4, 5), (5, 6), (7, 8), (10, 13), (16, 20), (1, 3)]


@pytest.mark.parametrize("k,n", FEC_DEC)
def test_fec_decode_vs_golden(golden, k, n):
    z = golden("fec_decode.npz")
    key = f"{k}_{n}"
    f = qa.FecParms(k, n)
    assert np.array_equal(f.matrix, z[f"matrix_{key}"])
    B = z[f"pk_in_{key}"].shape[2]
    for t in range(z[f"rc_{key}"].shape[0]):
        rc, after, idx = f.decode(z[f"pk_in_{key}"][t], z[f"idx_in_{key}"][t], B)
        assert rc == z[f"rc_{key}"][t]
        assert np.array_equal(idx, z[f"idx_out_{key}"][t])
        assert np.array_equal(after, z[f"pk_out_{key}"][t])


@pytest.mark.parametrize("flavour", ["cauchy", "vandermonde"])
@pytest.mark.parametrize("k,m,B", [(5, 2, 1024), (32, 8, 256), (20, 4, 1400), (9, 5, 100), (12, 4, 1024)])
def test_generic_shapes_vs_oracle(oracle, flavour, k, m, B):
    """Shapes without a templated kernel ((5,2), (9,5): runtime k, m loops), n > 24 ((32,8): host
    decode records) and templated shapes through the same calls."""
    G = 33
    code = getattr(qa.Code, flavour)(k, m)
    rows = code.rows
    data = synth_bytes(k * 1000 + m, G * k * B).reshape(G, k, B)
    pitch = round16(B)
    d = to_dev(padded(data, pitch))
    p = to_dev(np.zeros((G, m, pitch), np.uint8))
    code.encode(d, p, B)
    torch.cuda.synchronize()
    ref = np.zeros((G, m, B), np.uint8)
    (oracle.rs_encode if flavour == "cauchy" else oracle.fec_encode)(rows, data, ref, B)
    assert np.array_equal(p.cpu().numpy()[..., :B], ref)
    # reconstruct: random erasures incl. unrecoverable ones; random (inconsistent) parity
    par = synth_bytes(77 + k, G * m * B).reshape(G, m, B)
    gm = (np.random.default_rng(k).random((G, k + m)) < 0.2).astype(np.uint8)
    marks = marks_to_rs_layout(gm, k)
    d0 = data.copy()
    rc_ref = oracle.rs_reconstruct(rows, d0, par.copy(), marks, B)
    rs_path = qa.ReedSolomon(k, m) if flavour == "cauchy" and k + m <= 255 else None
    if rs_path is not None:
        d1 = data.copy()
        rs_path.reconstruct(d1, par.copy(), marks, B)  # explicit (host-record) path
        assert np.array_equal(d1, d0)
    # batched device API: LUT path for k + m <= 24, host-record path above
    dd = to_dev(padded(data, pitch))
    failed = torch.zeros(1, dtype=torch.int32, device=DEV)
    code.reconstruct(dd, to_dev(padded(par, pitch)), to_dev(marks), B, failed)
    torch.cuda.synchronize()
    assert np.array_equal(dd.cpu().numpy()[..., :B], d0)
    assert (int(failed.item()) > 0) == (rc_ref == -1)
    assert rc_ref in (0, -1)


@pytest.mark.parametrize("impl", [-1, 2, 3, 4, 8])
@pytest.mark.parametrize("k,m,B", [(10, 3, 1024), (16, 4, 1400), (4, 2, 100), (12, 4, 40), (3, 2, 1400),
                                   (10, 3, 1400), (4, 2, 1012), (16, 4, 1024), (12, 4, 1400), (8, 4, 1024),
                                   (5, 3, 1024), (6, 2, 1400), (7, 1, 1024), (8, 2, 200), (20, 4, 1400), (20, 4, 100)])
def test_reconstruct_impls_vs_oracle(oracle, impl, k, m, B):
    """Every LUT reconstruct body (-1 = the auto choice; exact-e rows on 16-B, 8-B and 12-B
    lanes, the 8-B body one group per block), the coefficient tables read from the 256-entry
    table at the record's offsets, against the oracle's rs.c
    restatement, on random erasure patterns (0..m+1 erasures, so unrecoverable groups too)
    with random, inconsistent parity: the survivor rule and the stale-row quirk have to match
    byte for byte.  Bytes past the 16-B span of a row (the pitch's padding) stay untouched."""
    G = 700
    code = qa.Code.cauchy(k, m)
    rng = np.random.default_rng(k * 100 + B)
    data = synth_bytes(k * 7 + B, G * k * B).reshape(G, k, B)
    par = synth_bytes(k * 11 + B, G * m * B).reshape(G, m, B)
    gm = np.zeros((G, k + m), np.uint8)
    for g in range(G):
        gm[g, rng.choice(k + m, size=int(rng.integers(0, m + 2)), replace=False)] = 1
    marks = marks_to_rs_layout(gm, k)
    expect = data.copy()
    expect.reshape(G * k, B)[marks[: G * k] == 1] = 0x5A
    damaged = expect.copy()
    oracle.rs_reconstruct(code.rows, expect, par.copy(), marks, B)
    pitch = round16(B) + 16  # one spare 16-B column per row that no body may write
    dd = to_dev(padded(damaged, pitch))
    failed = torch.zeros(1, dtype=torch.int32, device=DEV)
    qa.tune("recon_impl", impl)
    try:
        code.reconstruct(dd, to_dev(padded(par, pitch)), to_dev(marks), B, failed)
        torch.cuda.synchronize()
    finally:
        qa.tune("recon_impl", -1)
    out = dd.cpu().numpy()
    assert np.array_equal(out[..., :B], expect)
    assert np.array_equal(out[..., round16(B):], padded(damaged, pitch)[..., round16(B):])
    unrecoverable = int(((gm[:, :k].sum(1) > 0) & (gm.sum(1) > m)).sum())
    assert int(failed.item()) == unrecoverable


@pytest.mark.parametrize("lds", [0, 20480])
@pytest.mark.parametrize("k,m,B", [(10, 3, 1024), (16, 4, 1400), (10, 3, 1400)])
def test_probe_reconstruct_writes_only_erased_rows(k, m, B, lds):
    """qfec_probe_reconstruct (the reconstruct's memory skeleton, calibration only) writes the
    erased data rows of recoverable groups and nothing else; other shapes are refused."""
    G = 1000
    pitch = round16(B)
    rng = np.random.default_rng(B + k)
    gm = np.zeros((G, k + m), np.uint8)
    for g in range(G):
        gm[g, rng.choice(k + m, size=int(rng.integers(0, m + 2)), replace=False)] = 1
    marks = marks_to_rs_layout(gm, k)
    data = synth_bytes(B * 3 + k, G * k * pitch).reshape(G, k, pitch)
    dd = to_dev(data)
    qa.probe_reconstruct(dd, to_dev(np.zeros((G, m, pitch), np.uint8)), to_dev(marks), B, lds)
    torch.cuda.synchronize()
    out = dd.cpu().numpy()
    written = np.zeros((G, k), bool)
    ok = (gm[:, :k].sum(1) > 0) & (gm.sum(1) <= m)
    written[ok] = gm[ok, :k] == 1
    assert np.array_equal(out[~written], data[~written])
    with pytest.raises(qa.QfecError):
        qa.probe_reconstruct(to_dev(np.zeros((4, 4, 64), np.uint8)), to_dev(np.zeros((4, 2, 64), np.uint8)),
                             to_dev(np.zeros(24, np.uint8)), 64)


@pytest.mark.parametrize("block", [-1, 64])
@pytest.mark.parametrize("impl", [-1, 0, 2])
@pytest.mark.parametrize("flavour", ["cauchy", "vandermonde"])
@pytest.mark.parametrize("k,m,B,G", [(10, 3, 1024, 300), (16, 4, 1400, 300), (10, 3, 100, 300), (16, 4, 8, 300),
                                     (8, 2, 1400, 7), (6, 2, 1008, 13), (10, 3, 1400, 1)])
def test_encode_impls_vs_oracle(oracle, block, impl, flavour, k, m, B, G):
    """The encode bodies (-1 auto, 0 all rows at once, 2 all rows with the inputs
    loaded in halves) against the oracle's restatement of rs.c's code_some_shards on random
    groups (the rs.c quirk included: parity pre-filled with 0x5A), on the auto blocks and forced
    onto one-wave blocks (tuning "encode_block" 64), group counts that leave the last block part
    empty and lanes that straddle groups (B = 1400: 88 columns)."""
    code = qa.Code.cauchy(k, m) if flavour == "cauchy" else qa.Code.vandermonde(k, m)
    data = synth_bytes(k * 13 + B, G * k * B).reshape(G, k, B)
    expect = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(code.rows, data, expect, B)
    pitch = round16(B)
    p = to_dev(np.full((G, m, pitch), 0x5A, np.uint8))
    qa.tune("encode_impl", impl)
    qa.tune("encode_block", block)
    try:
        code.encode(to_dev(padded(data, pitch, 0xC3)), p, B)
        torch.cuda.synchronize()
    finally:
        qa.tune("encode_impl", -1)
        qa.tune("encode_block", -1)
    assert np.array_equal(p.cpu().numpy()[..., :B], expect)


_RESID_EXPECT = {}


@pytest.mark.parametrize("block", [-1, 64, 256])
@pytest.mark.parametrize("lds", [-1, 0, 16384, 40960, 65536, 163840])
@pytest.mark.parametrize("k,m,B,G", [(10, 3, 1024, 70000), (16, 4, 1400, 24000), (16, 4, 1024, 33000),
                                     (4, 2, 1024, 33000), (3, 2, 512, 66000), (8, 2, 1024, 40000),
                                     (6, 2, 1400, 40000)])
def test_encode_residency_caps_vs_oracle(oracle, block, lds, k, m, B, G):
    """The encode's residency cap (tuning "encode_lds": -1 auto, 0 none, else LDS bytes per block)
    and block size (tuning "encode_block": -1 auto -- one-wave blocks for k = 10 --, 64, 256)
    change only how many waves share a CU: outputs equal the oracle's at every setting, on
    launches large enough (>= 8 192 blocks) for the auto rule to apply (RS(10,3) at 100 000 groups
    is test_large_batch_roundtrip)."""
    assert G * round16(B) // 16 >= 8192 * 256
    code = qa.Code.cauchy(k, m)
    key = (k, m, B, G)
    if key not in _RESID_EXPECT:
        data = synth_bytes(k * 41 + B, G * k * B).reshape(G, k, B)
        expect = np.zeros((G, m, B), np.uint8)
        oracle.rs_encode(code.rows, data, expect, B)
        _RESID_EXPECT.clear()
        _RESID_EXPECT[key] = (to_dev(padded(data, round16(B), 0xC3)), expect)
    d, expect = _RESID_EXPECT[key]
    p = torch.full((G, m, round16(B)), 0x5A, dtype=torch.uint8, device=DEV)
    qa.tune("encode_lds", lds)
    qa.tune("encode_block", block)
    try:
        code.encode(d, p, B)
        torch.cuda.synchronize()
    finally:
        qa.tune("encode_lds", -1)
        qa.tune("encode_block", -1)
    assert np.array_equal(p.cpu().numpy()[..., :B], expect)


@pytest.mark.parametrize("pinned,zero_copy", [(False, 1), (True, 1), (True, 0)])
@pytest.mark.parametrize("k,m,B,chunk", [(10, 3, 1024, 7), (16, 4, 1400, 0), (4, 2, 37, 5)])
def test_encode_host_vs_oracle(oracle, k, m, B, chunk, pinned, zero_copy):
    """qfec_encode_host (host in, host out) against the oracle: pageable numpy buffers through
    pinned staging chunked over two streams (chunk = groups per chunk, 0: the ~32 MiB
    default), pinned torch tensors read and written by the kernel directly (zero copy), or
    pinned through the staged path."""
    G = 101
    code = qa.Code.cauchy(k, m)
    pitch = B if B % 16 else round16(B)
    data = synth_bytes(k * 31 + B, G * k * B).reshape(G, k, B)
    expect = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(code.rows, data, expect, B)
    hd = padded(data, pitch, 0xC3)
    if pinned:
        hd = torch.from_numpy(hd).pin_memory()
        hp = torch.full((G, m, pitch), 0x5A, dtype=torch.uint8).pin_memory()
    else:
        hp = np.full((G, m, pitch), 0x5A, np.uint8)
    qa.tune("host_chunk", chunk)
    qa.tune("host_zero_copy", zero_copy)
    try:
        code.encode_host(hd, hp, B)
    finally:
        qa.tune("host_chunk", 0)
        qa.tune("host_zero_copy", 1)
    got = hp.numpy() if pinned else hp
    assert np.array_equal(got[..., :B], expect)


@pytest.mark.parametrize("pinned,zero_copy", [(False, 1), (True, 1), (True, 0)])
@pytest.mark.parametrize("k,m,B,chunk", [(10, 3, 1024, 7), (16, 4, 1400, 0), (4, 2, 37, 5)])
def test_reconstruct_host_vs_oracle(oracle, k, m, B, chunk, pinned, zero_copy):
    """qfec_reconstruct_host against the oracle's rs.c restatement on random patterns with
    inconsistent parity, incl. unrecoverable groups: pageable buffers staged in chunks over two
    streams, pinned ones read and written by the kernel in place (zero copy: only the erased
    rows are written back), or pinned through the staged path."""
    G = 211
    code = qa.Code.cauchy(k, m)
    pitch = B if B % 16 else round16(B)
    rng = np.random.default_rng(k * 7 + B)
    data = synth_bytes(k * 17 + B, G * k * B).reshape(G, k, B)
    par = synth_bytes(k * 19 + B, G * m * B).reshape(G, m, B)
    gm = np.zeros((G, k + m), np.uint8)
    for g in range(G):
        gm[g, rng.choice(k + m, size=int(rng.integers(0, m + 2)), replace=False)] = 1
    marks = marks_to_rs_layout(gm, k)
    expect = data.copy()
    expect.reshape(G * k, B)[marks[: G * k] == 1] = 0x5A
    work = padded(expect, pitch, 0xC3)
    hpar = padded(par, pitch)
    if pinned:
        work, hpar = torch.from_numpy(work).pin_memory(), torch.from_numpy(hpar).pin_memory()
    oracle.rs_reconstruct(code.rows, expect, par.copy(), marks, B)
    qa.tune("host_chunk", chunk)
    qa.tune("host_zero_copy", zero_copy)
    try:
        nf = code.reconstruct_host(work, hpar, np.ascontiguousarray(marks), B)
    finally:
        qa.tune("host_chunk", 0)
        qa.tune("host_zero_copy", 1)
    if pinned:
        work = work.numpy()
    assert np.array_equal(work[..., :B], expect)
    assert nf == int(((gm[:, :k].sum(1) > 0) & (gm.sum(1) > m)).sum())


def test_large_batch_roundtrip(oracle):
    """BASELINE config 2/3 shape at full size: 100 000 groups x RS(10,3) x 1 KiB.
    Encode checked byte for byte against the oracle; reconstruct with 3 random erasures
    per group must return the original data (a size-independent property)."""
    k, m, B, G = 10, 3, 1024, 100_000
    code = qa.Code.cauchy(k, m)
    data = torch.empty((G, k, B), dtype=torch.uint8, device=DEV)
    qa.synth_fill(data, 0x5EED0002)
    par = torch.empty((G, m, B), dtype=torch.uint8, device=DEV)
    code.encode(data, par)
    torch.cuda.synchronize()
    h_data = data.cpu().numpy()
    ref = np.zeros((G, m, B), np.uint8)
    oracle.rs_encode(code.rows, h_data, ref, B)
    assert np.array_equal(par.cpu().numpy(), ref)
    gm = erasure_marks(0x5EED0003, G, k + m, 3)
    marks = to_dev(marks_to_rs_layout(gm, k))
    damaged = data.clone()
    lost = torch.from_numpy(gm[:, :k].astype(bool)).to(DEV)
    damaged[lost] = 0x5A
    failed = torch.zeros(1, dtype=torch.int32, device=DEV)
    code.reconstruct(damaged, par, marks, B, failed)
    torch.cuda.synchronize()
    assert int(failed.item()) == 0
    assert torch.equal(damaged, data)


def test_ldslog_variant_matches_perm():
    k, m, B, G = 10, 3, 1024, 2000
    code = qa.Code.vandermonde(k, m)
    data = torch.empty((G, k, B), dtype=torch.uint8, device=DEV)
    qa.synth_fill(data, 1234)
    p0 = torch.empty((G, m, B), dtype=torch.uint8, device=DEV)
    p1 = torch.empty_like(p0)
    code.encode(data, p0)
    qa.set_kernel_variant(qa._lib.QFEC_VARIANT_LDSLOG)
    code.encode(data, p1)
    torch.cuda.synchronize()
    assert torch.equal(p0, p1)


def test_device_pointer_abi_paths():
    """The per-call ABIs accept device pointers too (contiguous and gathered)."""
    import ctypes as C
    k, m, B, G = 4, 2, 64, 8
    rs = qa.ReedSolomon(k, m)
    data = torch.empty((G, k, B), dtype=torch.uint8, device=DEV)
    qa.synth_fill(data, 99)
    par = torch.zeros((G, m, B), dtype=torch.uint8, device=DEV)
    L = qa.lib()
    db, pb = data.data_ptr(), par.data_ptr()
    ptrs = (C.c_void_p * (G * (k + m)))(*([db + i * B for i in range(G * k)] + [pb + i * B for i in range(G * m)]))
    assert L.reed_solomon_encode(rs._h, ptrs, G * (k + m), B) == 0
    torch.cuda.synchronize()
    ref = np.zeros((G, m, B), np.uint8)
    hd = data.cpu().numpy()
    qa.ReedSolomon(k, m).encode(hd, ref, B)
    assert np.array_equal(par.cpu().numpy(), ref)


@pytest.mark.parametrize("path", ["abi", "abi_dev", "batched"])
@pytest.mark.parametrize("name", ["p42", "m42", "s42", "s103", "m103w", "m164w"])
def test_rs_edits_vs_golden(golden, name, path):
    """reed_solomon handles whose public matrices the caller edited, byte for byte and return
    code for return code against what the reference's rs.c produced (rs_edits.npz): encode
    reads `parity`, reconstruct decodes from `m` (data rows included) and, where an edit made a
    pattern's sub-matrix singular, with invert_mat's partial state and err unchanged
    (rs.c:505-556).  Paths: the ABI on host pointers, the ABI on device pointers, and the
    batched device API on the handle's code (qfec_rs_code)."""
    import ctypes as C
    from test_oracle_golden import rs_edit_case, rs_edit_match
    z = golden("rs_edits.npz")
    k, m, B, G, data0, par, marks = rs_edit_case(z, name)
    n = k + m
    rs = qa.ReedSolomon(k, m)
    rs.parity[:] = z[f"parity_{name}"]
    rs.m_matrix[:] = z[f"m_{name}"]
    L = qa.lib()
    enc = par is None
    d = data0.copy()
    d.reshape(G * k, B)[marks[: G * k] == 1] = 0x5A
    if path == "abi":
        if enc:
            par = np.full((G, m, B), 0x5A, np.uint8)
            assert rs.encode(data0, par, B) == 0
            assert rs_edit_match(z, f"enc_{name}", par)
        rc = rs.reconstruct(d, par.copy(), marks, B)
        out = d
    elif path == "abi_dev":
        dd, dp = to_dev(data0.copy()), to_dev(par if not enc else np.full((G, m, B), 0x5A, np.uint8))
        ptrs = (C.c_void_p * (G * n))(*([dd.data_ptr() + i * B for i in range(G * k)] +
                                         [dp.data_ptr() + i * B for i in range(G * m)]))
        if enc:
            assert L.reed_solomon_encode(rs._h, ptrs, G * n, B) == 0
            torch.cuda.synchronize()
            assert rs_edit_match(z, f"enc_{name}", dp.cpu().numpy())
        dd.copy_(to_dev(d))
        dmarks = to_dev(marks)
        rc = L.reed_solomon_reconstruct(rs._h, ptrs, C.c_void_p(dmarks.data_ptr()), G * n, B)
        torch.cuda.synchronize()
        out = dd.cpu().numpy()
    else:
        code = rs.code()
        pitch = round16(B)
        if enc:
            dp = to_dev(np.full((G, m, pitch), 0x5A, np.uint8))
            code.encode(to_dev(padded(data0, pitch)), dp, B)
            torch.cuda.synchronize()
            par = np.ascontiguousarray(dp.cpu().numpy()[..., :B])
            assert rs_edit_match(z, f"enc_{name}", par)
        dd = to_dev(padded(d, pitch))
        failed = torch.zeros(1, dtype=torch.int32, device=DEV)
        code.reconstruct(dd, to_dev(padded(par, pitch)), to_dev(marks), B, failed)
        torch.cuda.synchronize()
        out = dd.cpu().numpy()[..., :B]
        rc = -1 if int(failed.item()) else 0
    assert rc == z[f"rc_{name}"][0]
    assert rs_edit_match(z, f"out_{name}", out)
    rs.close()


@pytest.mark.parametrize("k,m,B,G", [(10, 3, 1024, 5000), (16, 4, 1400, 2000), (4, 2, 1024, 5000), (12, 4, 333, 3000)])
def test_batched_vs_reference_rs_live(k, m, B, G):
    """The batched device path (qfec_encode / qfec_reconstruct on HBM-resident batches, the
    kernels the bench times) against the reference's own module/rs.c (oracle/_ref/libref_rs.so)
    on the same bytes: encode, then reconstruct with 0..m+1 erasures per group (unrecoverable
    groups included) over inconsistent parity -- every byte and the failed-group count equal."""
    import ctypes as C
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle.oracle import RefCodec
    if not RefCodec.available():
        pytest.skip("reference libraries not built (make -C oracle ref)")
    ref = RefCodec()
    n = k + m
    rng = np.random.default_rng(k * 31 + B)
    data = synth_bytes(0xA5A5 + k + B, G * k * B).reshape(G, k, B)
    code = qa.Code.cauchy(k, m)
    dd, pd = to_dev(data), torch.zeros((G, m, B), dtype=torch.uint8, device=DEV)
    code.encode(dd, pd, B)
    torch.cuda.synchronize()
    par_ref = np.zeros((G, m, B), np.uint8)
    h = ref.rs.reed_solomon_new(k, m)
    try:
        rdata = data.copy()
        assert ref.rs_encode(h, ref.shard_ptrs(rdata, par_ref), G * n, B) == 0
        assert np.array_equal(pd.cpu().numpy(), par_ref)
        gm = np.zeros((G, n), np.uint8)
        for g in range(G):
            gm[g, rng.choice(n, size=int(rng.integers(0, m + 2)), replace=False)] = 1
        marks = marks_to_rs_layout(gm, k)
        damaged = data.copy()
        damaged.reshape(G * k, B)[marks[:G * k] == 1] = 0x5A
        par_in = synth_bytes(0x77 + B, G * m * B).reshape(G, m, B)  # inconsistent parity: pins the survivor rule
        ddev = to_dev(damaged)
        failed = torch.zeros(1, dtype=torch.int32, device=DEV)
        code.reconstruct(ddev, to_dev(par_in), to_dev(marks), B, failed)
        torch.cuda.synchronize()
        rd, rp = damaged.copy(), par_in.copy()
        rc = ref.rs_reconstruct(h, ref.shard_ptrs(rd, rp), marks, G * n, B)
        assert np.array_equal(ddev.cpu().numpy(), rd)
        unrecoverable = int(((gm[:, :k].sum(1) > 0) & (gm.sum(1) > m)).sum())
        assert int(failed.item()) == unrecoverable
        assert rc == (-1 if unrecoverable else 0)
    finally:
        ref.rs.reed_solomon_release(h)
