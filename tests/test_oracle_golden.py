"""Pin the CPU restatement (oracle/liboracle.so) against the golden vectors that the
reference itself produced (oracle/gen_golden.py over oracle/_ref/).  CPU only."""
import hashlib
import itertools

import numpy as np
import pytest

from quicknet_amd.synth import synth_bytes

ENC_CASES = [(2, 1), (4, 2), (10, 3), (16, 4), (7, 1), (3, 2)]
ENC_LENS = [1, 8, 1024, 1400, 37]


def test_field_tables(oracle):
    # test_gf() (module/fec.c:866-888): exp/log round trip, inverses, zero row/column
    L = oracle.L
    for i in range(1, 256):  # log(0) is the sentinel 255 (fec.c:302)
        assert L.orc_exp(L.orc_log(i)) == i
        if i:
            assert oracle.mul(i, oracle.L.orc_inv(i)) == 1
        assert oracle.mul(0, i) == 0 and oracle.mul(i, 0) == 0
    assert L.orc_log(0) == 255


def test_matrices(oracle, golden):
    z = golden("matrices.npz")
    for key in z.files:
        if key.startswith("rs_") and key != "rs_errors":
            k, m = map(int, key.split("_")[1:])
            assert np.array_equal(oracle.cauchy(k, m), z[key]), key
        elif key.startswith("fec_") and key != "fec_errors":
            k, n = map(int, key.split("_")[1:])
            full = z[key]
            assert np.array_equal(full[:k], np.eye(k, dtype=np.uint8)), key
            assert np.array_equal(oracle.vandermonde(k, n), full[k:]), key
    for k, m, err in z["rs_errors"]:
        assert oracle.cauchy(int(k), int(m)) is None and err == 1
    for k, n, ok in z["fec_errors"]:
        assert oracle.vandermonde(int(k), int(n)) is None and ok == 0


def test_survey_kat(golden):
    z = golden("encode.npz")
    assert [r.tobytes().hex() for r in z["kat_rs_10_3"]] == ["821ea73bc854ed71", "3647d4a5ef9e0d7c", "c3cad1d8e7eef5fc"]
    assert [r.tobytes().hex() for r in z["kat_fec_10_3"]] == ["c5c4c7c6c1c0c3c2", "dfdedddcdbdad9d8", "c2c3c0c1c6c7c4c5"]


@pytest.mark.parametrize("km,B", list(itertools.product(ENC_CASES, ENC_LENS)))
def test_encode(oracle, golden, km, B):
    z = golden("encode.npz")
    k, m = km
    key = f"{k}_{m}_{B}"
    G = 4
    data = synth_bytes(int(z[f"seed_{key}"][0]), G * k * B).reshape(G, k, B)
    par = np.full((G, m, B), 0x5A, dtype=np.uint8)
    oracle.rs_encode(oracle.cauchy(k, m), data, par, B)
    assert np.array_equal(par.reshape(G * m, B), z[f"rs_{key}"])
    fpar = np.full((G, m, B), 0xA5, dtype=np.uint8)
    oracle.fec_encode(oracle.vandermonde(k, k + m), data, fpar, B)
    assert np.array_equal(fpar.reshape(G * m, B), z[f"fec_{key}"])


def test_encode_quirk(oracle, golden):
    z = golden("encode.npz")
    k, m, B, G = 4, 2, 16, 2
    data = synth_bytes(int(z["quirk_seed"][0]), G * k * B).reshape(G, k, B)
    par = np.full((G, m, B), 0x5A, dtype=np.uint8)
    oracle.rs_encode(z["quirk_matrix"], data, par, B)
    assert np.array_equal(par.reshape(G * m, B), z["quirk_parity"])


RECON = [(4, 2, 16), (10, 3, 8), (16, 4, 8), (2, 1, 5), (3, 2, 33)]


@pytest.mark.parametrize("k,m,B", RECON)
def test_rs_reconstruct(oracle, golden, k, m, B):
    z = golden("reconstruct.npz")
    key = f"{k}_{m}_{B}"
    gm = z[f"marks_{key}"]
    G = gm.shape[0]
    data0 = synth_bytes(int(z[f"seed_{key}"][0]), G * k * B).reshape(G, k, B)
    rows = oracle.cauchy(k, m)
    par_c = np.zeros((G, m, B), dtype=np.uint8)
    oracle.rs_encode(rows, data0, par_c, B)
    assert hashlib.sha256(par_c.tobytes()).digest() == z[f"parc_{key}"].tobytes()
    par_i = synth_bytes(int(z[f"seed_{key}"][0]) ^ 0xFFFF, G * m * B).reshape(G, m, B)
    marks = np.concatenate([gm[:, :k].reshape(-1), gm[:, k:].reshape(-1)]).astype(np.uint8)
    for kind, par in (("cons", par_c), ("incons", par_i)):
        d = data0.copy()
        d.reshape(G * k, B)[marks[:G * k] == 1] = 0x5A
        rc = oracle.rs_reconstruct(rows, d, par.copy(), marks, B)
        assert rc == z[f"rc_{kind}_{key}"][0]
        if kind == "cons":
            assert hashlib.sha256(d.tobytes()).digest() == z[f"cons_{key}"].tobytes()
        else:
            assert np.array_equal(d.reshape(G * k, B), z[f"incons_{key}"])


RECON_LARGE = [(10, 3, 1024), (16, 4, 1400), (10, 3, 1400), (4, 2, 1024), (16, 4, 1024), (12, 4, 1400)]


def large_case(z, k, m, B):
    """Inputs of one reconstruct_large.npz case, regenerated from its seed (the fixture holds
    the reference's output digests, oracle/gen_golden.py gen_reconstruct_large)."""
    key = f"{k}_{m}_{B}"
    gm = z[f"marks_{key}"]
    G = gm.shape[0]
    seed = int(z[f"seed_{key}"][0])
    data0 = synth_bytes(seed, G * k * B).reshape(G, k, B)
    par_i = synth_bytes(seed ^ 0xFFFF, G * m * B).reshape(G, m, B)
    marks = np.concatenate([gm[:, :k].reshape(-1), gm[:, k:].reshape(-1)]).astype(np.uint8)
    return key, gm, data0, par_i, marks


@pytest.mark.parametrize("k,m,B", RECON_LARGE)
def test_rs_reconstruct_large(oracle, golden, k, m, B):
    """The oracle against the reference's rs.c reconstruct at the bench block sizes."""
    z = golden("reconstruct_large.npz")
    key, gm, data0, par_i, marks = large_case(z, k, m, B)
    G = gm.shape[0]
    rows = oracle.cauchy(k, m)
    par_c = np.zeros((G, m, B), dtype=np.uint8)
    oracle.rs_encode(rows, data0, par_c, B)
    for kind, par in (("cons", par_c), ("incons", par_i)):
        d = data0.copy()
        d.reshape(G * k, B)[marks[:G * k] == 1] = 0x5A
        rc = oracle.rs_reconstruct(rows, d, par.copy(), marks, B)
        assert rc == z[f"rc_{kind}_{key}"][0]
        assert hashlib.sha256(d.tobytes()).digest() == z[f"{kind}_{key}"].tobytes()


FEC_DEC = [(2, 4), (3, 5), (5, 8), (4, 6), (3, 4), (4, 5), (5, 6), (7, 8), (10, 13), (16, 20), (1, 3)]


@pytest.mark.parametrize("k,n", FEC_DEC)
def test_fec_decode(oracle, golden, k, n):
    z = golden("fec_decode.npz")
    key = f"{k}_{n}"
    full = z[f"matrix_{key}"]
    assert np.array_equal(oracle.vandermonde(k, n), full[k:])
    for t in range(z[f"rc_{key}"].shape[0]):
        rc, after, idx = oracle.fec_decode(k, n, full, z[f"pk_in_{key}"][t], z[f"idx_in_{key}"][t])
        assert rc == z[f"rc_{key}"][t]
        assert np.array_equal(idx, z[f"idx_out_{key}"][t])
        assert np.array_equal(after, z[f"pk_out_{key}"][t])


def test_fec_reconstruct_matches_rs_rule(oracle):
    """The NetFecCodec receive order (first k valid in group order) and the rs.c
    reconstruct rule (surviving data + first e surviving parity) pick the same
    survivors, so on inconsistent input both give identical bytes for the same matrix."""
    k, m, B, G = 10, 3, 16, 200
    from quicknet_amd.synth import erasure_marks, marks_to_rs_layout
    rows = oracle.vandermonde(k, k + m)
    data = synth_bytes(11, G * k * B).reshape(G, k, B)
    par = synth_bytes(12, G * m * B).reshape(G, m, B)
    marks = marks_to_rs_layout(erasure_marks(13, G, k + m, 3), k)
    a, b = data.copy(), data.copy()
    oracle.rs_reconstruct(rows, a, par.copy(), marks, B)
    bad = oracle.fec_reconstruct(rows, b, par.copy(), marks, B)
    assert bad == 0
    assert np.array_equal(a, b)


WIRE = [(4, 5), (4, 6), (3, 5), (5, 8), (7, 8), (10, 13), (2, 4), (3, 4), (14, 15), (1, 2)]


@pytest.mark.parametrize("k,n", WIRE)
@pytest.mark.parametrize("checksum", [1, 0])
def test_wire_pack_unpack(oracle, golden, k, n, checksum):
    """The FEC wire format vs the reference's own FecCodecBuf.cpp (send: set_fec_enc_buf,
    get_fec_encoded_pkt, pack_fec_head; receive: unpack_fec_head, dec_src_pkt_info)."""
    z = golden("wire.npz")
    key = f"{k}_{n}_{checksum}"
    sizes, payload, seq = z[f"sizes_{key}"], z[f"payload_{key}"], z[f"seq_{key}"]
    dg, dl, gmax = z[f"dgrams_{key}"], z[f"dlen_{key}"], z[f"gmax_{key}"]
    G = dg.shape[0]
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    full = np.concatenate([np.eye(k, dtype=np.uint8), oracle.vandermonde(k, n)])
    for g in range(G):
        out, ln, gm = oracle.pack_group(k, n, full, payload, offs[g * k:(g + 1) * k], sizes[g * k:(g + 1) * k],
                                        int(seq[g, 0]), int(seq[g, 1]), checksum, pitch=dg.shape[2])
        assert gm == gmax[g]
        assert np.array_equal(ln, dl[g])
        assert np.array_equal(out, dg[g])
    parsed, shards, srcinfo = z[f"parsed_{key}"], z[f"shards_{key}"], z[f"srcinfo_{key}"]
    for g in range(G):
        for ik in range(n):
            for var in range(2):
                d = dg[g, ik, :dl[g, ik]].copy()
                if var == 1 and dl[g, ik] > 14:
                    d[14] ^= 0x40
                rc, sent, src, nn, kk, ii, cs, body = oracle.unpack_head(d)
                ok = rc == 1
                assert int(ok) == parsed[g, ik, var, 0]
                if ok:
                    assert [sent, src, nn, kk, ii, len(body), cs] == list(parsed[g, ik, var, 1:8])
                    if var == 0:
                        assert np.array_equal(body, shards[g, ik, :len(body)])
                        if ik < k:
                            off, sz = oracle.dec_src(body, 2068, cs)
                            assert [off, sz] == list(srcinfo[g, ik]) or (off == -1 and srcinfo[g, ik, 0] == -1)


RS_EDIT_CASES = ["p42", "m42", "s42", "s103", "m103w", "m164w"]


def rs_edit_case(z, name):
    """Inputs of one rs_edits.npz case (oracle/gen_golden.py gen_rs_edits): the handle's edited
    matrices, the data, and the parity the reconstruct reads (None: the case encodes it first
    with the edited parity rows, over 0x5A)."""
    k, m, B = (int(x) for x in z[f"shape_{name}"])
    gm = z[f"marks_{name}"]
    G = gm.shape[0]
    seed = int(z[f"seed_{name}"][0])
    data0 = synth_bytes(seed, G * k * B).reshape(G, k, B)
    par = None if f"enc_{name}" in z.files else synth_bytes(seed ^ 0xFFFF, G * m * B).reshape(G, m, B)
    marks = np.concatenate([gm[:, :k].reshape(-1), gm[:, k:].reshape(-1)]).astype(np.uint8)
    return k, m, B, G, data0, par, marks


def rs_edit_match(z, key, arr):
    """The fixture holds small outputs whole and large ones as sha256 digests."""
    ref = z[key]
    a = np.ascontiguousarray(arr)
    if ref.dtype == np.uint8 and ref.ndim == 1 and ref.size == 32 and a.size != 32:
        return hashlib.sha256(a.tobytes()).digest() == ref.tobytes()
    return np.array_equal(a.reshape(ref.shape), ref)


@pytest.mark.parametrize("name", RS_EDIT_CASES)
def test_rs_edits(oracle, golden, name):
    """reed_solomon handles with an edited public parity / m (singular sub-matrices included):
    the oracle's rs.c restatement decodes from rs->m with invert_mat's partial state, as the
    reference did when it produced the fixture."""
    z = golden("rs_edits.npz")
    k, m, B, G, data0, par, marks = rs_edit_case(z, name)
    if par is None:
        par = np.full((G, m, B), 0x5A, np.uint8)
        oracle.rs_encode(z[f"parity_{name}"], data0, par, B)
        assert rs_edit_match(z, f"enc_{name}", par)
    d = data0.copy()
    d.reshape(G * k, B)[marks[: G * k] == 1] = 0x5A
    rc = oracle.rs_reconstruct_full(z[f"m_{name}"], d, par.copy(), marks, B)
    assert rc == z[f"rc_{name}"][0]
    assert rs_edit_match(z, f"out_{name}", d)
    if name == "m42":  # the edited data row of m matters: unit data rows decode differently
        d2 = data0.copy()
        d2.reshape(G * k, B)[marks[: G * k] == 1] = 0x5A
        assert oracle.rs_reconstruct(z[f"m_{name}"][k:], d2, par.copy(), marks, B) == rc
        assert not rs_edit_match(z, f"out_{name}", d2)
