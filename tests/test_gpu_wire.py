"""GPU parity of the FEC datagram batch kernels (quicknet_amd/csrc/qfec_wire.hip) against the
wire vectors the reference's own network/FecCodecBuf.cpp produced (tests/golden/wire.npz)
and against the oracle at larger sizes.  Bit-exact."""
import numpy as np
import pytest

import quicknet_amd as qa

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")
WIRE = [(4, 5), (4, 6), (3, 5), (5, 8), (7, 8), (10, 13), (2, 4), (3, 4), (14, 15), (1, 2)]
STAGED_ONLY = {(14, 15), (1, 2)}  # (k, n) without a fused instance


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def padded_payload(p):
    return dev(np.concatenate([p, np.zeros(16, np.uint8)]))  # 16 readable bytes past the end


@pytest.fixture(params=[(1, 0), (0, 0)], ids=["fused", "staged"])
def wire_fused(request):
    """Both datagram paths: fused (send: body + head launches; receive: one launch; templated
    (k, m)) and staged (build -> encode -> emit, parse -> reconstruct -> check), which every
    shape can take."""
    saved = {kk: qa.tune_get(kk) for kk in ("wire_fused", "wire_rx")}
    qa.tune("wire_fused", request.param[0])
    qa.tune("wire_rx", request.param[0])
    yield request.param
    for kk, v in saved.items():
        qa.tune(kk, v)


@pytest.fixture(params=[64, 16], ids=["wire64", "wire16"])
def wire_align(request):
    """Wire row pitch rounded to 64 B (the fused send writes whole 64-B lines: body from chunk
    4 or 0 up to the pitch, k_pack_line0 for the first line) or to 16 B (body + k_pack_head)."""
    return request.param


def wire_pitch_for(shard_pitch, align):
    return (shard_pitch + 13 + align - 1) // align * align


@pytest.mark.parametrize("k,n", WIRE)
@pytest.mark.parametrize("checksum", [1, 0])
def test_pack_vs_reference(golden, wire_fused, wire_align, k, n, checksum):
    z = golden("wire.npz")
    key = f"{k}_{n}_{checksum}"
    sizes, payload, seq = z[f"sizes_{key}"], z[f"payload_{key}"], z[f"seq_{key}"]
    dg, dl = z[f"dgrams_{key}"], z[f"dlen_{key}"]
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    code = qa.Code.vandermonde(k, n - k)
    sp = (int(sizes.max()) + (4 if checksum else 2) + 15) // 16 * 16
    shards, wire, wlen = code.pack_datagrams(padded_payload(payload), dev(offs), dev(sizes), dev(seq.astype(np.uint32)),
                                             checksum=bool(checksum), shard_pitch=sp,
                                             wire_pitch=wire_pitch_for(sp, wire_align))
    torch.cuda.synchronize()
    wlen = wlen.cpu().numpy()
    wire = wire.cpu().numpy()
    assert np.array_equal(wlen, dl)
    for g in range(dg.shape[0]):
        for j in range(n):
            assert np.array_equal(wire[g, j, :dl[g, j]], dg[g, j, :dl[g, j]]), (g, j)


@pytest.mark.parametrize("k,n", WIRE)
@pytest.mark.parametrize("checksum", [1, 0])
def test_unpack_vs_reference(golden, wire_fused, k, n, checksum):
    z = golden("wire.npz")
    key = f"{k}_{n}_{checksum}"
    dg, dl = z[f"dgrams_{key}"], z[f"dlen_{key}"]
    parsed, shards_ref, srcinfo = z[f"parsed_{key}"], z[f"shards_{key}"], z[f"srcinfo_{key}"]
    G = dg.shape[0]
    code = qa.Code.vandermonde(k, n - k)
    for var in range(2):
        w = np.zeros((G, n, 2080), np.uint8)
        w[..., : dg.shape[2]] = dg
        if var == 1:
            for g in range(G):
                for j in range(n):
                    if dl[g, j] > 14:
                        w[g, j, 14] ^= 0x40
        shards, status, psize, rx = code.unpack_datagrams(dev(w), dev(dl), checksum=bool(checksum))
        torch.cuda.synchronize()
        rx = rx.cpu().numpy()
        shards = shards.cpu().numpy()
        status = status.cpu().numpy()
        for g in range(G):
            for j in range(n):
                ok, unlen = parsed[g, j, var, 0], parsed[g, j, var, 6]
                assert (rx[g, j] >= 0) == bool(ok), (var, g, j)
                if ok:
                    assert rx[g, j] == unlen
                    # check-shard rows are scratch on the fused receive path
                    if var == 0 and (j < k or not wire_fused[0] or (k, n) in STAGED_ONLY):
                        assert np.array_equal(shards[g, j, :unlen], shards_ref[g, j, :unlen])
            if var == 0:  # nothing lost: every source row gets dec_src_pkt_info's verdict
                for i in range(k):
                    assert status[g, i] == srcinfo[g, i, 0], (g, i)


@pytest.mark.parametrize("k,n,checksum", [(10, 13, 1), (4, 6, 1), (14, 15, 0), (5, 8, 1), (10, 13, 0), (8, 12, 1)])
def test_lossy_roundtrip_vs_oracle(oracle, wire_fused, wire_align, k, n, checksum):
    """Pack G groups, drop and corrupt datagrams, unpack: every data packet comes back exactly
    when its group has k valid datagrams; the verdicts match the reference rules (oracle)."""
    rng = np.random.default_rng(k * 100 + n)
    G, m = 400, n - k
    sizes = rng.integers(0, 1401, size=G * k).astype(np.int32)
    payload = rng.integers(0, 256, size=int(sizes.sum()) + 1, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    seq = np.stack([np.arange(G, dtype=np.uint32) * n + 3, np.arange(G, dtype=np.uint32) * k + 9], 1)
    code = qa.Code.vandermonde(k, m)
    full = np.concatenate([np.eye(k, dtype=np.uint8), code.rows])
    sp = (int(sizes.max()) + (4 if checksum else 2) + 15) // 16 * 16
    shards, wire, wlen = code.pack_datagrams(padded_payload(payload), dev(offs), dev(sizes), dev(seq), bool(checksum),
                                             shard_pitch=sp, wire_pitch=wire_pitch_for(sp, wire_align))
    torch.cuda.synchronize()
    w = wire.cpu().numpy()
    wl = wlen.cpu().numpy()
    # oracle datagrams for a sample of groups
    for g in rng.choice(G, 25, replace=False):
        out, ln, _ = oracle.pack_group(k, n, full, payload, offs[g * k:(g + 1) * k], sizes[g * k:(g + 1) * k],
                                       int(seq[g, 0]), int(seq[g, 1]), checksum, pitch=w.shape[2])
        assert np.array_equal(ln, wl[g])
        for j in range(n):
            assert np.array_equal(out[j, :ln[j]], w[g, j, :ln[j]])
    # losses: drop up to m + 1 datagrams per group, corrupt one more in some groups
    drop = np.zeros((G, n), bool)
    corrupt = np.zeros((G, n), bool)
    for g in range(G):
        for j in rng.choice(n, int(rng.integers(0, m + 2)), replace=False):
            drop[g, j] = True
        if checksum and rng.random() < 0.3:
            j = int(rng.integers(0, n))
            if not drop[g, j] and wl[g, j] > 13:
                corrupt[g, j] = True
                w[g, j, 13] ^= 0x01
    rx_len = np.where(drop, 0, wl).astype(np.int32)
    sh, status, psize, rx = code.unpack_datagrams(dev(w), dev(rx_len), checksum=bool(checksum),
                                                  shard_pitch=shards.shape[2])
    torch.cuda.synchronize()
    sh, status, psize, rx = sh.cpu().numpy(), status.cpu().numpy(), psize.cpu().numpy(), rx.cpu().numpy()
    head = 4 if checksum else 2
    for g in range(G):
        valid = ~drop[g] & ~corrupt[g]
        assert np.array_equal(rx[g] >= 0, valid)
        recoverable = valid.sum() >= k
        for i in range(k):
            if not valid[i] and not recoverable:
                assert status[g, i] == -2
                continue
            assert status[g, i] == head, (g, i)
            sz = sizes[g * k + i]
            assert psize[g, i] == sz
            assert np.array_equal(sh[g, i, head:head + sz], payload[offs[g * k + i]:offs[g * k + i] + sz])


def test_pack_oversize_group(wire_fused):
    """A size the shard pitch cannot hold (or a negative one) voids its group only:
    wire_len -1 for its n datagrams, the other groups are packed as usual."""
    k, n, G = 4, 6, 6
    sizes = np.full(G * k, 100, np.int32)
    sizes[1 * k + 2] = 125  # 125 + 4 > 128
    sizes[4 * k + 0] = -3
    payload = np.arange(int(np.maximum(sizes, 0).sum()) + 1, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(np.maximum(sizes, 0))[:-1]]).astype(np.int64)
    seq = np.zeros((G, 2), np.uint32)
    code = qa.Code.vandermonde(k, n - k)
    _, wire, wlen = code.pack_datagrams(padded_payload(payload), dev(offs), dev(sizes), dev(seq), True, shard_pitch=128)
    torch.cuda.synchronize()
    wl = wlen.cpu().numpy()
    assert (wl[1] == -1).all() and (wl[4] == -1).all()
    good = [0, 2, 3, 5]
    assert (wl[good, :k] == 13 + 104).all() and (wl[good, k:] == 13 + 104).all()


@pytest.mark.parametrize("k,n,checksum,pitch", [(10, 13, 1, 1040), (10, 13, 0, 1040), (4, 6, 1, 1040), (8, 12, 1, 1040),
                                                (5, 8, 1, 1056), (8, 12, 1, 1056), (4, 6, 1, 1088), (4, 5, 0, 1088),
                                                (10, 13, 1, 528), (7, 8, 1, 544), (3, 5, 1, 1280), (10, 13, 1, 1408),
                                                (4, 6, 0, 1408), (5, 8, 1, 1536), (10, 13, 1, 1296)])
def test_unpack_row_tails(k, n, checksum, pitch):
    """Shard pitches whose passes leave a short row tail (1040 = 1024 + 16 and 528 = 512 + 16: k_rx
    runs the tail lane-mapped; 1056, 1088, 544, 1280, 1408, 1536, 1296: a partial last pass): every
    data packet of a recoverable group comes back exactly, and every form of the receive -- 16-B and
    8-B lanes, with and without the rows staged in LDS, and the staged three-launch path -- gives
    the same shard rows, verdicts and sizes.  Losses up to m + 1 per group, some datagrams corrupted
    inside the row tail, half the rows full to the pitch's limit."""
    rng = np.random.default_rng(pitch * 31 + k)
    G, m = 300, n - k
    head = 4 if checksum else 2
    maxsz = pitch - head
    sizes = rng.integers(0, maxsz + 1, size=G * k).astype(np.int32)
    sizes[rng.random(G * k) < 0.5] = maxsz  # full rows: tails end at the pitch
    sizes[rng.random(G * k) < 0.1] = maxsz - 13  # a datagram ending inside the tail
    payload = rng.integers(0, 256, size=int(sizes.sum()) + 1, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    seq = np.stack([np.arange(G, dtype=np.uint32) * n, np.arange(G, dtype=np.uint32) * k], 1)
    code = qa.Code.vandermonde(k, m)
    _, wire, wlen = code.pack_datagrams(padded_payload(payload), dev(offs), dev(sizes), dev(seq), bool(checksum),
                                        shard_pitch=pitch, wire_pitch=wire_pitch_for(pitch, 16))
    torch.cuda.synchronize()
    w, wl = wire.cpu().numpy(), wlen.cpu().numpy()
    drop = np.zeros((G, n), bool)
    for g in range(G):
        drop[g, rng.choice(n, int(rng.integers(0, m + 2)), replace=False)] = True
        if checksum and rng.random() < 0.2:
            j = int(rng.integers(0, n))
            if not drop[g, j] and wl[g, j] > pitch - 8:
                w[g, j, wl[g, j] - 1] ^= 0x10  # a byte inside the row tail
    rx_len = np.where(drop, 0, wl).astype(np.int32)
    outs = []
    # every form of the fused receive (tuning "wire_rx": 1 auto, 2 / 3 16-B lanes with / without
    # the rows staged in LDS, 4 / 5 8-B lanes likewise) and the staged three-launch path (0)
    saved = qa.tune_get("wire_rx")
    for rxk in (1, 2, 3, 4, 5, 0):
        qa.tune("wire_rx", rxk)
        try:
            sh, status, psize, rx = code.unpack_datagrams(dev(w), dev(rx_len), checksum=bool(checksum), shard_pitch=pitch)
            torch.cuda.synchronize()
        finally:
            qa.tune("wire_rx", saved)
        outs.append([t.cpu().numpy() for t in (sh, status, psize, rx)])
    sh, status, psize, rx = outs[0]
    for sh0, status0, psize0, rx0 in outs[1:]:
        assert np.array_equal(sh[:, :k], sh0[:, :k])
        assert np.array_equal(status, status0) and np.array_equal(psize, psize0) and np.array_equal(rx, rx0)
    for g in range(G):
        if (rx[g] >= 0).sum() < k:
            continue
        for i in range(k):
            if status[g, i] != head:
                continue
            sz = sizes[g * k + i]
            assert psize[g, i] == sz
            assert np.array_equal(sh[g, i, head:head + sz], payload[offs[g * k + i]:offs[g * k + i] + sz]), (g, i)
    ok_rows = (status[:, :] == head).sum()
    assert ok_rows > G * k // 2


@pytest.mark.parametrize("k,n,G,sp,wp", [(10, 13, 500, 1040, 1088), (4, 6, 500, 1040, 1088), (8, 12, 500, 1040, 1088),
                                         (5, 8, 500, 1040, 1088), (10, 13, 13, 1040, 1088), (10, 13, 500, 528, 576),
                                         (4, 6, 501, 528, 576), (10, 13, 13, 528, 576), (10, 13, 500, 1408, 1472),
                                         (4, 6, 500, 1408, 1472), (8, 12, 501, 1408, 1472), (10, 13, 13, 1408, 1472),
                                         (3, 5, 300, 1104, 1152), (10, 13, 200, 2096, 2112), (10, 13, 300, 784, 832),
                                         (4, 6, 301, 592, 640), (3, 5, 300, 1536, 1600), (4, 6, 77, 1408, 1472)])
def test_pack_wave64_matches_line0(oracle, k, n, G, sp, wp):
    """The fused send at the wire pitches the library picks its forms by -- one wave per group
    finishing line 0 itself (k_pack_wave64: 1 088 B on 16-B lanes, 576 B two groups per wave,
    1 104..1 600 B on 8-B lanes in three passes), the body + k_pack_line0 pair at other 64-B
    multiples (832, 640, 2 112) -- writes the same datagrams and lengths as the staged path
    (wire_fused 0), and both equal the oracle's on sampled groups.  Sizes 0 .. sp - 4 (half
    exactly sp - 16), one oversize group, G = 13 / 501 leave the last block partly (or a wave
    half) dead."""
    rng = np.random.default_rng(n * 7 + k + G + sp)
    m = n - k
    sizes = rng.integers(0, sp - 3, size=G * k).astype(np.int32)
    sizes[rng.random(G * k) < 0.5] = sp - 16
    sizes[:3] = [0, 1, 46]  # payloads ending inside line 0
    sizes[7 * k + 1] = sp  # sp + 4 > the shard pitch: group 7 is void
    payload = rng.integers(0, 256, size=int(np.maximum(sizes, 0).sum()) + 1, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    seq = np.stack([np.arange(G, dtype=np.uint32) * n + 5, np.arange(G, dtype=np.uint32) * k + 2], 1)
    code = qa.Code.vandermonde(k, m)
    full = np.concatenate([np.eye(k, dtype=np.uint8), code.rows])
    res = []
    saved = qa.tune_get("wire_fused")
    for w in (1, 0):
        qa.tune("wire_fused", w)
        try:
            _, wire, wlen = code.pack_datagrams(padded_payload(payload), dev(offs), dev(sizes), dev(seq), True,
                                                shard_pitch=sp, wire_pitch=wp)
            torch.cuda.synchronize()
        finally:
            qa.tune("wire_fused", saved)
        res.append((wire.cpu().numpy(), wlen.cpu().numpy()))
    (w1, l1), (w0, l0) = res
    assert np.array_equal(l1, l0)
    assert (l1[7] == -1).all()
    for g in range(G):
        if g == 7:
            continue
        for j in range(n):
            assert np.array_equal(w1[g, j, :l1[g, j]], w0[g, j, :l0[g, j]]), (g, j)
            assert not w1[g, j, l1[g, j]:].any(), (g, j)  # zeros up to the pitch (whole lines)
    for g in list(rng.choice(G, min(G, 20), replace=False)) + [0, G - 1]:
        if g == 7:
            continue
        out, ln, _ = oracle.pack_group(k, n, full, payload, offs[g * k:(g + 1) * k], sizes[g * k:(g + 1) * k],
                                       int(seq[g, 0]), int(seq[g, 1]), 1, shard_cap=max(2052, sp), pitch=wp)
        assert np.array_equal(ln, l1[g])
        for j in range(n):
            assert np.array_equal(out[j, :ln[j]], w1[g, j, :ln[j]]), (g, j)
