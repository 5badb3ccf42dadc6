"""GPU: FEC datagrams straight to / from ProtocolUdp frames in one pass (qfec_pack_frames /
qfec_unpack_frames) against the oracle's pack_group (network/FecCodecBuf.cpp, pinned by the
reference's own vectors) composed with its frame_udp / unframe_udp restatement
(network/ProtocolBasic.cpp:111-199, SessionDesc.cpp:69-77 -- parity unpinned: ProtocolBasic.cpp
does not build here), and against the two-call product path the one-pass kernels replace.
Bit-exact, both checksum modes, Session prefix on and off, per-datagram masks, the one-pass
pitches (1088 / 576) and a pitch that takes the two-call fallback, bad checksum / cmd / short /
too-long frames, a bad FEC header and a bad shard checksum inside well-formed frames."""
import numpy as np
import pytest

import quicknet_amd as qa

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")
GMASK = 0xA7


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def padded(p):
    return dev(np.concatenate([p, np.zeros(16, np.uint8)]))


def make_batch(rng, k, n, G, sp, oversize_group=None):
    sizes = rng.integers(0, sp - 3, size=G * k).astype(np.int32)
    sizes[rng.random(G * k) < 0.4] = sp - 16
    sizes[:3] = [0, 1, 40]  # payloads ending inside line 0
    if oversize_group is not None:
        sizes[oversize_group * k + 1] = sp  # sp + 4 > the shard pitch: the group is void
    payload = rng.integers(0, 256, size=int(sizes.sum()) + 1, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    seq = np.stack([np.arange(G, dtype=np.uint32) * n + 7, np.arange(G, dtype=np.uint32) * k + 3], 1)
    return sizes, payload, offs, seq


def oracle_frames(oracle, code, k, n, g, sizes, payload, offs, seq, checksum, masks, ch):
    full = np.concatenate([np.eye(k, dtype=np.uint8), code.rows])
    out, ln, _ = oracle.pack_group(k, n, full, payload, offs[g * k:(g + 1) * k], sizes[g * k:(g + 1) * k],
                                   int(seq[g, 0]), int(seq[g, 1]), checksum, pitch=2200)
    return [oracle.frame_udp(out[j, :ln[j]], masks[g * n + j], gmask=GMASK,
                             conv_hid=ch[g * n + j] if ch is not None else None) for j in range(n)]


CASES = [(10, 13, 500, 1040, 1), (4, 6, 501, 1040, 1), (8, 12, 13, 1040, 1), (10, 13, 500, 528, 1), (4, 6, 130, 1408, 1),
         (4, 6, 77, 528, 1), (10, 13, 200, 1408, 1), (10, 13, 150, 1040, 0), (5, 8, 120, 1040, 1)]


@pytest.mark.parametrize("session", [False, True], ids=["udp", "session"])
@pytest.mark.parametrize("k,n,G,sp,checksum", CASES)
def test_pack_frames_vs_oracle(oracle, k, n, G, sp, checksum, session):
    """One pass where it applies (checksums on, 1088 / 576-B frame pitch), the two-call path
    otherwise; both against pack_group o frame_udp, padding zero, a void group -1."""
    rng = np.random.default_rng(k * 1000 + G + sp + session)
    sizes, payload, offs, seq = make_batch(rng, k, n, G, sp, oversize_group=5)
    code = qa.Code.vandermonde(k, n - k)
    masks = rng.integers(0, 256, size=G * n, dtype=np.uint8)
    ch = rng.integers(0, 2**32, size=(G * n, 2), dtype=np.uint64).astype(np.uint32) if session else None
    P = 12 if session else 4
    res = []
    for fused in (1, 0):
        qa.tune("wire_fused", fused)
        try:
            fr, fl = code.pack_frames(padded(payload), dev(offs), dev(sizes), dev(seq), dev(masks), gmask=GMASK,
                                      conv_hid=dev(ch.view(np.int32)) if session else None, checksum=bool(checksum),
                                      shard_pitch=sp)
            torch.cuda.synchronize()
        finally:
            qa.tune("wire_fused", 1)
        res.append((fr.cpu().numpy(), fl.cpu().numpy()))
    (f1, l1), (f0, l0) = res
    assert f1.shape[2] == (sp + 13 + P + 63) // 64 * 64
    assert np.array_equal(l1, l0)
    assert (l1[5] == -1).all()
    for g in range(G):
        if g == 5:
            continue
        for j in range(n):
            assert np.array_equal(f1[g, j, :l1[g, j]], f0[g, j, :l0[g, j]]), (g, j)
            assert not f1[g, j, l1[g, j]:].any(), (g, j)  # bytes past the frame are zero
    for g in list(rng.choice(G, min(G, 25), replace=False)) + [0, G - 1]:
        if g == 5:
            continue
        ref = oracle_frames(oracle, code, k, n, g, sizes, payload, offs, seq, checksum, masks, ch)
        for j in range(n):
            assert l1[g, j] == len(ref[j]), (g, j)
            assert np.array_equal(f1[g, j, :len(ref[j])], ref[j]), (g, j)


def _reframe(oracle, dgram, mask, ch):
    return oracle.frame_udp(dgram, mask, gmask=GMASK, conv_hid=ch)


@pytest.mark.parametrize("session", [False, True], ids=["udp", "session"])
@pytest.mark.parametrize("k,n,G,sp,checksum", CASES)
def test_unpack_frames_vs_oracle(oracle, k, n, G, sp, checksum, session):
    """Frames with losses and every RecvPacket failure: statuses equal unframe_udp's (oracle);
    the FEC results equal unpack_datagrams over the datagrams the oracle unframes (failed
    frames not received); every payload of a group with k valid datagrams comes back exactly;
    the one-pass and two-call paths agree byte for byte."""
    rng = np.random.default_rng(k * 77 + G + sp + session)
    sizes, payload, offs, seq = make_batch(rng, k, n, G, sp)
    code = qa.Code.vandermonde(k, n - k)
    m = n - k
    masks = rng.integers(0, 256, size=G * n, dtype=np.uint8)
    ch = rng.integers(0, 2**31, size=(G * n, 2)).astype(np.int32) if session else None
    P = 12 if session else 4
    fr, fl = code.pack_frames(padded(payload), dev(offs), dev(sizes), dev(seq), dev(masks), gmask=GMASK,
                              conv_hid=dev(ch) if session else None, checksum=bool(checksum), shard_pitch=sp)
    torch.cuda.synchronize()
    f, fl = fr.cpu().numpy(), fl.cpu().numpy().copy()
    FP = f.shape[2]
    # losses and damage
    kinds = {}
    for g in range(G):
        for j in rng.choice(n, int(rng.integers(0, m + 2)), replace=False):
            fl[g, j] = 0
        if rng.random() < 0.5:
            j = int(rng.integers(0, n))
            if fl[g, j] > P + 13:
                kind = int(rng.integers(0, 7))
                kinds[(g, j)] = kind
                x = int(f[g, j, 0]) ^ GMASK ^ 0x5A
                w = f[g, j, :fl[g, j]] ^ np.uint8(x)  # un-XORed frame (byte 0 garbage)
                dg = w[P:].copy()
                if kind == 0:    # a payload byte: the frame checksum fails
                    f[g, j, fl[g, j] - 1] ^= 0x40
                elif kind == 1:  # cmd without 0xA0 but a correct checksum
                    w[2] = 0x11
                    s_ = int(w[2:].astype(np.int64).sum())
                    w[1] = (~((s_ >> 16) + (s_ & 0xFFFF))) & 0xFF
                    f[g, j, 1:fl[g, j]] = w[1:] ^ np.uint8(x)
                elif kind == 6:  # cmd without 0xA0 AND a bad checksum: RecvPacket says checksum (2)
                    w[2] = 0x11
                    s_ = int(w[2:].astype(np.int64).sum())
                    w[1] = ((~((s_ >> 16) + (s_ & 0xFFFF))) & 0xFF) ^ 0x01
                    f[g, j, 1:fl[g, j]] = w[1:] ^ np.uint8(x)
                elif kind == 2:  # short
                    fl[g, j] = P - 1
                elif kind == 3:  # longer than the pitch
                    fl[g, j] = FP + 1
                elif kind == 4:  # well-formed frame, bad FEC header (k field)
                    dg[9] ^= 0x10
                    new = _reframe(oracle, dg, masks[g * n + j], ch[g * n + j] if session else None)
                    f[g, j, :len(new)] = new
                else:            # well-formed frame, bad shard checksum (or, without checksums, bad size)
                    dg[-1] ^= 0x01
                    new = _reframe(oracle, dg, masks[g * n + j], ch[g * n + j] if session else None)
                    f[g, j, :len(new)] = new
    # the oracle's RecvPacket over every row, and the datagrams it hands to the FEC layer
    st_ref = np.zeros((G, n), np.int32)
    Wp = (sp + 13 + 15) // 16 * 16 + 16
    dgrams = np.zeros((G, n, Wp), np.uint8)
    dlen = np.zeros((G, n), np.int32)
    for g in range(G):
        for j in range(n):
            st, work, _ = oracle.unframe_udp(f[g, j, :max(fl[g, j], 0)] if fl[g, j] <= FP else f[g, j, :0],
                                             gmask=GMASK, session=session)
            if fl[g, j] > FP:
                st = 4
            st_ref[g, j] = st
            if st == 0:
                d = work[P:fl[g, j]]
                dgrams[g, j, :len(d)] = d
                dlen[g, j] = len(d)
    want = code.unpack_datagrams(dev(dgrams), dev(dlen), checksum=bool(checksum), shard_pitch=sp)
    torch.cuda.synchronize()
    want = [t.cpu().numpy() for t in want]
    outs = []
    saved = qa.tune_get("wire_rx")
    for rxk in (1, 0, 3, 4):  # one pass (auto, 16-B lanes unstaged, 8-B lanes staged), two calls
        qa.tune("wire_rx", rxk)
        try:
            got = code.unpack_frames(dev(f), dev(fl), gmask=GMASK, session=session, checksum=bool(checksum),
                                     shard_pitch=sp)
            torch.cuda.synchronize()
        finally:
            qa.tune("wire_rx", saved)
        outs.append([t.cpu().numpy() if t is not None else None for t in got])
    for sh, status, psize, rx, fst, cho in outs:
        assert np.array_equal(fst, st_ref)
        assert np.array_equal(rx, want[3])
        assert np.array_equal(status, want[1])
        assert np.array_equal(psize, want[2])
        head = 4 if checksum else 2
        for g in range(G):
            for i in range(k):
                if status[g, i] >= 0:
                    sz = psize[g, i]
                    assert np.array_equal(sh[g, i, :head + sz], want[0][g, i, :head + sz]), (g, i)
                    # without checksums a corrupted shard inside a good frame is undetectable: the
                    # group then decodes garbage (as the reference would); no truth check for it
                    silent = not checksum and any(kg == g and kd == 5 for (kg, _), kd in kinds.items())
                    if (g, i) not in kinds and not silent:
                        assert sz == sizes[g * k + i]
                        o = offs[g * k + i]
                        assert np.array_equal(sh[g, i, head:head + sz], payload[o:o + sz]), (g, i)
        if session:
            ok = fst == 0
            assert np.array_equal(cho[ok], ch.reshape(G, n, 2)[ok])
    if G >= 100:
        assert set(kinds.values()) >= {0, 1, 2, 3, 4, 5, 6}
    for (g, j), kd in kinds.items():  # both checks failing: the checksum verdict, as RecvPacket
        if kd == 6:
            assert st_ref[g, j] == 2
    # recoverable groups: every payload back
    (sh, status, psize, rx, fst, _) = outs[0]
    assert (status >= 0).sum() > G * k // 2
