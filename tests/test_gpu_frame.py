"""GPU parity of the ProtocolUdp framing kernels (qfec_frame_udp / qfec_unframe_udp,
network/ProtocolBasic.cpp:111-210 + SessionDesc.cpp:69-77) against the oracle's restatement.
Bit-exact.  Parity unpinned: ProtocolBasic.cpp does not build here, so the oracle itself is
checked only by hand-derived bytes and round trips (tests/test_frame_oracle.py)."""
import numpy as np
import pytest

import quicknet_amd as qa

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.mark.parametrize("session", [False, True])
@pytest.mark.parametrize("pitch", [64, 1056, 1088, 2080])
@pytest.mark.parametrize("op64", [False, True])
def test_frame_vs_oracle(oracle, session, pitch, op64):
    """With the default 16-B output pitch and a 64-B multiple one; two rows per wave, built in
    LDS and stored flat, up to 2 KiB rows, one row per wave above (2080).  301 rows: the last
    wave is partly empty."""
    rng = np.random.default_rng(pitch + session)
    R = 301
    lens = rng.integers(0, pitch + 1, size=R).astype(np.int32)
    lens[:4] = [0, 1, 15, pitch]
    rows = rng.integers(0, 256, size=(R, pitch), dtype=np.uint8)
    masks = rng.integers(0, 256, size=R, dtype=np.uint8)
    ch = rng.integers(0, 2**32, size=(R, 2), dtype=np.uint64).astype(np.uint32) if session else None
    gmask = 0x3C
    P = 12 if session else 4
    out, out_len = qa.frame_udp(dev(rows), dev(lens), dev(masks), gmask=gmask,
                                conv_hid=dev(ch.view(np.int32)) if session else None,
                                out_pitch=(pitch + P + 63) // 64 * 64 if op64 else None)
    torch.cuda.synchronize()
    out, out_len = out.cpu().numpy(), out_len.cpu().numpy()
    P = 12 if session else 4
    for r in range(R):
        ref = oracle.frame_udp(rows[r, :lens[r]], masks[r], gmask=gmask, conv_hid=ch[r] if session else None)
        if P + lens[r] > out.shape[1]:
            assert out_len[r] == -1
            assert not out[r].any(), r  # a rejected row is all zero (include/qfec.h)
            continue
        assert out_len[r] == len(ref), r
        assert np.array_equal(out[r, :len(ref)], ref), r
        assert not out[r, len(ref):].any(), r  # zero up to the pitch


@pytest.mark.parametrize("session", [False, True])
def test_unframe_roundtrip_and_errors(oracle, session):
    rng = np.random.default_rng(7 + session)
    R, pitch = 403, 1072  # odd: the last wave of two or four rows is partly empty
    P = 12 if session else 4
    lens = rng.integers(0, pitch - P + 1, size=R).astype(np.int32)
    rows = rng.integers(0, 256, size=(R, pitch), dtype=np.uint8)
    masks = rng.integers(0, 256, size=R, dtype=np.uint8)
    ch = rng.integers(0, 2**31, size=(R, 2)).astype(np.int32) if session else None
    frames, flen = qa.frame_udp(dev(rows), dev(lens), dev(masks), gmask=0x91, cmd=0x11, protocol=0xFF,
                                conv_hid=dev(ch) if session else None, out_pitch=pitch)
    torch.cuda.synchronize()
    f = frames.cpu().numpy()
    fl = flen.cpu().numpy().copy()
    # corrupt: a payload byte (checksum), the cmd byte (bad cmd after re-XOR), a short frame
    bad_sum, bad_cmd, short = 5, 6, 7
    lens[bad_sum] = max(lens[bad_sum], 3)
    f[bad_sum, P + 1] ^= 0x20
    # a well-formed frame whose cmd lacks 0xA0 (ProtocolBasic.cpp:186): re-sum with the new cmd
    x = int(f[bad_cmd, 0]) ^ 0x91 ^ 0x5A
    w = f[bad_cmd, :fl[bad_cmd]] ^ np.uint8(x)
    w[2] = 0x11
    s_ = int(w[2:].astype(np.int64).sum())
    w[1] = (~((s_ >> 16) + (s_ & 0xFFFF))) & 0xFF
    f[bad_cmd, 1:fl[bad_cmd]] = w[1:] ^ np.uint8(x)
    fl[short] = P - 1
    out, olen, status, info, ch_out = qa.unframe_udp(dev(f), dev(fl), gmask=0x91, session=session)
    torch.cuda.synchronize()
    out, olen, status, info = out.cpu().numpy(), olen.cpu().numpy(), status.cpu().numpy(), info.cpu().numpy()
    for r in range(R):
        st_ref, work, info_ref = oracle.unframe_udp(f[r, :fl[r]], gmask=0x91, session=session)
        assert status[r] == st_ref, r
        if st_ref == 1:
            assert olen[r] == -1
            continue
        assert olen[r] == fl[r] - P
        assert np.array_equal(out[r, :olen[r]], work[P:fl[r]]), r
        assert np.array_equal(info[r], info_ref), r
        if r not in (bad_sum, bad_cmd, short):
            assert st_ref == 0
            assert np.array_equal(out[r, :olen[r]], rows[r, :lens[r]])
            if session:
                assert np.array_equal(ch_out.cpu().numpy()[r], ch[r])
    assert status[bad_sum] == 2 and status[short] == 1 and status[bad_cmd] == 3


def test_frame_the_fec_datagrams(oracle):
    """The two stages in sequence, as the network stack runs them: pack_datagrams ->
    frame_udp (Session::TransmissionOutput's cmd/protocol) -> unframe_udp -> unpack."""
    k, n, G, S = 4, 6, 50, 700
    rng = np.random.default_rng(3)
    sizes = rng.integers(1, S + 1, size=G * k).astype(np.int32)
    payload = rng.integers(0, 256, size=int(sizes.sum()) + 16, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    seq = np.stack([np.arange(G) * n, np.arange(G) * k], 1).astype(np.uint32)
    code = qa.Code.vandermonde(k, n - k)
    _, wire, wlen = code.pack_datagrams(dev(payload), dev(offs), dev(sizes), dev(seq), True)
    Wp = wire.shape[2]
    masks = torch.arange(G * n, dtype=torch.int32, device=DEV).to(torch.uint8)
    ch = torch.zeros((G * n, 2), dtype=torch.int32, device=DEV)
    frames, flen = qa.frame_udp(wire.view(G * n, Wp), wlen.view(-1), masks, gmask=5, conv_hid=ch)
    data, dlen, status, info, _ = qa.unframe_udp(frames, flen, gmask=5, session=True, out_pitch=Wp)
    assert bool((status == 0).all())
    assert torch.equal(dlen, wlen.view(-1))
    sh, st, psize, rx = code.unpack_datagrams(data.view(G, n, Wp), dlen.view(G, n), True)
    torch.cuda.synchronize()
    assert bool((st == 4).all())
    sh = sh.cpu().numpy()
    for g in range(G):
        for i in range(k):
            o, s = offs[g * k + i], sizes[g * k + i]
            assert np.array_equal(sh[g, i, 4:4 + s], payload[o:o + s])
