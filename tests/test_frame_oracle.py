"""CPU checks of the oracle's ProtocolUdp framing restatement (oracle/qfec_oracle.c).
PARITY UNPINNED: network/ProtocolBasic.cpp does not build in this image (its
../system/option.h is absent), so no reference output exists; these tests pin the
restatement to bytes derived by hand from ProtocolBasic.cpp:56-150 and to round trips."""
import numpy as np


def test_frame_bytes_by_hand(oracle):
    data = np.arange(20, dtype=np.uint8)
    f = oracle.frame_udp(data, mask=7, gmask=3, cmd=0x11, protocol=0xFF, conv_hid=(0x11223344, 0x55667788))
    x = 7 ^ 3 ^ 0x5A
    assert f[0] == 7
    assert f[2] == (0x11 | 0xA0) ^ x and f[3] == 0xFF ^ x
    assert list(f[4:8] ^ x) == [0x44, 0x33, 0x22, 0x11] and list(f[8:12] ^ x) == [0x88, 0x77, 0x66, 0x55]
    assert np.array_equal(f[12:] ^ x, data)
    s = 0xB1 + 0xFF + sum([0x44, 0x33, 0x22, 0x11, 0x88, 0x77, 0x66, 0x55]) + int(data.sum())
    assert f[1] ^ x == (~((s >> 16) + (s & 0xFFFF))) & 0xFF


def test_frame_roundtrip_and_errors(oracle):
    rng = np.random.default_rng(1)
    for trial in range(200):
        n = int(rng.integers(0, 300))
        d = rng.integers(0, 256, size=n, dtype=np.uint8)
        sess = bool(trial & 1)
        f = oracle.frame_udp(d, mask=int(rng.integers(0, 256)), gmask=0x42, conv_hid=(1, 2) if sess else None)
        st, work, info = oracle.unframe_udp(f, gmask=0x42, session=sess)
        P = 12 if sess else 4
        assert st == 0 and np.array_equal(work[P:], d) and info[2] == 0x11 and info[3] == 0xFF
        if n:
            g = f.copy()
            g[P + int(rng.integers(0, n))] ^= 0x10
            assert oracle.unframe_udp(g, gmask=0x42, session=sess)[0] == 2
    assert oracle.unframe_udp(np.zeros(3, np.uint8))[0] == 1
