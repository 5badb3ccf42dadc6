"""CPU: the oracle's restatement of network/NetFecCodec.cpp (oracle/zfec_ref.py) and the
host-only paths of libqfec's exact layer (include/qfec_zfec.h).

The restatement's control flow is PARITY UNPINNED (NetFecCodec.cpp does not build here); these
tests pin what can be pinned: round trips through the reference's own compiled buffer code
(FecCodecBuf.cpp, fec.c), the delivery-order properties the cited lines imply, and the quirks
read off the source (codec-list collisions, the lost-rate -> (k, n) map).
"""
import os
import random

import pytest

from oracle import zfec_ref
from zfec_script import make_script, run_oracle

pytestmark = pytest.mark.skipif(not zfec_ref.available(), reason="oracle/_ref not built (make -C oracle ref)")


def _payloads(n, seed=0, hi=1400):
    rng = random.Random(seed)
    return [bytes(rng.getrandbits(8) for _ in range(rng.randint(0, hi))) for _ in range(n)]


def _pair(**kw):
    return zfec_ref.ZfecLayer(**kw), zfec_ref.ZfecLayer(**kw)


@pytest.mark.parametrize("is_sorted", [False, True])
def test_lossless_round_trip(is_sorted):
    A, B = _pair(is_sorted=is_sorted)
    pay = _payloads(40)
    for p in pay:
        A.pack_input(p)
    # 40 packets in (4, 5) groups: 10 groups, 50 datagrams, all 0xED (is_send_checksum)
    assert len(A.out) == 50 and all(d[0] == 0xED for d in A.out)
    for d in A.out:
        B.unpack_input(d)
    assert B.deliv == [(p, i) for i, p in enumerate(pay)]
    A.close()
    B.close()


@pytest.mark.parametrize("is_sorted", [False, True])
def test_one_loss_per_group_recovered(is_sorted):
    """n - k = 1 loss per group -> every payload delivered once; sorted mode delivers in source
    order (expected index + flush_avail_pkts), unsorted delivers survivors first."""
    A, B = _pair(is_sorted=is_sorted)
    pay = _payloads(40, seed=1)
    for p in pay:
        A.pack_input(p)
    rng = random.Random(2)
    for g in range(10):
        lost = rng.randrange(5)
        for j in range(5):
            if j != lost:
                B.unpack_input(A.out[5 * g + j])
    assert sorted(B.deliv, key=lambda x: x[1]) == [(p, i) for i, p in enumerate(pay)]
    srcs = [s for _, s in B.deliv]
    if is_sorted:
        assert srcs == sorted(srcs)
    assert B.fec_restore_count > 0
    A.close()
    B.close()


def test_unsorted_immediate_delivery_and_duplicates():
    """Unsorted: a source datagram is handed over on arrival (NetFecCodec.cpp:256-265), a
    duplicate of a delivered one is not (bUsed)."""
    A, B = _pair()
    pay = _payloads(8, seed=3)
    for p in pay:
        A.pack_input(p)
    d = A.out
    B.unpack_input(d[2])
    assert B.deliv == [(pay[2], 2)]
    B.unpack_input(d[2])
    assert len(B.deliv) == 1
    B.unpack_input(d[4])  # the check packet: 4 of 5 in? no -- 2 valid, nothing decodes
    assert len(B.deliv) == 1
    for j in (0, 3):
        B.unpack_input(d[j])
    # 4 valid (0, 2, 3, check) -> decode restores 1; 0 and 3 were delivered on arrival
    assert [s for _, s in B.deliv] == [2, 0, 3, 1]
    A.close()
    B.close()


def test_sorted_expected_index_trace():
    """Sorted mode as NetFecCodec.cpp:266-299 is written, IUINT32 arithmetic included: after an
    in-order delivery the skip-ahead test `i_recv - i_expected >= 2n` (:289) wraps (i_recv is
    one behind the incremented expected index) and resets the expected index to the group
    start, so the next source packet is buffered; a decode (k valid, not all in the window's
    first k slots, :523) flushes the buffer (:296-299) and delivers the group in order; a packet
    2n or more ahead jumps the expected index (:291-292); an old packet resets it backwards."""
    A, B = _pair(is_sorted=True)
    for i in range(40):
        A.pack_input(bytes([i]) * 10)
    d = A.out  # (4, 5) groups: datagram 5g + j, source 4g + j
    trace = []
    for j in [0, 1, 5, 6, 7, 8, 9, 20, 21, 22, 23, 24, 2, 3, 4]:
        B.unpack_input(d[j])
        trace.append(([s for _, s in B.deliv], B.i_expected_packet))
    T = [([0], 0), ([0], 0), ([0], 0), ([0], 0), ([0], 0), ([0, 1, 4, 5, 6, 7], 10), ([0, 1, 4, 5, 6, 7], 10),
         ([0, 1, 4, 5, 6, 7], 20), ([0, 1, 4, 5, 6, 7], 20), ([0, 1, 4, 5, 6, 7], 20),
         ([0, 1, 4, 5, 6, 7, 16, 17, 18, 19], 25)]
    T += [(T[-1][0], 25), (T[-1][0], 0), (T[-1][0], 0), (T[-1][0], 0)]
    assert trace == T
    assert all(p == bytes([s]) * 10 for p, s in B.deliv)
    A.close()
    B.close()


def test_fec_off_tag():
    A, B = _pair(enabled=False)
    pay = _payloads(5, seed=5)
    for p in pay:
        A.pack_input(p)
    assert A.out == [b"\x13" + p for p in pay]
    for d in A.out:
        B.unpack_input(d)
    assert B.deliv == [(p, 0) for p in pay]
    A.close()
    B.close()


def test_dynamic_kn_follows_lost_rate():
    """recalc_zfec_kn at each group end: get_codec_by(lost) over the redundancy-sorted list
    (0.125 (7,8), 0.167 (5,6), 0.2 (4,5), 0.25 (3,4), 0.333 (4,6), 0.375 (5,8), 0.4 (3,5),
    0.5 (2,4)): the first key >= lost."""
    A, _ = _pair()
    A.dynkn = True
    for lost, kn in [(0.3, (4, 6)), (0.0, (7, 8)), (0.19, (4, 5)), (0.45, (2, 4)), (0.9, (2, 4))]:
        A.lost_rate = lost
        k = A.fec_codec[0]
        for _ in range(k):
            A.pack_input(b"x")
        assert A.fec_codec[:2] == kn, lost
    A.close()


def test_codec_collision_leaves_null_entry():
    """add_new_codec of (4, 8): its redundancy 0.5 equals (2, 4)'s -> the map entry becomes
    NULL (FecCodec.cpp:86-93); find_codec then fails for both, while the sender keeps the new
    item as its current codec."""
    A, B = _pair()
    A.set_kn(4, 8, True)
    B.set_kn(4, 8, True)
    assert A.fec_codec[:2] == (4, 8)
    assert B.codecs.find(4, 8) is None and B.codecs.find(2, 4) is None
    pay = _payloads(4, seed=6)
    for p in pay:
        A.pack_input(p)
    for d in A.out[1:]:  # source 0 lost: the receiver has no (4, 8) codec, nothing decodes
        B.unpack_input(d)
    assert [s for _, s in B.deliv] == [1, 2, 3]
    A.close()
    B.close()


@pytest.mark.parametrize("seed", range(6))
def test_scripts_run_and_conserve(seed):
    """The lossy-channel scripts the GPU test replays: every delivery is a payload that was
    sent, at its own source index (or an FEC-off payload, handed over with index 0, possibly
    corrupted by the channel since nothing checks it)."""
    for pair in (dict(), dict(is_sorted=True)):
        sc = make_script(seed, pair=pair, forge=False)  # (forged check packets poison decodes)
        res, st = run_oracle(sc)
        sent, off = {}, set()
        for r in res:
            for d in r["datagrams"]:
                if d[0] == 0x13:
                    off.add(d[1:])
                    continue
                ikn = d[9] | d[10] << 8
                k, ik = (ikn >> 4) & 15, (ikn >> 8) & 15
                if ik < k:
                    size = d[13] | d[14] << 8
                    sent[int.from_bytes(d[5:9], "little")] = d[17:17 + size]
        n = 0
        off_lens = {len(x) for x in off}
        for r in res:
            for payload, src in r["deliv"]:
                # FEC-off datagrams carry no checksum: the channel's corruption reaches their
                # payloads unseen, so they are only held to their lengths
                assert payload == sent.get(src) or payload in off or (src == 0 and len(payload) in off_lens)
                n += 1
        assert n == len([1 for r in res for _ in r["deliv"]]) and st["fec_src_count"] <= n


def test_product_fec_off_host_only():
    """libqfec's exact layer with FEC off needs no device: its datagrams and deliveries equal
    the oracle's, sequence for sequence."""
    import quicknet_amd as qa
    z = qa.Zfec()
    A = z.session(enabled=False)
    B = z.session(enabled=False)
    pay = _payloads(12, seed=7)
    for p in pay:
        z.pack_input(A, p)
    sent, got = z.flush()
    assert [d for s, d in sent if s == A] == [b"\x13" + p for p in pay] and not got
    for _, d in sent:
        z.unpack_input(B, d)
    z.unpack_input(B, b"\x00abc")  # any non-FEC tag: handed over minus its first byte
    sent2, got2 = z.flush()
    assert not sent2
    assert [(p, s) for _, p, s in got2] == [(p, 0) for p in pay] + [(b"abc", 0)]
    assert z.stats(A)["i_sent_pkt"] == 0  # FEC-off packets are not numbered (:90)
    z.close()


def test_product_rejects_bad_arguments():
    import quicknet_amd as qa
    z = qa.Zfec()
    s = z.session()
    with pytest.raises(qa.QfecError):
        z.set_kn(s, 12, 14)  # k > kmax: the reference would encode with stale rows
    with pytest.raises(qa.QfecError):
        z.pack_input(s + 5, b"x")
    with pytest.raises(qa.QfecError):
        z.session(kmax=0)
    z.close()


def test_oracle_is_test_only():
    """The product never imports the oracle."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for dirpath, _, files in os.walk(os.path.join(root, "quicknet_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hpp", ".hip")):
                assert "zfec_ref" not in open(os.path.join(dirpath, f), errors="ignore").read(), f
