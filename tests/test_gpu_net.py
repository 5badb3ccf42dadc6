"""GPU tests of the batched NetFecCodec layer (include/qfec_net.h, quicknet_amd.NetFec):
sessions keep zfec_pack_input's numbering (network/NetFecCodec.cpp:68-175) and the wire bytes
equal the oracle's restatement of the per-packet path (itself pinned to the reference's
FecCodecBuf.cpp by tests/golden/wire.npz); the receive side delivers exactly the packets
zfec_unpack_input would (every source packet of a decodable group, else the received valid
ones), with their source indices."""
import numpy as np
import pytest

import quicknet_amd as qa

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)


def full_matrix(k, n):
    return np.concatenate([np.eye(k, dtype=np.uint8), qa.Code.vandermonde(k, n - k).rows])


@pytest.mark.parametrize("k,n,checksum", [(4, 6, True), (10, 13, True), (3, 5, False)])
def test_send_matches_per_packet_path(oracle, k, n, checksum):
    rng = np.random.default_rng(k + n)
    net = qa.NetFec(k, n, max_pkt_size=1400, checksum=checksum)
    S = [net.session() for _ in range(3)]
    sent = {s: [] for s in S}
    order = []
    for _ in range(3 * k * 5 + 2):  # 5 full groups per session plus a partial one
        s = int(rng.choice(S))
        p = rng.integers(0, 256, size=int(rng.integers(0, 1401)), dtype=np.uint8).tobytes()
        net.pack_input(s, p)
        sent[s].append(p)
        order.append(s)
    out = net.flush_pack()
    got = {s: [d for (ss, d) in out if ss == s] for s in S}
    full = full_matrix(k, n)
    for s in S:
        groups = len(sent[s]) // k
        assert len(got[s]) == groups * n
        for g in range(groups):
            pl = sent[s][g * k:(g + 1) * k]
            payload = np.frombuffer(b"".join(pl) + bytes(16), np.uint8)
            sizes = np.array([len(x) for x in pl], np.int32)
            offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
            ref, ln, _ = oracle.pack_group(k, n, full, payload, offs, sizes, g * n, g * k, int(checksum), pitch=1440)
            for j in range(n):
                assert got[s][g * n + j] == ref[j, :ln[j]].tobytes(), (s, g, j)
    # the open groups continue the numbering at the next flush
    for s in S:
        while len(sent[s]) % k:
            p = bytes([len(sent[s]) & 255]) * 7
            net.pack_input(s, p)
            sent[s].append(p)
    out2 = net.flush_pack()
    for s in S:
        mine = [d for (ss, d) in out2 if ss == s]
        g = len(sent[s]) // k - 1
        if mine:
            hdr = np.frombuffer(mine[0][:9], np.uint8)
            assert int.from_bytes(hdr[1:5].tobytes(), "little") == g * n
            assert int.from_bytes(hdr[5:9].tobytes(), "little") == g * k
    st = net.stats()
    assert st["datagrams_out"] == len(out) + len(out2)


def test_receive_delivers_what_the_reference_would():
    k, n = 4, 6
    rng = np.random.default_rng(11)
    tx = qa.NetFec(k, n, max_pkt_size=1400)
    S = [tx.session() for _ in range(3)]
    sent = {s: [] for s in S}
    for _ in range(8):  # 8 groups per session
        for s in S:
            for _ in range(k):
                p = rng.integers(0, 256, size=int(rng.integers(1, 1401)), dtype=np.uint8).tobytes()
                tx.pack_input(s, p)
                sent[s].append(p)
    out = tx.flush_pack()
    per = {s: [d for (ss, d) in out if ss == s] for s in S}
    rx = qa.NetFec(k, n, max_pkt_size=1400)
    R = [rx.session() for _ in S]
    expect = {s: [] for s in S}
    feed = []
    for s in S:
        for g in range(8):
            dg = per[s][g * n:(g + 1) * n]
            nlost = int(rng.integers(0, n - k + 2))          # up to m + 1 lost
            lost = set(rng.choice(n, nlost, replace=False).tolist())
            bad = None
            if g % 3 == 0:                                    # one corrupted datagram
                cand = [j for j in range(n) if j not in lost]
                bad = int(rng.choice(cand))
            valid = [j for j in range(n) if j not in lost and j != bad]
            for j in range(n):
                if j in lost:
                    continue
                d = bytearray(dg[j])
                if j == bad:
                    d[-1] ^= 0x5A
                feed.append((s, bytes(d)))
            src0 = g * k
            if len(valid) >= k:
                expect[s] += [(sent[s][g * k + i], src0 + i) for i in range(k)]
            else:
                expect[s] += [(sent[s][g * k + i], src0 + i) for i in range(k) if i in valid]
    order = rng.permutation(len(feed))
    for i in order:
        s, d = feed[i]
        assert rx.unpack_input(R[S.index(s)], d) == 1
    got = rx.flush_unpack(all_groups=True)
    for s in S:
        mine = [(p, src) for (ss, p, src) in got if ss == R[S.index(s)]]
        assert mine == expect[s], s
    # a datagram for a group already delivered is late
    assert rx.unpack_input(R[0], per[S[0]][0]) == 0
    assert rx.stats()["late"] == 1


def test_receive_groups_of_several_codes():
    """One receiving handle decodes groups of any (k, n) its headers name (the reference looks
    the codec up per header, NetFecCodec.cpp:301), next to FEC-off datagrams of the same
    session, which it hands over first with source index 0 (:200-209)."""
    rng = np.random.default_rng(3)
    codes = [(4, 6), (3, 5), (10, 13), (7, 8)]
    rx = qa.NetFec(10, 13, max_pkt_size=1400)
    sessions = [rx.session() for _ in codes]  # numbering is per session: one sender stream each
    expect = []
    for (k, n), r in zip(codes, sessions):
        tx = qa.NetFec(k, n, max_pkt_size=1400)
        s = tx.session()
        sent = [rng.integers(0, 256, size=int(rng.integers(0, 1401)), dtype=np.uint8).tobytes()
                for _ in range(3 * k)]
        for p in sent:
            tx.pack_input(s, p)
        dg = [d for _, d in tx.flush_pack()]
        for g in range(3):
            lost = set(rng.choice(n, n - k, replace=False).tolist())  # exactly k of n arrive
            for j in range(n):
                if j not in lost:
                    assert rx.unpack_input(r, dg[g * n + j]) == 1
        expect.append([(p, i) for i, p in enumerate(sent)])
    assert rx.unpack_input(sessions[0], b"\x13plain") == 1
    got = rx.flush_unpack()
    assert got[0] == (sessions[0], b"plain", 0)
    for r, exp in zip(sessions, expect):
        assert [(p, src) for (ss, p, src) in got[1:] if ss == r] == exp
