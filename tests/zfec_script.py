"""Seeded send/receive scripts for the exact FEC layer (include/qfec_zfec.h), run through the
oracle's NetFecCodec restatement (oracle/zfec_ref.py) and through libqfec's batched layer.

A script drives one or more PAIRS: a sending layer A and a receiving layer B (one
NetFecCodecLayer each, FecTransmission::Init defaults unless the pair says otherwise).  It is
made of phases; in each phase A takes a run of operations (pack_input, and configuration
calls -- set_zfec_kn at group boundaries, enable_zfec, enable_zfec_dynkn, lost rates), then
the phase's datagrams cross a seeded lossy channel (drops, bursts, duplicates, reordering,
shard corruption, late arrivals carried into later phases) into B, with B's own configuration
calls (sorted mode, codec list) in between.

The channel decides on datagram INDICES, so the product, whose datagrams are checked equal to
the oracle's first, receives exactly the same bytes in the same order.
"""
import random

SENTINEL_SET_KN = "set_kn"
# pair configurations the product tests run side by side in one context
PAIRS = [dict(), dict(is_sorted=True), dict(k=3, n=5, buf_items=24), dict(k=7, n=8, kmax=12, is_sorted=True),
         dict(max_pkt_size=1400, k=2, n=4), dict(enabled=False, is_sorted=True)]


def make_script(seed, phases=8, pair=None, forge=True):
    """-> dict(config, phases=[dict(tx=[op], rx_cfg=[op], chan=[...])]); ops are tuples."""
    rng = random.Random(seed)
    cfg = dict(max_pkt_size=2048, buf_items=48, kmax=10, k=4, n=5, enabled=True, is_sorted=False)
    cfg.update(pair or {})
    out = []
    for p in range(phases):
        tx, rx_cfg = [], []
        for _ in range(rng.randint(3, 40)):
            r = rng.random()
            if r < 0.80:
                size = rng.choice([0, 1, 2, 3, 17, rng.randint(1, 300), rng.randint(300, 1400), cfg["max_pkt_size"]])
                tx.append(("pack", bytes(rng.getrandbits(8) for _ in range(size))))
            elif r < 0.88:
                k = rng.randint(1, min(7, cfg["kmax"]))
                n = rng.randint(k + 1, max(k + 1, min(cfg["kmax"], k + 4)))  # ik < kmax: no undefined decodes
                tx.append((SENTINEL_SET_KN, k, n, rng.random() < 0.9))
            elif r < 0.92:
                tx.append(("enable", rng.random() < 0.8))
            elif r < 0.96:
                tx.append(("dynkn", rng.random() < 0.6))
            else:
                tx.append(("lost_rate", rng.choice([0.0, 0.05, 0.15, 0.2, 0.3, 0.45, 0.6, 0.9])))
        if rng.random() < 0.2:
            rx_cfg.append(("sorted", rng.random() < 0.5))
        chan = dict(seed=rng.getrandbits(32), loss=rng.choice([0.0, 0.05, 0.2, 0.35]),
                    dup=rng.choice([0.0, 0.05]), swap=rng.choice([0.0, 0.1, 0.4]),
                    corrupt=rng.choice([0.0, 0.03]), late=rng.choice([0.0, 0.05]),
                    burst=rng.random() < 0.2, forge=rng.choice([0.0, 0.0, 0.1]) if forge else 0.0)
        out.append(dict(tx=tx, rx_cfg=rx_cfg, chan=chan))
    return dict(config=cfg, phases=out)


def channel(datagrams, chan, carry):
    """The datagrams B receives this phase: `carry` (late ones from earlier phases) is a list
    updated in place.  Decisions depend only on the seed and indices."""
    rng = random.Random(chan["seed"])
    got = []
    burst_at = rng.randint(0, max(0, len(datagrams) - 1)) if chan["burst"] else -1
    burst_len = rng.randint(2, 6)
    for i, d in enumerate(datagrams):
        if burst_at >= 0 and burst_at <= i < burst_at + burst_len:
            continue
        if rng.random() < chan["loss"]:
            continue
        if rng.random() < chan["corrupt"] and len(d) > 14:
            b = bytearray(d)
            j = rng.randint(13, len(b) - 1)  # shard bytes only: the datagram checksum catches it
            b[j] ^= 1 << rng.randint(0, 7)
            d = bytes(b)
        if rng.random() < chan.get("forge", 0.0) and len(d) > 16 and d[0] == 0xED:
            # a forged check packet: shard bytes changed and the datagram checksum recomputed,
            # so it passes unpack_fec_head and poisons its group's decode (check packets carry
            # no payload checksum); the decoded rows' size fields are then arbitrary
            ikn = d[9] | d[10] << 8
            if (ikn >> 8) & 15 >= (ikn >> 4) & 15:
                b = bytearray(d)
                b[13 + rng.randint(0, min(3, len(b) - 14))] ^= rng.randint(1, 255)
                cs = sum(b[13:]) & 0xFFFF
                b[11], b[12] = cs & 0xFF, cs >> 8
                d = bytes(b)
        if rng.random() < chan["late"]:
            carry.append(d)
            continue
        got.append(d)
        if rng.random() < chan["dup"]:
            got.append(d)
    for i in range(len(got) - 1):
        if rng.random() < chan["swap"]:
            got[i], got[i + 1] = got[i + 1], got[i]
    if carry and rng.random() < 0.5:
        got.extend(carry)
        carry.clear()
    return got


def run_oracle(script):
    """The reference's per-packet layers. -> per phase: (datagrams of A, deliveries of B),
    plus final stats of B, and the ops actually applied (set_kn kept only at group
    boundaries, where qfec_zfec's rule coincides with the reference's)."""
    from oracle.zfec_ref import ZfecLayer
    cfg = script["config"]
    A = ZfecLayer(**cfg)
    B = ZfecLayer(**cfg)
    carry, res, applied = [], [], []
    try:
        for ph in script["phases"]:
            a0, b0 = len(A.out), len(B.deliv)
            tx_ops = []
            for op in ph["tx"]:
                if op[0] == SENTINEL_SET_KN:
                    if (A.i_sent_pkt - A.i_cur_segment_beg) & 0xFFFFFFFF:
                        continue  # mid-group: skipped (documented difference)
                    A.set_kn(op[1], op[2], op[3])
                    B.set_kn(op[1], op[2], op[3])  # the receiver learns the same codec list
                elif op[0] == "pack":
                    A.pack_input(op[1])
                elif op[0] == "enable":
                    A.is_enabled = op[1]
                elif op[0] == "dynkn":
                    A.dynkn = op[1]
                elif op[0] == "lost_rate":
                    A.lost_rate = op[1]
                tx_ops.append(op)
            dgrams = A.out[a0:]
            rx = channel(dgrams, ph["chan"], carry)
            for op in ph["rx_cfg"]:
                B.is_sorted = op[1]
            for d in rx:
                B.unpack_input(d)
            res.append(dict(tx_ops=tx_ops, datagrams=list(dgrams), rx=rx, deliv=list(B.deliv[b0:])))
        stats = dict(fec_src_count=B.fec_src_count, fec_restore_count=B.fec_restore_count, i_recv_pkt=B.i_recv_pkt,
                     i_expected_packet=B.i_expected_packet, i_sent_pkt=A.i_sent_pkt)
    finally:
        A.close()
        B.close()
    return res, stats


def _queue_tx(z, A, B, ops):
    for op in ops:
        if op[0] == "pack":
            z.pack_input(A, op[1])
        elif op[0] == SENTINEL_SET_KN:
            z.set_kn(A, op[1], op[2], op[3])
            z.set_kn(B, op[1], op[2], op[3])
        elif op[0] == "enable":
            z.enable(A, op[1])
        elif op[0] == "dynkn":
            z.dynkn(A, op[1])
        elif op[0] == "lost_rate":
            z.lost_rate(A, op[1])


def _queue_rx(z, B, ph_script, ph_oracle):
    for op in ph_script["rx_cfg"]:
        z.sorted(B, op[1])
    for d in ph_oracle["rx"]:
        z.unpack_input(B, d)


def _split(items, sess):
    return [x[1:] if len(x) > 2 else x[1] for x in items if x[0] == sess]


def _check_stats(z, B, st):
    got = z.stats(B)
    for key in ("fec_src_count", "fec_restore_count", "i_recv_pkt", "i_expected_packet"):
        assert got[key] == st[key], key
    assert got["undefined"] == 0


def replay(z, scripts, oracles, mode):
    """Run `scripts` through the product layer `z` (one sender and one receiver session per
    script, all in z) and assert its sequences equal the oracle's `oracles` (run_oracle)."""
    sess = []
    for sc in scripts:
        c = sc["config"]
        args = (c["max_pkt_size"], c["buf_items"], c["kmax"], c["k"], c["n"], c["enabled"], c["is_sorted"])
        sess.append((z.session(*args), z.session(*args)))
    nph = len(scripts[0]["phases"])
    if mode == "one_flush":
        for (A, B), sc, (res, _) in zip(sess, scripts, oracles):
            for p in range(nph):
                _queue_tx(z, A, B, res[p]["tx_ops"])
                _queue_rx(z, B, sc["phases"][p], res[p])
        sent, got = z.flush()
        for (A, B), (res, st) in zip(sess, oracles):
            assert _split(sent, A) == [d for r in res for d in r["datagrams"]]
            assert _split(got, B) == [d for r in res for d in r["deliv"]]
            assert not _split(sent, B) and not _split(got, A)
            _check_stats(z, B, st)
    else:
        for p in range(nph):
            for (A, B), (res, _) in zip(sess, oracles):
                _queue_tx(z, A, B, res[p]["tx_ops"])
            sent, got = z.flush()
            assert not got
            for (A, B), sc, (res, _) in zip(sess, scripts, oracles):
                assert _split(sent, A) == res[p]["datagrams"], (p, A)
                _queue_rx(z, B, sc["phases"][p], res[p])
            sent, got = z.flush()
            assert not sent
            for (A, B), (res, _) in zip(sess, oracles):
                assert _split(got, B) == res[p]["deliv"], (p, B)
        for (A, B), (_, st) in zip(sess, oracles):
            _check_stats(z, B, st)
