// qfec_zfec.cpp -- network/NetFecCodec.cpp's FEC layer, exact, batched (include/qfec_zfec.h).
//
// The host runs the reference's state machines (bookkeeping only: sequence numbers, groups,
// the receive window, expected indices, used flags, codec lists); every byte of work is done
// by device launches over all sessions' packets of a flush:
//   send      qfec_pack_datagrams  (shards, payload checksums, headers, datagram checksums,
//                                   check packets), one launch per (k, n), the payloads read
//                                   where the input calls put them
//   receive   qfec_gather_rows + qfec_unpack_datagrams, two uses:
//             verdicts  the flush's datagrams placed by ik into pseudo-groups: header and
//                       shard checksum (unpack_fec_head, FecCodecBuf.cpp:334-411) and, for
//                       source packets, dec_src_pkt_info (:107-133)
//             decodes   each decode the state machine calls for (fec_decode_pkts on the first k
//                       valid packets, NetFecCodec.cpp:306) as one group holding exactly those k
//                       shards: fec_decode + dec_src_pkt_info of every data row
// A decode's inputs can depend on earlier decodes' verdicts (sorted mode resets delivered slots,
// :437), so the receive machine is replayed from the flush's starting state until every decode
// it calls for has a device result (one replay when no decoded packet fails its checksum).
//
// Memory: every queued payload and datagram is copied once, at its input call, into a pinned
// arena (one per direction).  A flush mirrors the arenas to the device in one copy each, the
// kernels read rows where they lie (payload offsets; gathered datagram rows), and every host
// structure refers to bytes by arena offset (plain values, no per-packet allocation).  At the
// end of a flush the bytes something still refers to -- the window slots' datagrams, the open
// send groups' payloads -- move to the other arena of the pair, and the rest is dropped.
// Sessions' send and receive machines run on several threads; the callbacks run in session
#include "qfec_zfec_impl.hpp"

using namespace qfec_zfec_impl;

extern "C" {

qfec_zfec* qfec_zfec_new(void) { return new (std::nothrow) qfec_zfec(); }

void qfec_zfec_free(qfec_zfec* z) {
    if (!z) return;
    for (auto& kv : z->codes) qfec_code_free(kv.second);
    for (auto* a : {&z->rx[0], &z->rx[1], &z->tx[0], &z->tx[1], &z->io}) a->release();
    for (auto* b : {&z->d_rx, &z->d_tx, &z->d_io, &z->d_work}) b->release();
    delete z;
}

int qfec_zfec_session(qfec_zfec* z, void* peer, int max_pkt_size, int buf_items, int kmax, int k, int n, int enabled,
                      int is_sorted) {
    if (!z || max_pkt_size < 1 || max_pkt_size > 60000 || buf_items < 1 || buf_items > 4096 || kmax < 1 || kmax > 15)
        return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(z->mu);
    Session S;
    S.peer = peer;
    S.max_pkt = max_pkt_size;
    S.kmax = kmax;
    init_rx(S.rx, buf_items, max_pkt_size, kmax);
    S.rx.is_sorted = true;  // init_zfec_layer :634, then enable_sorted_zfec below
    // FecTransmission::Init (FecTransmission.cpp:240-257): the candidate list, then (k, n)
    const int ka[8] = {2, 3, 5, 4, 3, 4, 5, 7}, na[8] = {4, 5, 8, 6, 4, 5, 6, 8};
    int rk, rn;
    for (int i = 0; i < 8; ++i) {
        S.tx.codecs.add(ka[i], na[i], &rk, &rn);
        S.tx.have_codec = true;
        S.tx.k = rk;
        S.tx.n = rn;
    }
    S.rx.codecs = S.tx.codecs;
    // the same set_zfec_kn(k, n) both sides see, then enable_zfec and enable_sorted_zfec,
    // queued like any later call
    Op o;
    o.t = OP_SETKN;
    o.a = k;
    o.b = n;
    o.c = 1;
    S.ops.push_back(o);
    Op e;
    e.t = OP_ENABLE;
    e.a = enabled ? 1 : 0;
    S.ops.push_back(e);
    Op so;
    so.t = OP_SORTED;
    so.a = is_sorted ? 1 : 0;
    S.ops.push_back(so);
    z->sessions.push_back(std::move(S));
    return (int)z->sessions.size() - 1;
}

static int push_op(qfec_zfec* z, int s, Op&& op) {
    if (!z) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(z->mu);
    if (s < 0 || s >= (int)z->sessions.size()) return QFEC_EINVAL;
    z->sessions[s].ops.push_back(std::move(op));
    return QFEC_OK;
}

int qfec_zfec_set_kn(qfec_zfec* z, int s, int k, int n, int add_new) {
    if (!z) return QFEC_EINVAL;
    if (k > 15 || n > 15) return -3;
    {
        std::lock_guard<std::mutex> lk(z->mu);
        if (s >= 0 && s < (int)z->sessions.size() && k > z->sessions[s].kmax) return -3;
    }
    Op o;
    o.t = OP_SETKN;
    o.a = k;
    o.b = n;
    o.c = add_new ? 1 : 0;
    return push_op(z, s, std::move(o));
}
int qfec_zfec_enable(qfec_zfec* z, int s, int on) {
    Op o;
    o.t = OP_ENABLE;
    o.a = on != 0;
    return push_op(z, s, std::move(o));
}
int qfec_zfec_sorted(qfec_zfec* z, int s, int on) {
    Op o;
    o.t = OP_SORTED;
    o.a = on != 0;
    return push_op(z, s, std::move(o));
}
int qfec_zfec_dynkn(qfec_zfec* z, int s, int on) {
    Op o;
    o.t = OP_DYNKN;
    o.a = on != 0;
    return push_op(z, s, std::move(o));
}
int qfec_zfec_lost_rate(qfec_zfec* z, int s, float lost) {
    Op o;
    o.t = OP_LOST;
    o.f = lost;
    return push_op(z, s, std::move(o));
}
// the bytes go straight into the direction's pinned arena (no per-packet allocation)
static int queue_bytes(qfec_zfec* z, int s, OpType t, const void* p, unsigned int size) {
    if (!z || (!p && size)) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(z->mu);
    if (s < 0 || s >= (int)z->sessions.size()) return QFEC_EINVAL;
    HostArena& A = t == OP_PACK ? z->tx[z->txc] : z->rx[z->rxc];
    Op o;
    o.t = t;
    o.size = size;
    if (!A.append(p, size, &o.off)) return QFEC_ENOMEM;
    if (t == OP_UNPACK) {
        o.uid = z->next_uid++;
        parse_head(o, static_cast<const uint8_t*>(p), size);
    }
    z->sessions[s].ops.push_back(o);
    return QFEC_OK;
}
int qfec_zfec_pack_input(qfec_zfec* z, int s, const void* data, unsigned int size) {
    return queue_bytes(z, s, OP_PACK, data, size);
}
int qfec_zfec_unpack_input(qfec_zfec* z, int s, const void* datagram, unsigned int size) {
    return queue_bytes(z, s, OP_UNPACK, datagram, size);
}

}  // extern "C"


extern "C" {

int qfec_zfec_stats(const qfec_zfec* z, int s, long long* out8) {
    if (!z || !out8 || s < 0 || s >= (int)z->sessions.size()) return QFEC_EINVAL;
    const Session& S = z->sessions[s];
    out8[0] = S.rx.fec_src_count;
    out8[1] = S.rx.fec_restore_count;
    out8[2] = S.tx.i_sent_pkt;
    out8[3] = S.rx.i_recv_pkt;
    out8[4] = S.rx.i_expected_packet;
    out8[5] = S.tx.k;
    out8[6] = S.tx.n;
    out8[7] = S.rx.undefined;
    return QFEC_OK;
}

}  // extern "C"

