// qfec_zfec.cpp -- network/NetFecCodec.cpp's FEC layer, exact, batched (include/qfec_zfec.h).
//
// The host runs the reference's state machines (bookkeeping only: sequence numbers, groups,
// the receive window, expected indices, used flags, codec lists); every byte of work is done
// by device launches over all sessions' packets of a flush:
//   send      qfec_pack_datagrams  (shards, payload checksums, headers, datagram checksums,
//                                   check packets), one launch per (k, n)
//   receive   qfec_unpack_datagrams, two uses:
//             verdicts  the flush's datagrams placed by ik into pseudo-groups: header and
//                       shard checksum (unpack_fec_head, FecCodecBuf.cpp:334-411) and, for
//                       source packets, dec_src_pkt_info (:107-133)
//             decodes   each decode the state machine calls for (fec_decode_pkts on the first k
//                       valid packets, NetFecCodec.cpp:306) as one group holding exactly those k
//                       shards: fec_decode + dec_src_pkt_info of every data row
// A decode's inputs can depend on earlier decodes' verdicts (sorted mode resets delivered slots,
// :437), so the receive machine is replayed from the flush's starting state until every decode
// it calls for has a device result (one replay when no decoded packet fails its checksum).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

#include "../../include/qfec.h"
#include "../../include/qfec_zfec.h"

namespace {

inline size_t round16(size_t x) { return (x + 15) & ~(size_t)15; }
inline uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
inline int packed_size(int size) { return size < 0 ? 0 : size + 4 + 12 + 4; }  // getPackedPktSize, FecCodecBuf.cpp:16-25
inline int cmod(int a, int b) { return a % b; }                                   // C's % (truncating), as in :277

// ---- FecCodecList: std::map<float 1 - k/n, FecCodec*> (FecCodec.cpp:18-95)
struct CodecEntry {
    float key;
    int k, n;
    bool null;  // add_new_codec deleted it and std::map::insert did not replace it (:86-93)
};
struct CodecList {
    std::vector<CodecEntry> e;  // kept sorted by key (std::map order)
    const CodecEntry* find(int k, int n) const {  // find_codec (:18-34)
        for (auto& c : e)
            if (!c.null && c.k == k && c.n == n) return &c;
        return nullptr;
    }
    // add_new_codec (:77-95): the new item is returned; the map keeps it only for a new key
    void add(int k, int n, int* rk, int* rn) {
        const float key = 1.0f - float(k) / float(n);
        for (auto& c : e)
            if (c.key == key) {
                c.null = true;
                *rk = k;
                *rn = n;
                return;
            }
        e.push_back(CodecEntry{key, k, n, false});
        std::sort(e.begin(), e.end(), [](const CodecEntry& a, const CodecEntry& b) { return a.key < b.key; });
        *rk = k;
        *rn = n;
    }
    const CodecEntry* by_lost(float lost) const {  // get_codec_by (:36-72); NULL entries count
        if (e.empty()) return nullptr;
        float last_rate = 0.0f;
        const CodecEntry* last = nullptr;
        for (size_t i = 0; i < e.size(); ++i) {
            const CodecEntry* it = e[i].null ? nullptr : &e[i];
            if (i == 0) {
                if (lost >= last_rate && lost <= e[i].key && it) return it;
            } else if (lost > last_rate && lost <= e[i].key && it) {
                return it;
            }
            last_rate = e[i].key;
            last = it;
        }
        return last;
    }
};

// ---- one dec_pkts_buf entry (FecPacket.h): its FecBuf allocation is modelled byte for byte
// (MaxBufSize bytes), since dec_src_pkt_info may read past BufSize of a stale copy
struct Slot {
    int64_t iPacket = -1;
    std::vector<uint8_t> fec_buf;
    int BufSize = 0;
    bool bValid = false;
    int MaxBufSize = 0;
    bool bSourcePkt = true;
    uint32_t i_source_pkt = 0;
    bool bUsed = false;
    uint64_t uid = 0;   // which received datagram filled it (decode cache key)
    int ik = 0;         // the ik it was received with
    // dec_src_pkt_info's result on it, from the device verdict when it was received: only
    // source packets that passed it are stored (NetFecCodec.cpp:240-245), and a later
    // flush_avail_pkts check (:421) sees the same bytes under a dec_pkt_size that only grew
    std::vector<uint8_t> payload;
    void resize(int n) { fec_buf.resize((size_t)n, 0); }
    void set_packet(const uint8_t* p, int size, uint64_t id, int row, const std::vector<uint8_t>& pay) {  // SetPacket (:78-98)
        if (size > MaxBufSize) MaxBufSize = size;
        resize(MaxBufSize);
        std::fill(fec_buf.begin(), fec_buf.end(), 0);
        if (size) memcpy(fec_buf.data(), p, (size_t)size);
        BufSize = size;
        bValid = true;
        bUsed = false;
        uid = id;
        ik = row;
        payload = pay;
    }
    void reset(int max_size) {  // Reset (:99-122)
        iPacket = -1;
        BufSize = 0;
        resize(max_size);
        std::fill(fec_buf.begin(), fec_buf.end(), 0);
        MaxBufSize = max_size;
        bValid = false;
        bUsed = false;
    }
    void assign(const Slot& o) {  // operator= (:42-68): o's first BufSize bytes only
        iPacket = o.iPacket;
        MaxBufSize = o.MaxBufSize;
        resize(MaxBufSize);
        if (o.BufSize) memcpy(fec_buf.data(), o.fec_buf.data(), (size_t)o.BufSize);
        BufSize = o.BufSize;
        bValid = o.bValid;
        bSourcePkt = o.bSourcePkt;
        i_source_pkt = o.i_source_pkt;
        bUsed = o.bUsed;
        uid = o.uid;
        ik = o.ik;
        payload = o.payload;
    }
};

// receive state of one NetFecCodecLayer plus the FecCodecBuf fields its decisions read
struct RxState {
    std::vector<Slot> slots;
    uint32_t first = 0, second = 0;  // dec_buf_ipkt_range
    uint32_t i_recv_pkt = 0, i_expected_packet = 0;
    bool is_sorted = false;
    long long fec_src_count = 0, fec_restore_count = 0, undefined = 0;
    int dec_pkt_size = 0, dec_kmax = 0;  // FecCodecBuf (grow-only, realloc_fec_buf :506-640)
    bool is_checksum = false;            // set by every FEC datagram's tag (unpack_fec_head)
    CodecList codecs;                    // the receive side's view of the session's list
};

enum OpType { OP_PACK, OP_UNPACK, OP_SETKN, OP_ENABLE, OP_SORTED, OP_DYNKN, OP_LOST };
struct Op {
    OpType t;
    std::vector<uint8_t> data;
    int a = 0, b = 0, c = 0;
    float f = 0;
};

// send state (zfec_pack_input) and the open group carried across flushes
struct TxState {
    uint32_t i_sent_pkt = 0, i_sent_src_pkt = 0, i_cur_segment_beg = 0;
    bool enabled = false, dynkn = false;
    float lost_rate = 0.20f;
    bool have_codec = false;
    int k = 0, n = 0;  // fec_codec
    CodecList codecs;
    // the open group: (k, n) it started with, first indices, payloads so far, rows emitted
    int gk = 0, gn = 0;
    uint32_t g_sent0 = 0, g_src0 = 0;
    std::vector<std::vector<uint8_t>> g_pay;
    int g_emitted = 0;
};

struct Session {
    void* peer = nullptr;
    int max_pkt = 0, kmax = 0;
    TxState tx;
    RxState rx;
    std::vector<Op> ops;
};

// an output of one op, filled in after the device work
struct Emit {
    int kind = 0;        // 0 datagram from a send batch, 1 plain bytes, 2 delivery (bytes + src)
    int batch = -1, row = 0;
    long long group = 0;
    std::vector<uint8_t> bytes;
    uint32_t src = 0;
};

}  // namespace

struct qfec_zfec {
    std::mutex mu;
    std::vector<Session> sessions;
    std::map<std::pair<int, int>, qfec_code*> codes;  // (k, n) -> fec_new(k, n) matrix on the device
    uint64_t next_uid = 1;
};

namespace {

qfec_code* code_for(qfec_zfec* z, int k, int n) {
    qfec_code*& c = z->codes[std::make_pair(k, n)];
    if (!c) c = qfec_code_new(QFEC_VANDERMONDE, k, n - k);  // fec_new(k, n), FecCodec.cpp:84
    return c;
}

// ---------------------------------------------------------------- device batches
struct HostDev {
    std::vector<uint8_t> h;
    void* d = nullptr;
    size_t cap = 0;
    bool ensure(size_t bytes) {
        if (bytes <= cap) return true;
        if (d) (void)hipFree(d);
        d = nullptr;
        cap = 0;
        if (hipMalloc(&d, bytes + 4096) != hipSuccess) return false;
        cap = bytes + 4096;
        return true;
    }
    ~HostDev() {
        if (d) (void)hipFree(d);
    }
};

// send: complete or partial groups of one (k, n); payloads of missing rows are empty
struct PackGroup {
    uint32_t sent0, src0;
    std::vector<const std::vector<uint8_t>*> pay;  // k entries (nullptr = not yet given)
};
struct PackBatch {
    int k, n;
    std::vector<PackGroup> groups;
    std::vector<uint8_t> wire;   // results: [G][n][wp]
    std::vector<int> wlen;
    size_t wp = 0;
};

int run_pack(qfec_zfec* z, PackBatch& b, hipStream_t s) {
    const size_t G = b.groups.size();
    if (!G) return 0;
    size_t maxp = 1, total = 0;
    for (auto& g : b.groups)
        for (auto* p : g.pay)
            if (p) {
                maxp = std::max(maxp, p->size());
                total += p->size();
            }
    const size_t sp = round16(maxp + 4), wp = round16(sp + 13);
    std::vector<uint8_t> payload(round16(total + 16), 0);
    std::vector<long long> offs(G * b.k);
    std::vector<int> sizes(G * b.k);
    std::vector<uint32_t> seq(2 * G);
    size_t o = 0;
    for (size_t g = 0; g < G; ++g) {
        seq[2 * g] = b.groups[g].sent0;
        seq[2 * g + 1] = b.groups[g].src0;
        for (int i = 0; i < b.k; ++i) {
            const std::vector<uint8_t>* p = b.groups[g].pay[i];
            offs[g * b.k + i] = (long long)o;
            sizes[g * b.k + i] = p ? (int)p->size() : 0;
            if (p && !p->empty()) memcpy(payload.data() + o, p->data(), p->size());
            o += p ? p->size() : 0;
        }
    }
    HostDev dp, da, dsh, dw, dl;
    const size_t ob = offs.size() * 8, zb = sizes.size() * 4, qb = seq.size() * 4;
    if (!dp.ensure(payload.size()) || !da.ensure(ob + zb + qb) || !dsh.ensure(G * b.n * sp) || !dw.ensure(G * b.n * wp) ||
        !dl.ensure(G * b.n * 4))
        return QFEC_ENOMEM;
    uint8_t* a = static_cast<uint8_t*>(da.d);
    if (hipMemcpyAsync(dp.d, payload.data(), payload.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(a, offs.data(), ob, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(a + ob, sizes.data(), zb, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(a + ob + zb, seq.data(), qb, hipMemcpyHostToDevice, s) != hipSuccess)
        return QFEC_EHIP;
    int rc = qfec_pack_datagrams(code_for(z, b.k, b.n), static_cast<unsigned char*>(dp.d),
                                 reinterpret_cast<const long long*>(a), reinterpret_cast<const int*>(a + ob),
                                 reinterpret_cast<const unsigned int*>(a + ob + zb), (long long)G, 1 /* is_send_checksum */,
                                 static_cast<unsigned char*>(dsh.d), (long long)sp, static_cast<unsigned char*>(dw.d),
                                 (long long)wp, static_cast<int*>(dl.d), s);
    if (rc) return rc;
    b.wire.resize(G * b.n * wp);
    b.wlen.resize(G * b.n);
    b.wp = wp;
    if (hipMemcpyAsync(b.wire.data(), dw.d, b.wire.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(b.wlen.data(), dl.d, b.wlen.size() * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return QFEC_EHIP;
    return 0;
}

// receive: pseudo-groups of wire rows (datagrams, or 0xEC-wrapped shards for decodes)
struct UnpackRow {
    int group, ik;
    std::vector<uint8_t> bytes;  // the datagram
};
struct UnpackBatch {
    int k, n, checksum, dec_pkt_size;
    int groups = 0;
    std::vector<UnpackRow> rows;
    // results
    std::vector<uint8_t> shards;  // [G][n][sp]
    std::vector<int> rx, status, psize;
    size_t sp = 0;
};

int run_unpack(qfec_zfec* z, UnpackBatch& b, hipStream_t s) {
    const size_t G = (size_t)b.groups;
    if (!G) return 0;
    size_t maxd = 16;
    for (auto& r : b.rows) maxd = std::max(maxd, r.bytes.size());
    // shard rows hold any datagram's shard and dec_pkt_size + 4 bytes, so dec_src_pkt_info's
    // reads stay inside the row (the reference's buffers are dec_pkt_size long, zero-filled)
    const size_t sp = round16(std::max(maxd, (size_t)b.dec_pkt_size + 4)), wp = round16(sp + 13);
    std::vector<uint8_t> wire(G * b.n * wp, 0);
    std::vector<int> wlen(G * b.n, 0);
    for (auto& r : b.rows) {
        memcpy(wire.data() + ((size_t)r.group * b.n + r.ik) * wp, r.bytes.data(), r.bytes.size());
        wlen[(size_t)r.group * b.n + r.ik] = (int)r.bytes.size();
    }
    HostDev dw, dl, dsh, dsm;
    const size_t smb = round16(G * b.n) + (G * b.n + 2 * G * b.k) * 4;
    if (!dw.ensure(wire.size()) || !dl.ensure(wlen.size() * 4) || !dsh.ensure(G * b.n * sp) || !dsm.ensure(smb))
        return QFEC_ENOMEM;
    uint8_t* marks = static_cast<uint8_t*>(dsm.d);
    int* rx = reinterpret_cast<int*>(marks + round16(G * b.n));
    int* st = rx + G * b.n;
    int* ps = st + G * b.k;
    if (hipMemcpyAsync(dw.d, wire.data(), wire.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(dl.d, wlen.data(), wlen.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess)
        return QFEC_EHIP;
    int rc = qfec_unpack_datagrams(code_for(z, b.k, b.n), static_cast<unsigned char*>(dw.d), (long long)wp,
                                   static_cast<int*>(dl.d), (long long)G, b.checksum, b.dec_pkt_size,
                                   static_cast<unsigned char*>(dsh.d), (long long)sp, marks, rx, st, ps, s);
    if (rc) return rc;
    b.shards.resize(G * b.n * sp);
    b.rx.resize(G * b.n);
    b.status.resize(G * b.k);
    b.psize.resize(G * b.k);
    b.sp = sp;
    if (hipMemcpyAsync(b.shards.data(), dsh.d, b.shards.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(b.rx.data(), rx, b.rx.size() * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(b.status.data(), st, b.status.size() * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(b.psize.data(), ps, b.psize.size() * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return QFEC_EHIP;
    return 0;
}

// ---------------------------------------------------------------- receive verdicts and decodes
struct Verdict {  // of one received FEC datagram
    bool fec = false;      // tag 0xEC / 0xED and size >= 11
    bool ok = false;       // unpack_fec_head returned the shard (header + shard checksum)
    bool usable = false;   // a header qfec_zfec can check (1 <= k < n <= 15, ik < n)
    std::vector<uint8_t> shard;  // the unpacked shard (after header and checksum)
    bool src_ok = false;   // dec_src_pkt_info on it (source packets)
    int src_size = 0;      // its size field
    std::vector<uint8_t> payload;
};

struct DecodeKey {
    int session, k, n, mode, dec_pkt_size;
    std::vector<std::pair<uint64_t, int>> rows;  // (slot uid, ik) in iValid order
    bool operator<(const DecodeKey& o) const {
        return std::tie(session, k, n, mode, dec_pkt_size, rows) < std::tie(o.session, o.k, o.n, o.mode, o.dec_pkt_size, o.rows);
    }
};
struct DecodeOut {
    bool ok[16] = {};
    std::vector<uint8_t> payload[16];
};
struct DecodeReq {
    DecodeKey key;
    std::vector<std::pair<std::vector<uint8_t>, int>> shards;  // (shard bytes, ik)
};

struct RxPass {
    std::map<DecodeKey, DecodeOut>* cache;
    std::vector<DecodeReq>* missing;
    bool emit;
};

// the receive side of one session over its queued ops (NetFecCodec.cpp:189-371)
class RxMachine {
   public:
    RxMachine(Session& S, int sidx, const std::vector<Verdict>& verd, RxPass& pass, std::vector<std::vector<Emit>>& out)
        : S(S), R(S.rx), sidx(sidx), verd(verd), pass(pass), out(out) {}

    void run() {
        size_t v = 0;
        for (size_t oi = 0; oi < S.ops.size(); ++oi) {
            const Op& op = S.ops[oi];
            cur = &out[oi];
            if (op.t == OP_UNPACK) unpack(op, verd[v++]);
            else if (op.t == OP_SETKN) set_kn(op.a, op.b, op.c != 0);
            else if (op.t == OP_SORTED) R.is_sorted = op.a != 0;
        }
    }

   private:
    Session& S;
    RxState& R;
    int sidx;
    const std::vector<Verdict>& verd;
    RxPass& pass;
    std::vector<std::vector<Emit>>& out;
    std::vector<Emit>* cur = nullptr;

    void deliver(const uint8_t* p, size_t n, uint32_t src) {
        if (!pass.emit) return;
        Emit e;
        e.kind = 2;
        e.bytes.assign(p, p + n);
        e.src = src;
        cur->push_back(std::move(e));
    }
    void set_kn(int k, int n, bool add) {  // the receive side's codec list (find_codec at :301)
        if (k < 0 || n < 0 || k > n) return;
        if (!R.codecs.find(k, n) && add) {
            int a, b;
            R.codecs.add(k, n, &a, &b);
        }
    }
    bool used(uint32_t i) const {  // is_fec_dec_buf_used :556-564
        return i >= R.first && i < R.second ? R.slots[i - R.first].bUsed : false;
    }
    void set_used(uint32_t i, bool u) {  // :566-572
        if (i >= R.first && i < R.second) R.slots[i - R.first].bUsed = u;
    }
    void update_window(uint32_t seg_beg, int n) {  // update_fec_dec_buf :540-554
        const uint32_t end = seg_beg + (uint32_t)n;
        if (end > R.second) {
            const int ns = (int)(end - R.second);
            const int span = (int)(R.second - R.first);
            for (int is = ns; is < span; ++is) {
                R.slots[is - ns].assign(R.slots[is]);
                R.slots[is].reset(R.slots[is].MaxBufSize);
            }
            R.first += (uint32_t)ns;
            R.second += (uint32_t)ns;
        }
    }
    bool flush_avail(uint32_t lastis, uint32_t lastie) {  // flush_avail_pkts :407-443
        bool ret = false;
        if (lastie > lastis && lastis >= R.first && lastis < R.second && lastie > R.first && lastie <= R.second) {
            for (uint32_t i = lastis; i < lastie; ++i) {
                Slot& s = R.slots[i - R.first];
                if (s.bValid && s.bSourcePkt) {  // (a stored source packet passed dec_src_pkt_info)
                    if (!used(i)) {
                        R.fec_src_count++;
                        deliver(s.payload.data(), s.payload.size(), s.i_source_pkt);
                        set_used(i, true);
                    }
                    s.reset(s.MaxBufSize);
                    ret = true;
                }
            }
        }
        return ret;
    }
    // add_packet_fec_buf :485-535; fills `rows` with the first k valid slots (iValid order)
    bool add_packet(uint32_t ipkt, uint32_t isrc, const Verdict& vd, uint64_t uid, int ik, int k, int n,
                    uint32_t seg_beg, int* max_size, std::vector<int>* rows, bool* undefined) {
        if (ipkt >= R.first && ipkt < R.second) {
            Slot& s = R.slots[ipkt - R.first];
            s.set_packet(vd.shard.data(), (int)vd.shard.size(), uid, ik, vd.payload);
            s.iPacket = (int64_t)ipkt;
            s.bSourcePkt = ipkt - seg_beg < (uint32_t)k;
            s.i_source_pkt = isrc;
        } else {
            return false;
        }
        int valid = 0;
        bool all_src = true;
        *undefined = false;
        rows->clear();
        for (int i = 0; valid < k && i < n; ++i) {
            const int ck = (int)(seg_beg - R.first + (uint32_t)i);
            if (ck < 0 || ck >= (int)R.slots.size()) continue;
            const Slot& s = R.slots[ck];
            if (s.bValid && s.iPacket == (int64_t)(uint32_t)(seg_beg + (uint32_t)i)) {
                // set_fec_dec_buf (FecCodecBuf.cpp:160-178): grows dec_pkt_size / dec_kmax, and
                // leaves the decoder slot unset for an index or ik >= dec_kmax (undefined decode);
                // realloc_fec_buf returns early for a zero size (:508-511)
                if (i > R.dec_kmax && s.BufSize > 0) R.dec_kmax = i;
                if (s.BufSize > R.dec_pkt_size) R.dec_pkt_size = s.BufSize;
                if (valid >= R.dec_kmax || i >= R.dec_kmax) *undefined = true;
                rows->push_back(ck);
                *max_size = valid == 0 ? s.BufSize : std::max(*max_size, s.BufSize);
                ++valid;
                if (ck >= k) all_src = false;  // (sic: the window index, :523)
            }
        }
        return valid == k && !all_src;
    }

    void unpack(const Op& op, const Verdict& vd) {  // zfec_unpack_input :189-371
        const uint8_t* d = op.data.data();
        const uint32_t size = (uint32_t)op.data.size();
        if (size > (uint32_t)R.dec_pkt_size) R.dec_pkt_size = (int)size;  // unpack_fec_head realloc (:345-352)
        if (!vd.fec) {  // not an FEC datagram: handed over minus its tag, source index 0 (:201-209)
            if (size >= 1) deliver(d + 1, size - 1, 0u);
            return;
        }
        R.is_checksum = d[0] == 0xED;  // (:364)
        if (!vd.ok || !vd.usable) return;  // (:210-213)
        const uint32_t i_recv = rd32(d + 1), src = rd32(d + 5);
        const uint32_t ikn = (uint32_t)d[9] | (uint32_t)d[10] << 8;
        const int cur_n = (int)(ikn & 0xF), cur_k = (int)((ikn >> 4) & 0xF), cur_ni = (int)((ikn >> 8) & 0xF);
        const uint32_t seg_beg = i_recv - (uint32_t)cur_ni;
        R.i_recv_pkt = std::max(i_recv, R.i_recv_pkt);
        const uint32_t seg_src_beg = cur_ni < cur_k ? src - (uint32_t)cur_ni : src - (uint32_t)cur_k + 1u;
        update_window(seg_beg, cur_n);
        bool bused = false;
        if (cur_ni < cur_k) {  // a source packet (:238-283)
            if (!vd.src_ok || vd.src_size >= R.dec_pkt_size) return;  // dec_src_pkt_info NULL: dropped
            if (!R.is_sorted) {
                if (!used(i_recv)) {
                    R.fec_src_count++;
                    deliver(vd.payload.data(), vd.payload.size(), seg_src_beg + (uint32_t)cur_ni);
                }
                bused = true;
            }
            if (i_recv == R.i_expected_packet && R.is_sorted) {
                R.fec_src_count++;
                deliver(vd.payload.data(), vd.payload.size(), seg_src_beg + (uint32_t)cur_ni);
                bused = true;
                R.i_expected_packet++;
                if (cmod((int)(R.i_expected_packet - seg_beg), cur_n) == cur_k) R.i_expected_packet = seg_beg + (uint32_t)cur_n;
            }
        }
        int max_size = 0;
        std::vector<int> rows;
        bool undefined = false;
        const bool dec = add_packet(i_recv, src, vd, (uint64_t)(uint32_t)op.b << 32 | (uint32_t)op.c, cur_ni, cur_k,
                                    cur_n, seg_beg, &max_size, &rows, &undefined);
        set_used(i_recv, bused);
        if (!dec && i_recv - R.i_expected_packet >= (uint32_t)(2 * cur_n) && R.is_sorted) {  // :289-293
            flush_avail(R.i_expected_packet, seg_beg);
            R.i_expected_packet = seg_beg;
        }
        if (!dec) return;
        if (R.is_sorted) flush_avail(R.i_expected_packet, seg_beg);  // :296-299
        if (!R.codecs.find(cur_k, cur_n)) return;                     // :301-305
        // a decoder slot the reference leaves unset (its fec_decode reads a stale buffer), or
        // fec_decode_pkts refusing maxSize <= 0 (FecCodecBuf.cpp:200) and delivering stale buffers
        if (undefined || max_size <= 0) {
            R.undefined++;
            return;
        }
        // fec_decode_pkts on the first k valid packets (:306): a device result, by content
        DecodeKey key;
        key.session = sidx;
        key.k = cur_k;
        key.n = cur_n;
        key.mode = R.is_checksum ? 1 : 0;
        key.dec_pkt_size = R.dec_pkt_size;
        for (int ck : rows) key.rows.emplace_back(R.slots[ck].uid, R.slots[ck].ik);
        auto it = pass.cache->find(key);
        const DecodeOut* res = it == pass.cache->end() ? nullptr : &it->second;
        if (!res) {
            DecodeReq q;
            q.key = key;
            for (int ck : rows)
                q.shards.emplace_back(std::vector<uint8_t>(R.slots[ck].fec_buf.begin(),
                                                           R.slots[ck].fec_buf.begin() + R.slots[ck].BufSize),
                                      R.slots[ck].ik);
            pass.missing->push_back(std::move(q));
        }
        for (int i = 0; i < cur_k; ++i) {  // :308-366
            // an unknown result counts as a good packet for this pass (it is not emitted)
            if (res && !res->ok[i]) continue;
            const uint32_t pk = seg_beg + (uint32_t)i;
            if (!R.is_sorted) {
                if (!used(pk)) {
                    if (res) deliver(res->payload[i].data(), res->payload[i].size(), seg_src_beg + (uint32_t)i);
                    set_used(pk, true);
                    R.fec_src_count++;
                    R.fec_restore_count++;
                }
            }
            if (pk >= R.i_expected_packet && R.is_sorted) {
                if (!used(pk)) {
                    if (res) deliver(res->payload[i].data(), res->payload[i].size(), seg_src_beg + (uint32_t)i);
                    set_used(pk, true);
                    R.fec_src_count++;
                    R.fec_restore_count++;
                }
                R.i_expected_packet = seg_beg + (uint32_t)i + 1u;
                if (cmod((int)(R.i_expected_packet - seg_beg), cur_n) == cur_k) R.i_expected_packet = seg_beg + (uint32_t)cur_n;
            }
            set_used(i_recv, bused);
        }
    }
};

void init_rx(RxState& R, int max_pkt, int buf_items, int kmax) {
    R.slots.assign((size_t)buf_items, Slot());
    for (auto& s : R.slots) s.reset(max_pkt + 16);  // init_zfec_layer :653-664
    R.first = 0;
    R.second = (uint32_t)buf_items;
    R.dec_pkt_size = packed_size(max_pkt);  // init_fec_buf :433-434
    R.dec_kmax = kmax;
    R.is_checksum = false;
}

}  // namespace

extern "C" {

qfec_zfec* qfec_zfec_new(void) { return new (std::nothrow) qfec_zfec(); }

void qfec_zfec_free(qfec_zfec* z) {
    if (!z) return;
    for (auto& kv : z->codes) qfec_code_free(kv.second);
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
    init_rx(S.rx, max_pkt_size, buf_items, kmax);
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
    z->sessions.push_back(std::move(S));
    const int s = (int)z->sessions.size() - 1;
    Session& T = z->sessions[s];
    T.rx.codecs = T.tx.codecs;
    // the same set_zfec_kn(k, n) both sides see, queued like any later call
    Op o;
    o.t = OP_SETKN;
    o.a = k;
    o.b = n;
    o.c = 1;
    T.ops.push_back(o);
    Op e;
    e.t = OP_ENABLE;
    e.a = enabled ? 1 : 0;
    T.ops.push_back(e);
    Op so;
    so.t = OP_SORTED;
    so.a = is_sorted ? 1 : 0;
    T.ops.push_back(so);
    return s;
}

static int push_op(qfec_zfec* z, int s, Op&& op) {
    if (!z) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(z->mu);
    if (s < 0 || s >= (int)z->sessions.size()) return QFEC_EINVAL;
    if (op.t == OP_UNPACK) {  // a uid for the datagram (decode cache keys), in the spare fields
        const uint64_t uid = z->next_uid++;
        op.b = (int)(uid >> 32);
        op.c = (int)(uint32_t)uid;
    }
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
int qfec_zfec_pack_input(qfec_zfec* z, int s, const void* data, unsigned int size) {
    if (!data && size) return QFEC_EINVAL;
    Op o;
    o.t = OP_PACK;
    o.data.assign(static_cast<const uint8_t*>(data), static_cast<const uint8_t*>(data) + size);
    return push_op(z, s, std::move(o));
}
int qfec_zfec_unpack_input(qfec_zfec* z, int s, const void* datagram, unsigned int size) {
    if (!datagram && size) return QFEC_EINVAL;
    Op o;
    o.t = OP_UNPACK;
    o.data.assign(static_cast<const uint8_t*>(datagram), static_cast<const uint8_t*>(datagram) + size);
    return push_op(z, s, std::move(o));
}

int qfec_zfec_flush(qfec_zfec* z, qfec_pack_output_fn pack_out, qfec_unpack_output_fn unpack_out, void* stream) {
    if (!z) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(z->mu);
    hipStream_t st = (hipStream_t)stream;
    const size_t NS = z->sessions.size();
    std::vector<std::vector<std::vector<Emit>>> outs(NS);
    // ---- send: zfec_pack_input (NetFecCodec.cpp:68-175) over every queue; groups to pack
    std::map<std::pair<int, int>, PackBatch> packs;
    std::deque<std::vector<uint8_t>> hold;  // payload copies the batches point at (stable addresses)
    for (size_t si = 0; si < NS; ++si) {
        Session& S = z->sessions[si];
        TxState& T = S.tx;
        outs[si].resize(S.ops.size());
        // a group whose rows span this flush: (batch, index) of its pack entry
        auto open_entry = [&](std::vector<Emit>& out, int row) {
            Emit e;
            e.kind = 0;
            e.row = row;
            e.batch = T.gk << 4 | T.gn;
            out.push_back(e);
        };
        std::vector<std::pair<size_t, int>> pending;  // (op, row) of the open group's rows in this flush
        auto close_group = [&](bool complete) {
            if (T.g_pay.empty() && !complete) return;
            PackBatch& b = packs[std::make_pair(T.gk, T.gn)];
            b.k = T.gk;
            b.n = T.gn;
            PackGroup g;
            g.sent0 = T.g_sent0;
            g.src0 = T.g_src0;
            g.pay.assign((size_t)T.gk, nullptr);
            for (size_t i = 0; i < T.g_pay.size() && i < (size_t)T.gk; ++i) {
                hold.push_back(T.g_pay[i]);
                g.pay[i] = &hold.back();
            }
            const long long gi = (long long)b.groups.size();
            b.groups.push_back(std::move(g));
            for (auto& pr : pending) {
                Emit& e = outs[si][pr.first][(size_t)pr.second];
                e.group = gi;
            }
            pending.clear();
        };
        for (size_t oi = 0; oi < S.ops.size(); ++oi) {
            Op& op = S.ops[oi];
            std::vector<Emit>& out = outs[si][oi];
            if (op.t == OP_SETKN) {  // set_zfec_kn :591-611 (send side); the open group keeps its (k, n)
                if (op.a < 0 || op.b < 0 || op.a > op.b) continue;
                const CodecEntry* c = T.codecs.find(op.a, op.b);
                if (c) {
                    T.have_codec = true;
                    T.k = c->k;
                    T.n = c->n;
                } else if (op.c) {
                    int rk, rn;
                    T.codecs.add(op.a, op.b, &rk, &rn);
                    T.have_codec = true;
                    T.k = rk;
                    T.n = rn;
                }
            } else if (op.t == OP_ENABLE) {
                T.enabled = op.a != 0;
            } else if (op.t == OP_DYNKN) {
                T.dynkn = op.a != 0;
            } else if (op.t == OP_LOST) {
                T.lost_rate = op.f;
            } else if (op.t == OP_PACK) {
                if (!T.enabled || !T.have_codec) {  // :75-94: [0x13][payload], numbering unchanged
                    Emit e;
                    e.kind = 1;
                    e.bytes.reserve(op.data.size() + 1);
                    e.bytes.push_back(0x13);
                    e.bytes.insert(e.bytes.end(), op.data.begin(), op.data.end());
                    out.push_back(std::move(e));
                    continue;
                }
                if (T.g_pay.empty() && T.g_emitted == 0) {  // a group starts (its (k, n) fixed)
                    T.gk = T.k;
                    T.gn = T.n;
                    T.g_sent0 = T.i_sent_pkt;
                    T.g_src0 = T.i_sent_src_pkt;
                }
                const int k = T.gk, n = T.gn;
                const int ik = (int)((T.i_sent_pkt - T.i_cur_segment_beg) % (uint32_t)n);
                if (ik < k) {
                    T.g_pay.push_back(op.data);
                    open_entry(out, ik);
                    pending.emplace_back(oi, (int)out.size() - 1);
                    T.i_sent_pkt++;
                    T.i_sent_src_pkt++;
                }
                if (ik == k - 1) {  // the check packets (:133-172)
                    for (int j = k; j < n; ++j) {
                        open_entry(out, j);
                        pending.emplace_back(oi, (int)out.size() - 1);
                        T.i_sent_pkt++;
                    }
                    close_group(true);
                    T.g_pay.clear();
                    T.g_emitted = 0;
                    if (T.dynkn) {  // recalc_zfec_kn (:51-65)
                        const CodecEntry* c = T.codecs.by_lost(T.lost_rate);
                        if (c) {
                            T.k = c->k;
                            T.n = c->n;
                        }
                    }
                    T.i_cur_segment_beg = T.i_sent_pkt;
                }
            }
        }
        // a group still open: its source rows of this flush go out now (they do not depend on
        // the rest of the group); the group is packed again, whole, when it completes
        if (!pending.empty()) {
            close_group(false);
            T.g_emitted = (int)T.g_pay.size();
        }
    }
    int rc = 0;
    for (auto& kv : packs)
        if ((rc = run_pack(z, kv.second, st))) return rc;
    // ---- receive: verdicts of this flush's FEC datagrams (pseudo-groups by (k, n, tag, dec_pkt_size))
    std::vector<std::vector<Verdict>> verd(NS);
    std::map<std::tuple<int, int, int, int>, UnpackBatch> vb;
    struct Where {
        std::tuple<int, int, int, int> b;
        int group, ik;
    };
    std::vector<std::vector<Where>> where(NS);
    // rows taken in each pseudo-group (shared by all sessions: a row's verdict is its own)
    std::map<std::tuple<int, int, int, int>, std::vector<std::vector<bool>>> open;
    for (size_t si = 0; si < NS; ++si) {
        Session& S = z->sessions[si];
        int dps = S.rx.dec_pkt_size;  // its growth over the queue (unpack_fec_head realloc)
        for (auto& op : S.ops) {
            if (op.t != OP_UNPACK) continue;
            Verdict v;
            const uint8_t* d = op.data.data();
            const size_t size = op.data.size();
            if ((int)size > dps) dps = (int)size;
            v.fec = size >= 11 && (d[0] == 0xEC || d[0] == 0xED);
            Where w{};
            w.group = -1;
            if (v.fec) {
                const uint32_t ikn = (uint32_t)d[9] | (uint32_t)d[10] << 8;
                const int n = (int)(ikn & 0xF), k = (int)((ikn >> 4) & 0xF), ik = (int)((ikn >> 8) & 0xF);
                v.usable = k >= 1 && k < n && n <= 15 && ik < n;
                if (v.usable) {
                    const auto key = std::make_tuple(k, n, d[0] == 0xED ? 1 : 0, dps);
                    UnpackBatch& b = vb[key];
                    b.k = k;
                    b.n = n;
                    b.checksum = d[0] == 0xED ? 1 : 0;
                    b.dec_pkt_size = dps;
                    auto& used = open[key];
                    int g = -1;
                    for (size_t gi = 0; gi < used.size(); ++gi)
                        if (!used[gi][(size_t)ik]) {
                            g = (int)gi;
                            break;
                        }
                    if (g < 0) {
                        used.emplace_back((size_t)n, false);
                        g = b.groups++;
                    }
                    used[(size_t)g][(size_t)ik] = true;
                    b.rows.push_back(UnpackRow{g, ik, op.data});
                    w.b = key;
                    w.group = g;
                    w.ik = ik;
                }
            }
            verd[si].push_back(std::move(v));
            where[si].push_back(w);
        }
    }
    for (auto& kv : vb)
        if ((rc = run_unpack(z, kv.second, st))) return rc;
    for (size_t si = 0; si < NS; ++si) {
        size_t v = 0;
        for (auto& op : z->sessions[si].ops) {
            if (op.t != OP_UNPACK) continue;
            Verdict& vd = verd[si][v];
            const Where& w = where[si][v];
            ++v;
            if (w.group < 0) continue;
            const UnpackBatch& b = vb[w.b];
            const size_t row = (size_t)w.group * b.n + w.ik;
            const uint8_t* d = op.data.data();
            const int hdr = d[0] == 0xED ? 13 : 11;
            vd.ok = b.rx[row] >= 0;
            if (vd.ok) vd.shard.assign(d + hdr, d + op.data.size());
            if (w.ik < b.k && vd.ok) {
                const int stt = b.status[(size_t)w.group * b.k + w.ik];
                vd.src_ok = stt >= 0;
                vd.src_size = b.psize[(size_t)w.group * b.k + w.ik];
                if (vd.src_ok) {
                    const uint8_t* sh = b.shards.data() + row * b.sp;
                    vd.payload.assign(sh + stt, sh + stt + vd.src_size);
                }
            }
        }
    }
    // ---- the receive machines: replay until every decode they call for has its device result
    std::map<DecodeKey, DecodeOut> cache;
    std::vector<RxState> start(NS);
    for (size_t si = 0; si < NS; ++si) start[si] = z->sessions[si].rx;
    for (;;) {
        std::vector<DecodeReq> missing;
        RxPass pass{&cache, &missing, true};
        for (size_t si = 0; si < NS; ++si) {
            Session& S = z->sessions[si];
            S.rx = start[si];
            for (auto& o : outs[si])
                o.erase(std::remove_if(o.begin(), o.end(), [](const Emit& e) { return e.kind == 2; }), o.end());
            RxMachine m(S, (int)si, verd[si], pass, outs[si]);
            m.run();
        }
        if (missing.empty()) break;
        // one launch per (k, n, mode, dec_pkt_size): each decode is a group holding exactly its k
        // shards, wrapped as 0xEC datagrams (no shard checksum to re-check)
        std::map<std::tuple<int, int, int, int>, UnpackBatch> db;
        std::map<std::tuple<int, int, int, int>, std::vector<const DecodeReq*>> reqs;
        for (auto& q : missing) {
            if (cache.count(q.key)) continue;
            const auto key = std::make_tuple(q.key.k, q.key.n, q.key.mode, q.key.dec_pkt_size);
            UnpackBatch& b = db[key];
            b.k = q.key.k;
            b.n = q.key.n;
            b.checksum = q.key.mode;
            b.dec_pkt_size = q.key.dec_pkt_size;
            const int g = b.groups++;
            for (auto& sh : q.shards) {
                std::vector<uint8_t> dg(11 + sh.first.size(), 0);
                dg[0] = 0xEC;
                const uint32_t ikn = (uint32_t)b.n | (uint32_t)b.k << 4 | (uint32_t)sh.second << 8;
                dg[9] = (uint8_t)(ikn & 0xFF);
                dg[10] = (uint8_t)(ikn >> 8);
                if (!sh.first.empty()) memcpy(dg.data() + 11, sh.first.data(), sh.first.size());
                b.rows.push_back(UnpackRow{g, sh.second, std::move(dg)});
            }
            reqs[key].push_back(&q);
            cache[q.key];  // placeholder, filled below
        }
        for (auto& kv : db) {
            UnpackBatch& b = kv.second;
            if ((rc = run_unpack(z, b, st))) return rc;
            const auto& rq = reqs[kv.first];
            for (size_t g = 0; g < rq.size(); ++g) {
                DecodeOut& o = cache[rq[g]->key];
                for (int i = 0; i < b.k; ++i) {
                    const int stt = b.status[g * b.k + i];
                    o.ok[i] = stt >= 0;
                    if (stt >= 0) {
                        const uint8_t* sh = b.shards.data() + (g * b.n + i) * b.sp;
                        o.payload[i].assign(sh + stt, sh + stt + b.psize[g * b.k + i]);
                    }
                }
            }
        }
    }  // (terminates: a pass that asks for decodes adds their keys to the cache)
    // ---- callbacks, session by session, op by op
    int calls = 0;
    for (size_t si = 0; si < NS; ++si) {
        Session& S = z->sessions[si];
        for (size_t oi = 0; oi < S.ops.size(); ++oi) {
            for (auto& e : outs[si][oi]) {
                if (e.kind == 0) {
                    const PackBatch& b = packs[std::make_pair(e.batch >> 4, e.batch & 15)];
                    const size_t row = (size_t)e.group * b.n + e.row;
                    if (b.wlen[row] > 0 && pack_out)
                        pack_out(S.peer, reinterpret_cast<const char*>(b.wire.data() + row * b.wp), (unsigned)b.wlen[row]);
                } else if (e.kind == 1) {
                    if (pack_out) pack_out(S.peer, reinterpret_cast<const char*>(e.bytes.data()), (unsigned)e.bytes.size());
                } else if (unpack_out) {
                    unpack_out(S.peer, reinterpret_cast<const char*>(e.bytes.data()), (unsigned)e.bytes.size(), e.src);
                }
                ++calls;
            }
        }
        S.ops.clear();
    }
    return calls;
}

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
