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
//
// Bytes are never copied on the host beyond what the device needs: datagrams, shards and
// payloads are views into the queued datagrams (reference-counted, so window slots can hold
// them across flushes), the device's inputs and outputs go through persistent pinned arenas
// with one copy each way per launch, and a verdict launch returns only the per-row verdicts
// (a received source packet's payload is the datagram's own bytes).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
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

using Buf = std::shared_ptr<const std::vector<uint8_t>>;
struct View {  // bytes [off, off + len) of a shared buffer
    Buf b;
    uint32_t off = 0, len = 0;
    const uint8_t* p() const { return b ? b->data() + off : nullptr; }
};

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

// ---- one dec_pkts_buf entry (FecPacket.h).  Its FecBuf is the received shard (a view): the
// decode reads its BufSize bytes, zero-padded (set_fec_dec_buf, FecCodecBuf.cpp:171-172), and
// flush_avail_pkts delivers the payload dec_src_pkt_info found in it when it was received
// (only source packets that passed are stored, NetFecCodec.cpp:240-245; dec_pkt_size only grows)
struct Slot {
    int64_t iPacket = -1;
    int BufSize = 0;
    bool bValid = false;
    bool bSourcePkt = true;
    uint32_t i_source_pkt = 0;
    bool bUsed = false;
    uint64_t uid = 0;  // which received datagram filled it (decode cache key)
    int ik = 0;        // the ik it was received with
    View shard, payload;
    void set_packet(const View& sh, uint64_t id, int row, const View& pay) {  // SetPacket (FecPacket.h:78-98)
        shard = sh;
        BufSize = (int)sh.len;
        bValid = true;
        bUsed = false;
        uid = id;
        ik = row;
        payload = pay;
    }
    void reset() {  // Reset (:99-122)
        iPacket = -1;
        BufSize = 0;
        bValid = false;
        bUsed = false;
    }
    // operator= (:42-68) copies every field the machine reads: the plain copy
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
    Buf data;  // OP_PACK payload / OP_UNPACK datagram
    int a = 0, b = 0, c = 0;
    float f = 0;
    uint64_t uid = 0;  // OP_UNPACK: the datagram's id (decode cache keys)
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
    std::vector<Buf> g_pay;
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
    int kind = 0;  // 0 datagram of a send batch, 1 owned bytes, 2 delivery (view + src),
                   // 3 delivery of a decoded row whose result is pending (batch = request, row)
    int batch = -1, row = 0;
    long long group = 0;
    View v;
    uint32_t src = 0;
};

// persistent pinned host + device memory, grow-only, re-made when the current device changes
struct Arena {
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    size_t hcap = 0, dcap = 0;
    int dev = -1;
    void release() {
        if (h) (void)hipHostFree(h);
        if (d) (void)hipFree(d);
        h = d = nullptr;
        hcap = dcap = 0;
    }
    int ensure(size_t hbytes, size_t dbytes) {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return QFEC_ENODEV;
        if (cur != dev) release();
        dev = cur;
        if (hbytes > hcap) {
            if (h) (void)hipHostFree(h);
            h = nullptr;
            hcap = 0;
            const size_t cap = round16(hbytes + (hbytes >> 2) + 4096);
            if (hipHostMalloc(reinterpret_cast<void**>(&h), cap, hipHostMallocDefault) != hipSuccess) {
                fprintf(stderr, "[qfec] qfec_zfec_flush: hipHostMalloc(%zu) failed\n", cap);
                h = nullptr;
                return QFEC_ENOMEM;
            }
            hcap = cap;
        }
        if (dbytes > dcap) {
            if (d) (void)hipFree(d);
            d = nullptr;
            dcap = 0;
            const size_t cap = round16(dbytes + (dbytes >> 2) + 4096);
            if (hipMalloc(reinterpret_cast<void**>(&d), cap) != hipSuccess) {
                fprintf(stderr, "[qfec] qfec_zfec_flush: hipMalloc(%zu) failed\n", cap);
                d = nullptr;
                return QFEC_ENOMEM;
            }
            dcap = cap;
        }
        return QFEC_OK;
    }
};

}  // namespace

struct qfec_zfec {
    std::mutex mu;
    std::vector<Session> sessions;
    std::map<std::pair<int, int>, qfec_code*> codes;  // (k, n) -> fec_new(k, n) matrix on the device
    uint64_t next_uid = 1;
    Arena pack_arena, rx_arena, dec_arena;
};

namespace {

qfec_code* code_for(qfec_zfec* z, int k, int n) {
    qfec_code*& c = z->codes[std::make_pair(k, n)];
    if (!c) c = qfec_code_new(QFEC_VANDERMONDE, k, n - k);  // fec_new(k, n), FecCodec.cpp:84
    return c;
}

// ---------------------------------------------------------------- device batches
// send: complete or partial groups of one (k, n); payloads of missing rows are empty
struct PackGroup {
    uint32_t sent0, src0;
    std::vector<Buf> pay;  // k entries (null = not yet given)
};
struct PackBatch {
    int k, n;
    std::vector<PackGroup> groups;
    // layout in the pack arena (host and device alike; shards device-only, last)
    size_t base = 0, total = 0, sp = 0, wp = 0;
    size_t o_offs = 0, o_sizes = 0, o_seq = 0, o_wlen = 0, o_wire = 0, o_end = 0, o_shards = 0;
    const uint8_t* wire = nullptr;  // results, in the pinned arena
    const int* wlen = nullptr;
};

void pack_layout(PackBatch& b, size_t base) {
    const size_t G = b.groups.size();
    size_t maxp = 1, total = 0;
    for (auto& g : b.groups)
        for (auto& p : g.pay)
            if (p) {
                maxp = std::max(maxp, p->size());
                total += p->size();
            }
    b.total = total;
    b.sp = round16(maxp + 4);
    b.wp = (b.sp + 13 + 63) & ~(size_t)63;  // the 64-B multiple: the fused send writes whole lines
    b.base = base;
    size_t o = base + round16(total + 16);  // payload (16 readable bytes past the last)
    b.o_offs = o;
    o += round16(G * b.k * 8);
    b.o_sizes = o;
    o += round16(G * b.k * 4);
    b.o_seq = o;
    o += round16(G * 8);
    b.o_wlen = o;
    o += round16(G * b.n * 4);
    b.o_wire = o;
    o += G * b.n * b.wp;
    b.o_end = o;
    b.o_shards = o;  // device only
}

int run_pack(qfec_zfec* z, PackBatch& b, hipStream_t s) {
    const size_t G = b.groups.size();
    Arena& A = z->pack_arena;
    uint8_t* h = A.h;
    long long* offs = reinterpret_cast<long long*>(h + b.o_offs);
    int* sizes = reinterpret_cast<int*>(h + b.o_sizes);
    uint32_t* seq = reinterpret_cast<uint32_t*>(h + b.o_seq);
    size_t o = 0;
    for (size_t g = 0; g < G; ++g) {
        seq[2 * g] = b.groups[g].sent0;
        seq[2 * g + 1] = b.groups[g].src0;
        for (int i = 0; i < b.k; ++i) {
            const Buf& p = b.groups[g].pay[(size_t)i];
            offs[g * b.k + i] = (long long)o;
            sizes[g * b.k + i] = p ? (int)p->size() : 0;
            if (p && !p->empty()) memcpy(h + b.base + o, p->data(), p->size());
            o += p ? p->size() : 0;
        }
    }
    memset(h + b.base + o, 0, 16);
    if (hipMemcpyAsync(A.d + b.base, h + b.base, b.o_wlen - b.base, hipMemcpyHostToDevice, s) != hipSuccess)
        return QFEC_EHIP;
    uint8_t* d = A.d;
    int rc = qfec_pack_datagrams(code_for(z, b.k, b.n), d + b.base, reinterpret_cast<const long long*>(d + b.o_offs),
                                 reinterpret_cast<const int*>(d + b.o_sizes),
                                 reinterpret_cast<const unsigned int*>(d + b.o_seq), (long long)G, 1 /* is_send_checksum */,
                                 d + b.o_shards, (long long)b.sp, d + b.o_wire, (long long)b.wp,
                                 reinterpret_cast<int*>(d + b.o_wlen), s);
    if (rc) return rc;
    if (hipMemcpyAsync(h + b.o_wlen, d + b.o_wlen, b.o_end - b.o_wlen, hipMemcpyDeviceToHost, s) != hipSuccess)
        return QFEC_EHIP;
    b.wire = h + b.o_wire;
    b.wlen = reinterpret_cast<const int*>(h + b.o_wlen);
    return QFEC_OK;
}

// receive: pseudo-groups of wire rows (datagrams, or 0xEC-wrapped shards for decodes)
struct UnpackRow {
    int group, ik;
    View hdr_src;    // bytes written from the row start: the datagram (verdicts) ...
    int wrap = 0;    // ... or, for decodes, a synthesized 11-byte 0xEC header (wrap = 1) + the shard
};
struct UnpackBatch {
    int k, n, checksum, dec_pkt_size;
    int groups = 0;
    bool want_shards = false;  // decodes: the data rows come back
    size_t need = 0;           // row bytes dec_src_pkt_info may read (head + size field), if known
    std::vector<UnpackRow> rows;
    // layout in an arena (host and device alike up to o_hend; marks and the device's shard
    // matrix after it); results in its host side
    size_t base = 0, sp = 0, wp = 0;
    size_t o_wlen = 0, o_rx = 0, o_st = 0, o_ps = 0, o_hsh = 0, o_hend = 0, o_marks = 0, o_dsh = 0, o_dend = 0;
    const int *rx = nullptr, *status = nullptr, *psize = nullptr;
    const uint8_t* shards = nullptr;  // want_shards: the data rows, [G][k][sp]
};

// shard rows hold every shard and every byte dec_src_pkt_info may read (the reference's buffers
// are dec_pkt_size long, zero-filled): `need` (verdicts: the largest head + size field among the
// rows; decodes: 0 -- a decoded row is zero past its inputs' longest shard, so a genuine packet
// fits; a row the pitch cuts short is re-decoded at dec_pkt_size + 4, see the decode loop)
void unpack_layout(UnpackBatch& b, size_t base) {
    const size_t G = (size_t)b.groups;
    size_t maxd = 16;
    for (auto& r : b.rows) maxd = std::max(maxd, (size_t)r.hdr_src.len + (r.wrap ? 11u : 0u));
    b.sp = round16(std::max(maxd, std::min(b.need, (size_t)b.dec_pkt_size + 4)));
    b.wp = round16(b.sp + 13);
    b.base = base;
    size_t o = base + G * b.n * b.wp;  // wire
    b.o_wlen = o;
    o += round16(G * b.n * 4);
    b.o_rx = o;
    o += round16(G * b.n * 4);
    b.o_st = o;
    o += round16(G * b.k * 4);
    b.o_ps = o;
    o += round16(G * b.k * 4);
    b.o_hsh = o;
    if (b.want_shards) o += G * b.k * b.sp;
    b.o_hend = o;
    b.o_marks = o;
    o += round16(G * b.n);
    b.o_dsh = o;
    o += G * b.n * b.sp;
    b.o_dend = o;
}

// rows copied into the pinned wire on several threads when there are many bytes
template <class F>
void parallel_rows(size_t nrows, size_t bytes, F&& f) {
    const unsigned hw = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    const unsigned T = bytes > ((size_t)8 << 20) ? hw : 1u;
    if (T <= 1) {
        f(0, nrows);
        return;
    }
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; ++t) th.emplace_back(f, nrows * t / T, nrows * (t + 1) / T);
    for (auto& x : th) x.join();
}

int run_unpack(qfec_zfec* z, Arena& A, UnpackBatch& b, hipStream_t s) {
    const size_t G = (size_t)b.groups;
    uint8_t* h = A.h;
    uint8_t* wire = h + b.base;
    int* wlen = reinterpret_cast<int*>(h + b.o_wlen);
    memset(wlen, 0, G * b.n * 4);
    size_t bytes = 0;
    for (auto& r : b.rows) bytes += r.hdr_src.len;
    parallel_rows(b.rows.size(), bytes, [&](size_t r0, size_t r1) {
        for (size_t i = r0; i < r1; ++i) {
            const UnpackRow& r = b.rows[i];
            uint8_t* row = wire + ((size_t)r.group * b.n + r.ik) * b.wp;
            size_t len = r.hdr_src.len;
            if (r.wrap) {  // [0xEC][sent 0][src 0][n | k << 4 | ik << 8][shard]
                memset(row, 0, 11);
                row[0] = 0xEC;
                const uint32_t ikn = (uint32_t)b.n | (uint32_t)b.k << 4 | (uint32_t)r.ik << 8;
                row[9] = (uint8_t)(ikn & 0xFF);
                row[10] = (uint8_t)(ikn >> 8);
                if (len) memcpy(row + 11, r.hdr_src.p(), len);
                len += 11;
            } else if (len) {
                memcpy(row, r.hdr_src.p(), len);
            }
            wlen[(size_t)r.group * b.n + r.ik] = (int)len;
        }
    });
    uint8_t* d = A.d;
    if (hipMemcpyAsync(d + b.base, h + b.base, b.o_rx - b.base, hipMemcpyHostToDevice, s) != hipSuccess)
        return QFEC_EHIP;
    int rc = qfec_unpack_datagrams(code_for(z, b.k, b.n), d + b.base, (long long)b.wp, reinterpret_cast<int*>(d + b.o_wlen),
                                   (long long)G, b.checksum, b.dec_pkt_size, d + b.o_dsh, (long long)b.sp,
                                   d + b.o_marks, reinterpret_cast<int*>(d + b.o_rx), reinterpret_cast<int*>(d + b.o_st),
                                   reinterpret_cast<int*>(d + b.o_ps), s);
    if (rc) return rc;
    if (hipMemcpyAsync(h + b.o_rx, d + b.o_rx, b.o_hsh - b.o_rx, hipMemcpyDeviceToHost, s) != hipSuccess)
        return QFEC_EHIP;
    if (b.want_shards &&  // the k data rows of each group only
        hipMemcpy2DAsync(h + b.o_hsh, (size_t)b.k * b.sp, d + b.o_dsh, (size_t)b.n * b.sp, (size_t)b.k * b.sp, G,
                         hipMemcpyDeviceToHost, s) != hipSuccess)
        return QFEC_EHIP;
    b.rx = reinterpret_cast<const int*>(h + b.o_rx);
    b.status = reinterpret_cast<const int*>(h + b.o_st);
    b.psize = reinterpret_cast<const int*>(h + b.o_ps);
    b.shards = b.want_shards ? h + b.o_hsh : nullptr;
    return QFEC_OK;
}

// ---------------------------------------------------------------- receive verdicts and decodes
struct Verdict {  // of one received FEC datagram
    bool fec = false;     // tag 0xEC / 0xED and size >= 11
    bool ok = false;      // unpack_fec_head returned the shard (header + shard checksum)
    bool usable = false;  // a header qfec_zfec can check (1 <= k < n <= 15, ik < n)
    View shard;           // the unpacked shard (after header and checksum)
    bool src_ok = false;  // dec_src_pkt_info on it (source packets)
    int src_size = 0;     // its size field
    View payload;
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
    View payload[16];
};
struct DecodeReq {
    DecodeKey key;
    std::vector<std::pair<View, int>> shards;  // (shard, ik)
};

struct RxPass {
    std::map<DecodeKey, DecodeOut>* cache;
    std::vector<DecodeReq>* missing;
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

    void deliver(const View& v, uint32_t src) {
        Emit e;
        e.kind = 2;
        e.v = v;
        e.src = src;
        cur->push_back(std::move(e));
    }
    // a decoded row: its payload, or a placeholder (kind 3) naming the request and row
    void deliver_decoded(const DecodeOut* res, int req, int i, uint32_t src) {
        if (res) {
            deliver(res->payload[i], src);
            return;
        }
        Emit e;
        e.kind = 3;
        e.batch = req;
        e.row = i;
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
                R.slots[is - ns] = R.slots[is];
                R.slots[is].reset();
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
                        deliver(s.payload, s.i_source_pkt);
                        set_used(i, true);
                    }
                    s.reset();
                    ret = true;
                }
            }
        }
        return ret;
    }
    // add_packet_fec_buf :485-535; fills `rows` with the first k valid slots (iValid order)
    bool add_packet(uint32_t ipkt, uint32_t isrc, const Verdict& vd, uint64_t uid, int ik, int k, int n,
                    uint32_t seg_beg, int* max_size, int* rows, int* nrows, bool* undefined) {
        if (ipkt >= R.first && ipkt < R.second) {
            Slot& s = R.slots[ipkt - R.first];
            s.set_packet(vd.shard, uid, ik, vd.payload);
            s.iPacket = (int64_t)ipkt;
            s.bSourcePkt = ipkt - seg_beg < (uint32_t)k;
            s.i_source_pkt = isrc;
        } else {
            return false;
        }
        int valid = 0;
        bool all_src = true;
        *undefined = false;
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
                rows[valid] = ck;
                *max_size = valid == 0 ? s.BufSize : std::max(*max_size, s.BufSize);
                ++valid;
                if (ck >= k) all_src = false;  // (sic: the window index, :523)
            }
        }
        *nrows = valid;
        return valid == k && !all_src;
    }

    void unpack(const Op& op, const Verdict& vd) {  // zfec_unpack_input :189-371
        const uint8_t* d = op.data->data();
        const uint32_t size = (uint32_t)op.data->size();
        if (size > (uint32_t)R.dec_pkt_size) R.dec_pkt_size = (int)size;  // unpack_fec_head realloc (:345-352)
        if (!vd.fec) {  // not an FEC datagram: handed over minus its tag, source index 0 (:201-209)
            if (size >= 1) deliver(View{op.data, 1, size - 1}, 0u);
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
                    deliver(vd.payload, seg_src_beg + (uint32_t)cur_ni);
                }
                bused = true;
            }
            if (i_recv == R.i_expected_packet && R.is_sorted) {
                R.fec_src_count++;
                deliver(vd.payload, seg_src_beg + (uint32_t)cur_ni);
                bused = true;
                R.i_expected_packet++;
                if (cmod((int)(R.i_expected_packet - seg_beg), cur_n) == cur_k) R.i_expected_packet = seg_beg + (uint32_t)cur_n;
            }
        }
        int max_size = 0, rows[16], nrows = 0;
        bool undefined = false;
        const bool dec = add_packet(i_recv, src, vd, op.uid, cur_ni, cur_k, cur_n, seg_beg, &max_size, rows, &nrows,
                                    &undefined);
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
        key.rows.reserve((size_t)nrows);
        for (int r = 0; r < nrows; ++r) key.rows.emplace_back(R.slots[rows[r]].uid, R.slots[rows[r]].ik);
        auto it = pass.cache->find(key);
        const DecodeOut* res = it == pass.cache->end() ? nullptr : &it->second;
        int req = -1;  // index of this decode's request (placeholders refer to it)
        if (!res) {
            DecodeReq q;
            q.key = std::move(key);
            for (int r = 0; r < nrows; ++r) q.shards.emplace_back(R.slots[rows[r]].shard, R.slots[rows[r]].ik);
            pass.missing->push_back(std::move(q));
            req = (int)pass.missing->size() - 1;
        }
        for (int i = 0; i < cur_k; ++i) {  // :308-366
            // an unknown result counts as a good packet for this pass (it is not emitted)
            if (res && !res->ok[i]) continue;
            const uint32_t pk = seg_beg + (uint32_t)i;
            if (!R.is_sorted) {
                if (!used(pk)) {
                    deliver_decoded(res, req, i, seg_src_beg + (uint32_t)i);
                    set_used(pk, true);
                    R.fec_src_count++;
                    R.fec_restore_count++;
                }
            }
            if (pk >= R.i_expected_packet && R.is_sorted) {
                if (!used(pk)) {
                    deliver_decoded(res, req, i, seg_src_beg + (uint32_t)i);
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

void init_rx(RxState& R, int buf_items, int max_pkt, int kmax) {
    R.slots.assign((size_t)buf_items, Slot());  // init_zfec_layer :653-664
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
    z->pack_arena.release();
    z->rx_arena.release();
    z->dec_arena.release();
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
    if (op.t == OP_UNPACK) op.uid = z->next_uid++;
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
static Buf copy_bytes(const void* p, unsigned int size) {
    return std::make_shared<const std::vector<uint8_t>>(static_cast<const uint8_t*>(p), static_cast<const uint8_t*>(p) + size);
}
int qfec_zfec_pack_input(qfec_zfec* z, int s, const void* data, unsigned int size) {
    if (!data && size) return QFEC_EINVAL;
    Op o;
    o.t = OP_PACK;
    o.data = copy_bytes(data, size);
    return push_op(z, s, std::move(o));
}
int qfec_zfec_unpack_input(qfec_zfec* z, int s, const void* datagram, unsigned int size) {
    if (!datagram && size) return QFEC_EINVAL;
    Op o;
    o.t = OP_UNPACK;
    o.data = copy_bytes(datagram, size);
    return push_op(z, s, std::move(o));
}

int qfec_zfec_flush(qfec_zfec* z, qfec_pack_output_fn pack_out, qfec_unpack_output_fn unpack_out, void* stream) {
    if (!z) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(z->mu);
    // QFEC_ZFEC_TIMING=1: phase times of each flush on stderr (profiling aid)
    static const bool timing = getenv("QFEC_ZFEC_TIMING") != nullptr;
    auto t_prev = std::chrono::steady_clock::now();
    auto phase = [&](const char* name) {
        if (!timing) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[qfec] zfec flush %-12s %8.3f ms\n", name, std::chrono::duration<double, std::milli>(t - t_prev).count());
        t_prev = t;
    };
    hipStream_t st = (hipStream_t)stream;
    const size_t NS = z->sessions.size();
    std::vector<std::vector<std::vector<Emit>>> outs(NS);
    // ---- send: zfec_pack_input (NetFecCodec.cpp:68-175) over every queue; groups to pack
    std::vector<PackBatch> packs;
    std::map<std::pair<int, int>, int> pack_of;  // (k, n) -> index in packs
    auto batch_for = [&](int k, int n) -> int {
        auto it = pack_of.find(std::make_pair(k, n));
        if (it != pack_of.end()) return it->second;
        PackBatch b;
        b.k = k;
        b.n = n;
        packs.push_back(std::move(b));
        pack_of.emplace(std::make_pair(k, n), (int)packs.size() - 1);
        return (int)packs.size() - 1;
    };
    for (size_t si = 0; si < NS; ++si) {
        Session& S = z->sessions[si];
        TxState& T = S.tx;
        outs[si].resize(S.ops.size());
        std::vector<std::pair<size_t, int>> pending;  // (op, index in its outputs) of the open group's rows
        auto open_entry = [&](std::vector<Emit>& out, size_t oi, int row) {
            Emit e;
            e.kind = 0;
            e.row = row;
            e.batch = batch_for(T.gk, T.gn);
            out.push_back(e);
            pending.emplace_back(oi, (int)out.size() - 1);
        };
        auto close_group = [&]() {  // the open group's rows so far, as one group of its batch
            PackBatch& b = packs[(size_t)batch_for(T.gk, T.gn)];
            PackGroup g;
            g.sent0 = T.g_sent0;
            g.src0 = T.g_src0;
            g.pay.assign((size_t)T.gk, nullptr);
            for (size_t i = 0; i < T.g_pay.size() && i < (size_t)T.gk; ++i) g.pay[i] = T.g_pay[i];
            const long long gi = (long long)b.groups.size();
            b.groups.push_back(std::move(g));
            for (auto& pr : pending) outs[si][pr.first][(size_t)pr.second].group = gi;
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
                    auto v = std::make_shared<std::vector<uint8_t>>();
                    v->reserve(op.data->size() + 1);
                    v->push_back(0x13);
                    v->insert(v->end(), op.data->begin(), op.data->end());
                    Emit e;
                    e.kind = 1;
                    e.v = View{v, 0, (uint32_t)v->size()};
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
                    open_entry(out, oi, ik);
                    T.i_sent_pkt++;
                    T.i_sent_src_pkt++;
                }
                if (ik == k - 1) {  // the check packets (:133-172)
                    for (int j = k; j < n; ++j) {
                        open_entry(out, oi, j);
                        T.i_sent_pkt++;
                    }
                    close_group();
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
            close_group();
            T.g_emitted = (int)T.g_pay.size();
        }
    }
    phase("tx machine");
    int rc = 0;
    {
        // batches laid out back to back at their device extents (the device-only shard
        // scratch is each batch's last region), so no two batches share arena bytes
        size_t hend = 0, dend = 0;
        for (auto& b : packs) {
            pack_layout(b, dend);
            hend = b.o_end;
            dend = b.o_shards + b.groups.size() * b.n * b.sp;
        }
        if (!packs.empty()) {
            if ((rc = z->pack_arena.ensure(hend, dend))) return rc;
            for (auto& b : packs)
                if ((rc = run_pack(z, b, st))) return rc;
        }
    }
    phase("pack launch");
    // ---- receive: verdicts of this flush's FEC datagrams (pseudo-groups by (k, n, tag, dec_pkt_size))
    std::vector<std::vector<Verdict>> verd(NS);
    std::vector<UnpackBatch> vb;
    std::map<std::tuple<int, int, int, int>, int> vb_of;
    struct Where {
        int batch = -1, group = -1, ik = 0;
    };
    std::vector<std::vector<Where>> where(NS);
    // rows taken in each pseudo-group (shared by all sessions: a row's verdict is its own)
    std::vector<std::vector<uint16_t>> taken;  // per batch, per group: bit ik
    for (size_t si = 0; si < NS; ++si) {
        Session& S = z->sessions[si];
        int dps = S.rx.dec_pkt_size;  // its growth over the queue (unpack_fec_head realloc)
        for (auto& op : S.ops) {
            if (op.t != OP_UNPACK) continue;
            Verdict v;
            const uint8_t* d = op.data->data();
            const size_t size = op.data->size();
            if ((int)size > dps) dps = (int)size;
            v.fec = size >= 11 && (d[0] == 0xEC || d[0] == 0xED);
            Where w;
            if (v.fec) {
                const uint32_t ikn = (uint32_t)d[9] | (uint32_t)d[10] << 8;
                const int n = (int)(ikn & 0xF), k = (int)((ikn >> 4) & 0xF), ik = (int)((ikn >> 8) & 0xF);
                v.usable = k >= 1 && k < n && n <= 15 && ik < n;
                if (v.usable) {
                    const int cs = d[0] == 0xED ? 1 : 0;
                    const auto key = std::make_tuple(k, n, cs, dps);
                    auto it = vb_of.find(key);
                    int bi;
                    if (it == vb_of.end()) {
                        UnpackBatch b;
                        b.k = k;
                        b.n = n;
                        b.checksum = cs;
                        b.dec_pkt_size = dps;
                        vb.push_back(std::move(b));
                        taken.emplace_back();
                        bi = (int)vb.size() - 1;
                        vb_of.emplace(key, bi);
                    } else {
                        bi = it->second;
                    }
                    UnpackBatch& b = vb[(size_t)bi];
                    auto& used = taken[(size_t)bi];
                    int g = -1;
                    for (size_t gi = used.size() > 8 ? used.size() - 8 : 0; gi < used.size(); ++gi)
                        if (!((used[gi] >> ik) & 1u)) {
                            g = (int)gi;
                            break;
                        }
                    if (g < 0) {
                        used.push_back(0);
                        g = b.groups++;
                    }
                    used[(size_t)g] |= (uint16_t)(1u << ik);
                    b.rows.push_back(UnpackRow{g, ik, View{op.data, 0, (uint32_t)size}, 0});
                    // the row bytes dec_src_pkt_info may read: head + the shard's size field
                    const size_t hdr = cs ? 13 : 11;
                    if (ik < k && size >= hdr + 2)
                        b.need = std::max(b.need, (size_t)(cs ? 4 : 2) + (d[hdr] | (size_t)d[hdr + 1] << 8));
                    w.batch = bi;
                    w.group = g;
                    w.ik = ik;
                }
            }
            verd[si].push_back(std::move(v));
            where[si].push_back(w);
        }
    }
    phase("rx grouping");
    if (!vb.empty()) {
        size_t hend = 0, dend = 0;
        for (auto& b : vb) {
            unpack_layout(b, dend);
            hend = b.o_hend;
            dend = b.o_dend;
        }
        if ((rc = z->rx_arena.ensure(hend, dend))) return rc;
        for (auto& b : vb)
            if ((rc = run_unpack(z, z->rx_arena, b, st))) return rc;
        if (hipStreamSynchronize(st) != hipSuccess) return QFEC_EHIP;
    }
    for (size_t si = 0; si < NS; ++si) {
        size_t v = 0;
        for (auto& op : z->sessions[si].ops) {
            if (op.t != OP_UNPACK) continue;
            Verdict& vd = verd[si][v];
            const Where& w = where[si][v];
            ++v;
            if (w.group < 0) continue;
            const UnpackBatch& b = vb[(size_t)w.batch];
            const size_t row = (size_t)w.group * b.n + w.ik;
            const uint32_t size = (uint32_t)op.data->size();
            const uint32_t hdr = op.data->data()[0] == 0xED ? 13 : 11;
            vd.ok = b.rx[row] >= 0;
            if (vd.ok) vd.shard = View{op.data, hdr, size - hdr};
            if (w.ik < b.k && vd.ok) {
                const int stt = b.status[(size_t)w.group * b.k + w.ik];
                vd.src_ok = stt >= 0;
                vd.src_size = b.psize[(size_t)w.group * b.k + w.ik];
                // a received row's payload is the datagram's own bytes
                if (vd.src_ok) vd.payload = View{op.data, hdr + (uint32_t)stt, (uint32_t)vd.src_size};
            }
        }
    }
    phase("verdicts");
    // ---- the receive machines.  A pass that meets a decode without a device result assumes
    // every row of it decoded and passed (the common case) and leaves placeholders for its
    // deliveries; after the launches the placeholders are filled when that held for every such
    // decode, and otherwise the machines are replayed from the flush's starting state.
    std::map<DecodeKey, DecodeOut> cache;
    std::vector<RxState> start(NS);
    for (size_t si = 0; si < NS; ++si) start[si] = z->sessions[si].rx;
    // sessions are independent: their machines run on several threads (the decode cache is
    // only read during a pass), each session collecting its own decode requests; the requests
    // are then numbered in session order, as one thread would have numbered them
    size_t rx_ops = 0;
    for (size_t si = 0; si < NS; ++si) rx_ops += verd[si].size();
    unsigned rx_threads =
        rx_ops < 4096 ? 1u : std::max(1u, std::min({8u, std::thread::hardware_concurrency(), (unsigned)NS}));
    if (const char* e = getenv("QFEC_ZFEC_RX_THREADS"))  // tests: force the threaded machines
        rx_threads = (unsigned)std::max(1, std::min(64, atoi(e)));
    for (int pass_no = 0;; ++pass_no) {
        std::vector<DecodeReq> missing;
        std::vector<std::vector<DecodeReq>> miss_s(NS);
        auto run_session = [&](size_t si) {
            Session& S = z->sessions[si];
            if (pass_no) S.rx = start[si];
            if (pass_no)
                for (auto& o : outs[si])
                    o.erase(std::remove_if(o.begin(), o.end(), [](const Emit& e) { return e.kind >= 2; }), o.end());
            RxPass pass{&cache, &miss_s[si]};
            RxMachine m(S, (int)si, verd[si], pass, outs[si]);
            m.run();
        };
        if (rx_threads <= 1) {
            for (size_t si = 0; si < NS; ++si) run_session(si);
        } else {
            std::atomic<size_t> next{0};
            std::vector<std::thread> th;
            for (unsigned t = 0; t < rx_threads; ++t)
                th.emplace_back([&]() {
                    for (size_t si; (si = next.fetch_add(1)) < NS;) run_session(si);
                });
            for (auto& x : th) x.join();
        }
        for (size_t si = 0; si < NS; ++si) {
            const int base = (int)missing.size();
            if (base)
                for (auto& o : outs[si])
                    for (auto& e : o)
                        if (e.kind == 3) e.batch += base;
            for (auto& q : miss_s[si]) missing.push_back(std::move(q));
        }
        phase("rx machine");
        if (missing.empty()) break;
        // one launch per (k, n, mode, dec_pkt_size): each decode is a group holding exactly its k
        // shards, wrapped as 0xEC datagrams (no shard checksum to re-check).  Round 0 decodes at
        // the shards' own length; a row whose size field reaches past that pitch (only a corrupt
        // one can) is decoded again at dec_pkt_size + 4 in round 1, as the reference reads it.
        std::vector<const DecodeReq*> todo;
        for (auto& q : missing)
            if (!cache.count(q.key)) {
                cache[q.key];  // filled below
                todo.push_back(&q);
            }
        for (int round = 0; round < 2 && !todo.empty(); ++round) {
            std::vector<UnpackBatch> db;
            std::map<std::tuple<int, int, int, int>, int> db_of;
            std::vector<std::vector<const DecodeReq*>> reqs;
            for (const DecodeReq* q : todo) {
                const auto key = std::make_tuple(q->key.k, q->key.n, q->key.mode, q->key.dec_pkt_size);
                auto it = db_of.find(key);
                int bi;
                if (it == db_of.end()) {
                    UnpackBatch b;
                    b.k = q->key.k;
                    b.n = q->key.n;
                    b.checksum = q->key.mode;
                    b.dec_pkt_size = q->key.dec_pkt_size;
                    b.want_shards = true;
                    b.need = round ? (size_t)b.dec_pkt_size + 4 : 0;
                    db.push_back(std::move(b));
                    reqs.emplace_back();
                    bi = (int)db.size() - 1;
                    db_of.emplace(key, bi);
                } else {
                    bi = it->second;
                }
                UnpackBatch& b = db[(size_t)bi];
                const int g = b.groups++;
                for (auto& sh : q->shards) b.rows.push_back(UnpackRow{g, sh.second, sh.first, 1});
                reqs[(size_t)bi].push_back(q);
            }
            size_t hend = 0, dend = 0;
            for (auto& b : db) {
                unpack_layout(b, dend);
                hend = b.o_hend;
                dend = b.o_dend;
            }
            if ((rc = z->dec_arena.ensure(hend, dend))) return rc;
            for (auto& b : db)
                if ((rc = run_unpack(z, z->dec_arena, b, st))) return rc;
            if (hipStreamSynchronize(st) != hipSuccess) return QFEC_EHIP;
            std::vector<const DecodeReq*> again;
            for (size_t bi = 0; bi < db.size(); ++bi) {
                const UnpackBatch& b = db[bi];
                const auto& rq = reqs[bi];
                const int head = b.checksum ? 4 : 2;
                // A decode's input rows come back unchanged (zero past their shard), so a
                // delivered payload that lies inside its input shard is a view of that shard;
                // only the rebuilt rows (and payloads reaching past an input's shard) outlive
                // this round's arena as one owned copy per batch.
                std::vector<std::pair<size_t, size_t>> copy;  // (row in b.shards, bytes)
                std::vector<const View*> src_of((size_t)b.k);
                size_t keep_bytes = 0;
                for (size_t g = 0; g < rq.size(); ++g) {
                    bool cut = false;
                    DecodeOut& o = cache[rq[g]->key];
                    std::fill(src_of.begin(), src_of.end(), nullptr);
                    for (auto& sh : rq[g]->shards)
                        if (sh.second < b.k) src_of[(size_t)sh.second] = &sh.first;
                    for (int i = 0; i < b.k; ++i) {
                        const int stt = b.status[g * b.k + i], ps = b.psize[g * b.k + i];
                        cut |= stt == -1 && ps < b.dec_pkt_size && (size_t)(head + ps) > b.sp;
                        o.ok[i] = stt >= 0;
                        o.payload[i] = View{};
                        if (stt < 0) continue;
                        const View* in = src_of[(size_t)i];
                        if (in && (size_t)stt + (size_t)ps <= in->len) {
                            o.payload[i] = View{in->b, in->off + (uint32_t)stt, (uint32_t)ps};
                        } else {
                            o.payload[i] = View{nullptr, (uint32_t)keep_bytes, (uint32_t)ps};  // buffer set below
                            copy.emplace_back((g * b.k + i) * b.sp + (size_t)stt, (size_t)ps);
                            keep_bytes += (size_t)ps;
                        }
                    }
                    if (cut && round == 0) again.push_back(rq[g]);
                }
                if (!copy.empty()) {
                    auto keep = std::make_shared<std::vector<uint8_t>>(keep_bytes);
                    size_t o = 0;
                    for (auto& c : copy) {
                        if (c.second) memcpy(keep->data() + o, b.shards + c.first, c.second);
                        o += c.second;
                    }
                    const Buf kb = keep;
                    for (size_t g = 0; g < rq.size(); ++g) {
                        DecodeOut& o2 = cache[rq[g]->key];
                        for (int i = 0; i < b.k; ++i)
                            if (o2.ok[i] && !o2.payload[i].b) o2.payload[i].b = kb;
                    }
                }
            }
            todo.swap(again);
        }
        phase("decodes");
        bool all_ok = true;
        for (auto& q : missing) {
            const DecodeOut& o = cache[q.key];
            for (int i = 0; i < q.key.k; ++i) all_ok &= o.ok[i];
        }
        if (!all_ok) continue;  // replay with the results
        for (size_t si = 0; si < NS; ++si)  // the assumption held: fill the placeholders
            for (auto& o : outs[si])
                for (auto& e : o)
                    if (e.kind == 3) {
                        e.kind = 2;
                        e.v = cache[missing[(size_t)e.batch].key].payload[e.row];
                    }
        break;
    }  // (terminates: a pass that asks for decodes adds their keys to the cache)
    if (!packs.empty() && hipStreamSynchronize(st) != hipSuccess) return QFEC_EHIP;
    // ---- callbacks, session by session, op by op
    int calls = 0;
    for (size_t si = 0; si < NS; ++si) {
        Session& S = z->sessions[si];
        for (size_t oi = 0; oi < S.ops.size(); ++oi) {
            for (auto& e : outs[si][oi]) {
                if (e.kind == 0) {
                    const PackBatch& b = packs[(size_t)e.batch];
                    const size_t row = (size_t)e.group * b.n + e.row;
                    if (b.wlen[row] > 0 && pack_out)
                        pack_out(S.peer, reinterpret_cast<const char*>(b.wire + row * b.wp), (unsigned)b.wlen[row]);
                } else if (e.kind == 1) {
                    if (pack_out) pack_out(S.peer, reinterpret_cast<const char*>(e.v.p()), e.v.len);
                } else if (unpack_out) {
                    unpack_out(S.peer, reinterpret_cast<const char*>(e.v.p()), e.v.len, e.src);
                }
                ++calls;
            }
        }
        S.ops.clear();
    }
    phase("callbacks");
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
