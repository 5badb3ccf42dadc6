// qfec_zfec_impl.hpp -- internals of the exact NetFecCodec layer (include/qfec_zfec.h), shared by
// qfec_zfec.cpp (the per-session calls) and qfec_zfec_flush.cpp (the flush: the state machines
// replayed over the queued calls and the batched device launches).  See qfec_zfec.cpp for the design.
#pragma once

// order, op order, on the flushing thread.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/qfec.h"
#include "../../include/qfec_zfec.h"
#include "qfec_pool.hpp"

namespace qfec_zfec_impl {

inline size_t round16(size_t x) { return (x + 15) & ~(size_t)15; }
inline uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
inline int packed_size(int size) { return size < 0 ? 0 : size + 4 + 12 + 4; }  // getPackedPktSize, FecCodecBuf.cpp:16-25
inline int cmod(int a, int b) { return a % b; }                                   // C's % (truncating), as in :277

// where a View's bytes live
enum Src : uint8_t { SRC_NONE = 0, SRC_RX, SRC_TX, SRC_DEC, SRC_OWN, SRC_IO };
struct View {  // bytes [off, off + len) of one of the flush's buffers
    uint8_t src = SRC_NONE;
    uint32_t off = 0, len = 0;
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

// ---- one dec_pkts_buf entry (FecPacket.h).  Its FecBuf is the received shard: the decode
// reads its BufSize bytes, zero-padded (set_fec_dec_buf, FecCodecBuf.cpp:171-172), and
// flush_avail_pkts delivers the payload dec_src_pkt_info found in it when it was received
// (only source packets that passed are stored, NetFecCodec.cpp:240-245; dec_pkt_size only grows).
// shard and payload lie inside the datagram [dg_off, dg_off + dg_len) of the receive arena.
struct Slot {
    int64_t iPacket = -1;
    int BufSize = 0;
    bool bValid = false;
    bool bSourcePkt = true;
    uint32_t i_source_pkt = 0;
    bool bUsed = false;
    uint64_t uid = 0;  // which received datagram filled it (decode cache key)
    int ik = 0;        // the ik it was received with
    uint32_t dg_off = 0, dg_len = 0;
    View shard, payload;
    void set_packet(const View& sh, uint64_t id, int row, const View& pay, uint32_t doff, uint32_t dlen) {
        shard = sh;  // SetPacket (FecPacket.h:78-98)
        BufSize = (int)sh.len;
        bValid = true;
        bUsed = false;
        uid = id;
        ik = row;
        payload = pay;
        dg_off = doff;
        dg_len = dlen;
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

enum OpType : uint8_t { OP_PACK, OP_UNPACK, OP_SETKN, OP_ENABLE, OP_SORTED, OP_DYNKN, OP_LOST };
struct Op {
    OpType t;
    uint32_t off = 0, size = 0;  // OP_PACK payload (send arena) / OP_UNPACK datagram (receive arena)
    int a = 0, b = 0, c = 0;
    float f = 0;
    uint64_t uid = 0;  // OP_UNPACK: the datagram's id (decode cache keys)
};
// OP_UNPACK: the header fields the flush reads, taken at the input call while the datagram is in
// cache (the flush would otherwise miss on every arena header): a = tag (d[0], -1 if empty),
// b = i_recv (d[1..4]), c = src (d[5..8]), f's bits = ik|k|n (d[9..10]) << 16 | the shard's size
// field (the two bytes after the header; 0 if the datagram ends first)
inline void parse_head(Op& o, const uint8_t* d, uint32_t size) {
    o.a = size >= 1 ? d[0] : -1;
    uint32_t ikn = 0, szf = 0;
    if (size >= 11) {
        o.b = (int)rd32(d + 1);
        o.c = (int)rd32(d + 5);
        ikn = (uint32_t)d[9] | (uint32_t)d[10] << 8;
        const uint32_t hdr = d[0] == 0xED ? 13 : 11;
        if (size >= hdr + 2) szf = (uint32_t)d[hdr] | (uint32_t)d[hdr + 1] << 8;
    }
    const uint32_t w = ikn << 16 | szf;
    memcpy(&o.f, &w, 4);
}
inline uint32_t op_ikn(const Op& o) {
    uint32_t w;
    memcpy(&w, &o.f, 4);
    return w >> 16;
}
inline uint32_t op_szf(const Op& o) {
    uint32_t w;
    memcpy(&w, &o.f, 4);
    return w & 0xFFFF;
}

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
    std::vector<View> g_pay;  // send-arena views
    int g_emitted = 0;
};

struct alignas(64) Session {  // (one cache line boundary per session: threads run adjacent ones)
    void* peer = nullptr;
    int max_pkt = 0, kmax = 0;
    TxState tx;
    RxState rx;
    std::vector<Op> ops;
};

// an output of one op, filled in after the device work
struct Emit {
    uint32_t op = 0;  // the op it belongs to (callbacks run in op order)
    uint8_t kind = 0;  // 0 datagram of a send batch (batch, group, row), 1 owned bytes (v),
                       // 2 delivery (v + src), 3 delivery of a decoded row whose result is
                       // pending (batch = request, row)
    int batch = -1, row = 0;
    long long group = 0;
    View v;
    uint32_t src = 0;
};

// pinned host memory, grow-only; offsets stay valid when it grows.  Without a device (FEC-off
// sessions need none) it is ordinary memory.
struct HostArena {
    uint8_t* h = nullptr;
    size_t cap = 0, used = 0;
    bool pinned = false;
    bool mapped = false;  // an mmap'd 2 MiB-page block registered with the runtime
    void release() {
        if (h) {
            if (mapped) {
                (void)hipHostUnregister(h);
                munmap(h, cap);
            } else if (pinned) {
                (void)hipHostFree(h);
            } else {
                free(h);
            }
        }
        h = nullptr;
        cap = used = 0;
        mapped = false;
    }
    // The arenas are 2 MiB-page mappings registered with the runtime, hipHostMalloc'd memory
    // where that fails: alternating processes on one box, the receive flush 14.4-14.9 -> 11.7-12.5 ms
    // and the send flush 16.6-16.8 -> 14.9-15.1 ms (fewer page translations for the arena's H2D and
    // D2H and for the callbacks' reads; profiles/r05w)
    // A registration that fails once (no device: FEC-off contexts need none) is not tried again:
    // later growths go straight to hipHostMalloc / malloc instead of mapping, zeroing and unmapping
    // a block each time.
    static std::atomic<bool>& register_failed() {
        static std::atomic<bool> f{false};
        return f;
    }
    static uint8_t* map_huge(size_t bytes) {
        if (register_failed().load(std::memory_order_relaxed)) return nullptr;
        void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) return nullptr;
        (void)madvise(p, bytes, MADV_HUGEPAGE);
        memset(p, 0, bytes);  // the pages exist before they are registered
        if (hipHostRegister(p, bytes, hipHostRegisterMapped) != hipSuccess) {
            (void)hipGetLastError();
            munmap(p, bytes);
            register_failed().store(true, std::memory_order_relaxed);
            return nullptr;
        }
        return static_cast<uint8_t*>(p);
    }
    bool reserve(size_t need) {
        if (need <= cap) return true;
        size_t ncap = std::max(need + (need >> 1), (size_t)4 << 20);
        uint8_t* nh = nullptr;
        bool pin = true, map = false;
        {
            const size_t hcap = (ncap + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1);
            nh = map_huge(hcap);
            map = nh != nullptr;
            if (map) ncap = hcap;
        }
        if (!nh && (hipHostMalloc(reinterpret_cast<void**>(&nh), ncap, hipHostMallocDefault) != hipSuccess || !nh)) {
            (void)hipGetLastError();
            pin = false;
            nh = static_cast<uint8_t*>(malloc(ncap));
            if (!nh) return false;
        }
        if (used) memcpy(nh, h, used);
        const size_t u = used;
        release();
        h = nh;
        cap = ncap;
        used = u;
        pinned = pin;
        mapped = map;
        return true;
    }
    // n bytes at a 16-B aligned offset, 16 readable bytes after them (the kernels' loads)
    bool append(const void* p, size_t n, uint32_t* off) {
        const size_t o = round16(used);
        if (o + round16(n) + 16 > (size_t)UINT32_MAX || !reserve(o + round16(n) + 16)) return false;
        if (n) memcpy(h + o, p, n);
        memset(h + o + n, 0, 16);
        used = o + n;
        *off = (uint32_t)o;
        return true;
    }
};

// device memory, grow-only, re-made when the current device changes
struct DevBuf {
    uint8_t* d = nullptr;
    size_t cap = 0;
    int dev = -1;
    void release() {
        if (d) (void)hipFree(d);
        d = nullptr;
        cap = 0;
    }
    int ensure(size_t bytes) {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return QFEC_ENODEV;
        if (cur != dev) release();
        dev = cur;
        if (bytes <= cap) return QFEC_OK;
        release();
        dev = cur;
        const size_t ncap = round16(bytes + (bytes >> 2) + 4096);
        if (hipMalloc(reinterpret_cast<void**>(&d), ncap) != hipSuccess) {
            fprintf(stderr, "[qfec] qfec_zfec_flush: hipMalloc(%zu) failed\n", ncap);
            d = nullptr;
            return QFEC_ENOMEM;
        }
        cap = ncap;
        return QFEC_OK;
    }
};

}  // namespace qfec_zfec_impl

using namespace qfec_zfec_impl;

struct qfec_zfec {
    std::mutex mu;
    std::vector<Session> sessions;
    std::map<std::pair<int, int>, qfec_code*> codes;  // (k, n) -> fec_new(k, n) matrix on the device
    uint64_t next_uid = 1;
    HostArena rx[2], tx[2];  // queued datagrams / payloads (+ what the state holds), and their spares
    int rxc = 0, txc = 0;
    HostArena io;            // per-flush pinned staging: tables in, results and datagrams out
    DevBuf d_rx, d_tx, d_io, d_work;
    std::unique_ptr<qfec::HostPool> pool;  // the flush's session threads (kept between flushes)
};

namespace qfec_zfec_impl {

inline qfec_code* code_for(qfec_zfec* z, int k, int n) {
    qfec_code*& c = z->codes[std::make_pair(k, n)];
    if (!c) c = qfec_code_new(QFEC_VANDERMONDE, k, n - k);  // fec_new(k, n), FecCodec.cpp:84
    return c;
}

// the flush's byte sources, resolved by View::src
struct Bufs {
    const uint8_t* rx = nullptr;
    const uint8_t* tx = nullptr;
    const uint8_t* dec = nullptr;
    const uint8_t* io = nullptr;
    const std::vector<std::vector<uint8_t>>* own = nullptr;  // per session
    const uint8_t* p(const View& v, size_t session) const {
        switch (v.src) {
            case SRC_RX: return rx + v.off;
            case SRC_TX: return tx + v.off;
            case SRC_DEC: return dec + v.off;
            case SRC_OWN: return (*own)[session].data() + v.off;
            case SRC_IO: return io + v.off;
            default: return nullptr;
        }
    }
};

// run f(i) for i < count on up to `threads` threads of the context's pool (the calling thread
// is one of them; the pool's threads stay between flushes)
template <class F>
void parallel_for(qfec_zfec* z, size_t count, unsigned threads, F&& f) {
    if (threads <= 1 || count <= 1) {
        for (size_t i = 0; i < count; ++i) f(i);
        return;
    }
    if (!z->pool || z->pool->threads() < (int)threads) z->pool.reset(new qfec::HostPool((int)threads));
    std::atomic<size_t> next{0};
    z->pool->run(
        [&](int, int) {
            for (size_t i; (i = next.fetch_add(1)) < count;) f(i);
        },
        (int)threads);
}

// staging bump allocator over the pinned io arena and its device twin (same offsets)
struct Stage {
    size_t o = 0;
    size_t take(size_t n) {
        const size_t r = o;
        o = round16(o + n);
        return r;
    }
};

// ---------------------------------------------------------------- device batches
// send: complete or partial groups of one (k, n); payloads of missing rows are empty
struct PackGroup {
    uint32_t sent0, src0;
    View pay[15];  // k entries (len 0 + SRC_NONE = not yet given)
};
struct PackBatch {
    int k, n;
    std::vector<PackGroup> groups;
    size_t sp = 0, wp = 0;
    size_t o_offs = 0, o_sizes = 0, o_seq = 0, o_wlen = 0, o_wire = 0, d_shards = 0;  // results: io arena
};

// receive: pseudo-groups of rows (datagrams, or bare shards for decodes)
struct UnpackRow {
    int group, ik;
    uint32_t off, len;  // the row's bytes in the receive arena
};
struct UnpackBatch {
    int k, n, checksum, dec_pkt_size;
    int groups = 0;
    int wrap = 0;              // decodes: rows are shards (an 0xEC header synthesized on the device)
    bool want_shards = false;  // decodes: rows of the shard matrix come back (`fetch`)
    std::vector<uint32_t> fetch;  // decodes: the rows (g * n + i) to bring back, in this order
    size_t need = 0;           // row bytes dec_src_pkt_info may read (head + size field), if known
    std::vector<UnpackRow> rows;
    // verdicts: the sessions' own row lists, each with its first group's index in this batch
    // (placed on the session threads; visited in place, not merged)
    std::vector<std::pair<const std::vector<UnpackRow>*, int>> segs;
    template <class F>
    void for_rows(F&& f) const {
        for (auto& r : rows) f(r.group, r);
        for (auto& sg : segs)
            for (auto& r : *sg.first) f(r.group + sg.second, r);
    }
    size_t sp = 0, wp = 0;
    // staging (io arena, host and device alike): offsets and lengths in, results out
    size_t o_off = 0, o_len = 0, o_rx = 0, o_st = 0, o_ps = 0, o_hsh = 0;
    // device work buffer: gathered wire, its lengths, marks, shard matrix
    size_t w_wire = 0, w_wlen = 0, w_marks = 0, w_sh = 0;
    const int *rx = nullptr, *status = nullptr, *psize = nullptr;
    const uint8_t* shards = nullptr;  // want_shards: the fetched rows, [fetch.size()][sp]
    size_t o_foff = 0, o_flen = 0, w_cmp = 0;
};

// shard rows hold every shard and every byte dec_src_pkt_info may read (the reference's buffers
// are dec_pkt_size long, zero-filled): `need` (verdicts: the largest head + size field among the
// rows; decodes: 0 -- a decoded row is zero past its inputs' longest shard, so a genuine packet
// fits; a row the pitch cuts short is re-decoded at dec_pkt_size + 4, see the decode loop)
inline void unpack_layout(UnpackBatch& b, Stage& io, Stage& work) {
    const size_t G = (size_t)b.groups, R = G * b.n;
    size_t maxd = 16;
    b.for_rows([&](int, const UnpackRow& r) { maxd = std::max(maxd, (size_t)r.len + (b.wrap ? 11u : 0u)); });
    b.sp = round16(std::max(maxd, std::min(b.need, (size_t)b.dec_pkt_size + 4)));
    b.wp = round16(b.sp + 13);
    b.o_off = io.take(R * 8);
    b.o_len = io.take(R * 4);
    b.o_rx = io.take(R * 4);
    b.o_st = io.take(G * b.k * 4);
    b.o_ps = io.take(G * b.k * 4);
    const size_t F = b.fetch.size();
    b.o_hsh = b.want_shards ? io.take(F * b.sp) : 0;
    b.o_foff = b.want_shards ? io.take(F * 8) : 0;
    b.o_flen = b.want_shards ? io.take(F * 4) : 0;
    b.w_cmp = b.want_shards ? work.take(F * b.sp + 16) : 0;
    b.w_wire = work.take(R * b.wp);
    b.w_wlen = work.take(R * 4);
    b.w_marks = work.take(R);
    b.w_sh = work.take(R * b.sp);
}

// fill the tables, gather the rows on the device, verdicts / decodes, results back (async)
inline int run_unpack(qfec_zfec* z, UnpackBatch& b, const uint8_t* d_rx, hipStream_t s) {
    const size_t G = (size_t)b.groups, R = G * b.n;
    uint8_t* h = z->io.h;
    uint8_t* d = z->d_io.d;
    uint8_t* w = z->d_work.d;
    unsigned long long* off = reinterpret_cast<unsigned long long*>(h + b.o_off);
    int* len = reinterpret_cast<int*>(h + b.o_len);
    memset(off, 0, R * 8);
    memset(len, 0, R * 4);
    b.for_rows([&](int g, const UnpackRow& r) {
        const size_t i = (size_t)g * b.n + r.ik;
        off[i] = r.off;
        len[i] = (int)r.len;
    });
    if (hipMemcpyAsync(d + b.o_off, h + b.o_off, b.o_rx - b.o_off, hipMemcpyHostToDevice, s) != hipSuccess)
        return QFEC_EHIP;
    int rc = qfec_gather_rows(d_rx, reinterpret_cast<const unsigned long long*>(d + b.o_off),
                              reinterpret_cast<const int*>(d + b.o_len), (long long)R, b.wrap ? b.n : 0,
                              b.wrap ? b.k : 0, w + b.w_wire, (long long)b.wp, reinterpret_cast<int*>(w + b.w_wlen), s);
    if (rc) return rc;
    rc = qfec_unpack_datagrams(code_for(z, b.k, b.n), w + b.w_wire, (long long)b.wp, reinterpret_cast<int*>(w + b.w_wlen),
                               (long long)G, b.checksum, b.dec_pkt_size, w + b.w_sh, (long long)b.sp, w + b.w_marks,
                               reinterpret_cast<int*>(d + b.o_rx), reinterpret_cast<int*>(d + b.o_st),
                               reinterpret_cast<int*>(d + b.o_ps), s);
    if (rc) return rc;
    if (hipMemcpyAsync(h + b.o_rx, d + b.o_rx, (b.o_ps + G * b.k * 4) - b.o_rx, hipMemcpyDeviceToHost, s) != hipSuccess)
        return QFEC_EHIP;
    if (b.want_shards && !b.fetch.empty()) {  // only the rows asked for, gathered on the device first
        const size_t F = b.fetch.size();
        unsigned long long* fo = reinterpret_cast<unsigned long long*>(h + b.o_foff);
        int* fl = reinterpret_cast<int*>(h + b.o_flen);
        for (size_t i = 0; i < F; ++i) {
            fo[i] = (unsigned long long)b.fetch[i] * b.sp;
            fl[i] = (int)b.sp;
        }
        if (hipMemcpyAsync(d + b.o_foff, h + b.o_foff, b.o_flen + F * 4 - b.o_foff, hipMemcpyHostToDevice, s) !=
            hipSuccess)
            return QFEC_EHIP;
        rc = qfec_gather_rows(w + b.w_sh, reinterpret_cast<const unsigned long long*>(d + b.o_foff),
                              reinterpret_cast<const int*>(d + b.o_flen), (long long)F, 0, 0, w + b.w_cmp,
                              (long long)b.sp, reinterpret_cast<int*>(d + b.o_flen), s);
        if (rc) return rc;
        if (hipMemcpyAsync(h + b.o_hsh, w + b.w_cmp, F * b.sp, hipMemcpyDeviceToHost, s) != hipSuccess) return QFEC_EHIP;
    }
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
    int batch = -1, group = -1, ik = 0;  // its place in the verdict launch
};

struct DecodeKey {  // a decode by content: the session, code, mode and exactly which rows
    int session = 0, k = 0, n = 0, mode = 0, dec_pkt_size = 0, nrows = 0;
    uint64_t uid[16] = {};  // slot uids in iValid order
    uint8_t ik[16] = {};
    bool operator==(const DecodeKey& o) const {
        if (session != o.session || k != o.k || n != o.n || mode != o.mode || dec_pkt_size != o.dec_pkt_size ||
            nrows != o.nrows)
            return false;
        for (int i = 0; i < nrows; ++i)
            if (uid[i] != o.uid[i] || ik[i] != o.ik[i]) return false;
        return true;
    }
};
struct DecodeKeyHash {
    size_t operator()(const DecodeKey& x) const {
        uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)x.session * 0x100000001B3ull;
        h = (h ^ ((uint64_t)x.k << 40 | (uint64_t)x.n << 32 | (uint64_t)x.mode << 24 | (uint64_t)(uint32_t)x.dec_pkt_size)) *
            0x100000001B3ull;
        for (int i = 0; i < x.nrows; ++i) h = (h ^ (x.uid[i] * 31 + x.ik[i])) * 0x100000001B3ull;
        return (size_t)(h ^ (h >> 29));
    }
};
struct DecodeOut {
    bool ok[16] = {};
    View payload[16];
};
struct DecodeReq {
    DecodeKey key;
    bool fresh = false;  // the first request of its key (the one that is launched)
    int nsh = 0;
    View shard[16];  // the k shards, ik in key.ik
    DecodeOut* out = nullptr;
};
using DecodeCache = std::unordered_map<DecodeKey, DecodeOut, DecodeKeyHash>;

struct RxPass {
    const DecodeCache* cache;
    std::vector<DecodeReq>* missing;
};

// the receive side of one session over its queued ops (NetFecCodec.cpp:189-371)
class RxMachine {
   public:
    RxMachine(Session& S, int sidx, const std::vector<Verdict>& verd, RxPass& pass, std::vector<Emit>& out)
        : S(S), R(S.rx), sidx(sidx), verd(verd), pass(pass), out(out) {}

    void run() {
        size_t v = 0;
        for (size_t oi = 0; oi < S.ops.size(); ++oi) {
            const Op& op = S.ops[oi];
            cur = (uint32_t)oi;
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
    std::vector<Emit>& out;
    uint32_t cur = 0;

    void deliver(const View& v, uint32_t src) {
        Emit e;
        e.op = cur;
        e.kind = 2;
        e.v = v;
        e.src = src;
        out.push_back(e);
    }
    // a decoded row: its payload, or a placeholder (kind 3) naming the request and row
    void deliver_decoded(const DecodeOut* res, int req, int i, uint32_t src) {
        if (res) {
            deliver(res->payload[i], src);
            return;
        }
        Emit e;
        e.op = cur;
        e.kind = 3;
        e.batch = req;
        e.row = i;
        e.src = src;
        out.push_back(e);
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
                    uint32_t seg_beg, const Op& op, int* max_size, int* rows, int* nrows, bool* undefined) {
        if (ipkt >= R.first && ipkt < R.second) {
            Slot& s = R.slots[ipkt - R.first];
            s.set_packet(vd.shard, uid, ik, vd.payload, op.off, op.size);
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
        const uint32_t size = op.size;
        if (size > (uint32_t)R.dec_pkt_size) R.dec_pkt_size = (int)size;  // unpack_fec_head realloc (:345-352)
        if (!vd.fec) {  // not an FEC datagram: handed over minus its tag, source index 0 (:201-209)
            if (size >= 1) deliver(View{SRC_RX, op.off + 1, size - 1}, 0u);
            return;
        }
        R.is_checksum = op.a == 0xED;  // (:364)
        if (!vd.ok || !vd.usable) return;  // (:210-213)
        const uint32_t i_recv = (uint32_t)op.b, src = (uint32_t)op.c;  // (header fields, parse_head)
        const uint32_t ikn = op_ikn(op);
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
        const bool dec = add_packet(i_recv, src, vd, op.uid, cur_ni, cur_k, cur_n, seg_beg, op, &max_size, rows, &nrows,
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
        key.nrows = nrows;
        for (int r = 0; r < nrows; ++r) {
            key.uid[r] = R.slots[rows[r]].uid;
            key.ik[r] = (uint8_t)R.slots[rows[r]].ik;
        }
        auto it = pass.cache->find(key);
        const DecodeOut* res = it == pass.cache->end() ? nullptr : &it->second;
        int req = -1;  // index of this decode's request (placeholders refer to it)
        if (!res && !pass.missing->empty() && pass.missing->back().key == key) {
            req = (int)pass.missing->size() - 1;  // the same decode as this session's last request
        } else if (!res) {
            pass.missing->emplace_back();
            DecodeReq& q = pass.missing->back();
            q.key = key;
            q.nsh = nrows;
            for (int r = 0; r < nrows; ++r) q.shard[r] = R.slots[rows[r]].shard;
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

inline void init_rx(RxState& R, int buf_items, int max_pkt, int kmax) {
    R.slots.assign((size_t)buf_items, Slot());  // init_zfec_layer :653-664
    R.first = 0;
    R.second = (uint32_t)buf_items;
    R.dec_pkt_size = packed_size(max_pkt);  // init_fec_buf :433-434
    R.dec_kmax = kmax;
    R.is_checksum = false;
}

// ---- the send machine of one session (zfec_pack_input, NetFecCodec.cpp:68-175): its closed
// groups (session-local ids; PackOut::batch is filled when the sessions' groups are merged) and
// its emits; the FEC-off datagrams [0x13][payload] go to the session's own buffer
struct LocalGroup {
    int k, n;
    PackGroup g;
};
inline void tx_machine(Session& S, std::vector<Emit>& out, std::vector<LocalGroup>& groups, std::vector<uint8_t>& own,
                const uint8_t* txa) {
    TxState& T = S.tx;
    std::vector<size_t> pending;  // emits of the open group's rows
    auto open_entry = [&](uint32_t oi, int row) {
        Emit e;
        e.op = oi;
        e.kind = 0;
        e.row = row;
        out.push_back(e);
        pending.push_back(out.size() - 1);
    };
    auto close_group = [&]() {  // the open group's rows so far, as one group
        LocalGroup lg;
        lg.k = T.gk;
        lg.n = T.gn;
        lg.g.sent0 = T.g_sent0;
        lg.g.src0 = T.g_src0;
        for (size_t i = 0; i < T.g_pay.size() && i < (size_t)T.gk; ++i) lg.g.pay[i] = T.g_pay[i];
        const long long gi = (long long)groups.size();
        groups.push_back(lg);
        for (size_t e : pending) {
            out[e].group = gi;
            out[e].batch = -1;
        }
        pending.clear();
    };
    for (size_t oi = 0; oi < S.ops.size(); ++oi) {
        const Op& op = S.ops[oi];
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
                e.op = (uint32_t)oi;
                e.kind = 1;
                e.v = View{SRC_OWN, (uint32_t)own.size(), op.size + 1};
                own.push_back(0x13);
                own.insert(own.end(), txa + op.off, txa + op.off + op.size);
                out.push_back(e);
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
                T.g_pay.push_back(View{SRC_TX, op.off, op.size});
                open_entry((uint32_t)oi, ik);
                T.i_sent_pkt++;
                T.i_sent_src_pkt++;
            }
            if (ik == k - 1) {  // the check packets (:133-172)
                for (int j = k; j < n; ++j) {
                    open_entry((uint32_t)oi, j);
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

inline unsigned flush_threads(size_t work, size_t sessions) {
    // at most 8: a CPU quota (the box gives a process 16 CPUs) throttles a flush that runs more
    // threads than it allows for a whole scheduling period
    unsigned t = work < 4096 ? 1u : std::max(1u, std::min({8u, std::thread::hardware_concurrency(), (unsigned)sessions}));
    if (const char* e = getenv("QFEC_ZFEC_RX_THREADS"))  // tests: force the threaded machines
        t = (unsigned)std::max(1, std::min(64, atoi(e)));
    return t;
}

}  // namespace qfec_zfec_impl
