// qfec_rs_abi.cpp -- module/rs.h on the GPU: reed_solomon_init / new / release / encode /
// reconstruct / error (module/rs.h:22-49, module/rs.c:387-643).  Every caller shard pointer is
// classified; arrays of host pointers run the two-slot pipelines below, device arrays run in place,
// mixes are staged row by row.
#include "qfec_rt.hpp"

#include <immintrin.h>

using namespace qfec;

// ====================================================================== host-buffer paths
namespace {

// rows laid out back to back from ptrs[0] with stride len (a contiguous device batch)
bool contiguous(unsigned char* const* ptrs, size_t count, int len) {
    for (size_t i = 1; i < count; ++i)
        if (ptrs[i] != ptrs[0] + i * (size_t)len) return false;
    return true;
}

constexpr size_t kChunkBytes = (size_t)256 << 20;  // staging chunk for host-buffer batches

// ---- module/rs.h on arrays of caller shard pointers (round 5)
//
// Kinds of caller pointers: device (or managed) memory against host memory.  A device verdict
// comes only from the runtime (hipPointerGetAttributes), and the whole allocation it belongs to
// (hipMemGetAddressRange) then answers for later pointers without a probe.  A host verdict is
// reused for other pointers in the same 64 KiB window, within one call only.  Device allocations
// are placed in the GPU address apertures the runtime reserves, which host mappings do not share
// at that granularity; a managed allocation that a reused host verdict covers is still memory
// the CPU copies can read and write.  So no reused verdict can move a wrong byte.
struct PtrClass {
    std::map<uintptr_t, uintptr_t> dev;      // device allocation ranges, lo -> hi (ordered,
                                             // so arrays of many separate allocations stay O(log n))
    std::unordered_set<uintptr_t> host_win;  // 64 KiB windows with a host verdict
    uintptr_t last_lo = 0, last_hi = 0, last_win = ~(uintptr_t)0;
    bool is_dev(const void* p) {
        const uintptr_t u = (uintptr_t)p, w = u >> 16;
        if (u >= last_lo && u < last_hi) return true;
        auto it = dev.upper_bound(u);
        if (it != dev.begin() && u < (--it)->second) {
            last_lo = it->first;
            last_hi = it->second;
            return true;
        }
        if (w == last_win) return false;
        if (host_win.count(w)) {
            last_win = w;
            return false;
        }
        hipPointerAttribute_t attr;
        const hipError_t e = hipPointerGetAttributes(&attr, p);
        if (e == hipSuccess && (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged)) {
            void* base = nullptr;
            size_t size = 0;
            if (hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) == hipSuccess && base && size) {
                last_lo = (uintptr_t)base;
                last_hi = last_lo + size;
            } else {
                (void)hipGetLastError();
                last_lo = u;  // this pointer only
                last_hi = u + 1;
            }
            dev[last_lo] = last_hi;
            return true;
        }
        if (e != hipSuccess) (void)hipGetLastError();
        host_win.insert(w);
        last_win = w;
        return false;
    }
};


constexpr size_t kMapsMinPointers = 4096;

// kind of every pointer of ptrs[0 .. count) (kind[i] = 1: device or managed memory; kind may be
// null), classified on the host pool's threads; returns the number of device pointers
size_t classify_ptrs(unsigned char* const* ptrs, size_t count, HostPool& pool, uint8_t* kind) {
    // reading the maps costs ~0.1-0.3 ms: worth it for large arrays only; a call with a few
    // groups probes its pointers directly (a probe per 64 KiB window, ~0.1 us each)
    MapSnap maps;
    const bool have_maps = count >= kMapsMinPointers && maps.load();
    std::atomic<size_t> ndev{0};
    pool.run(
        [&](int t, int nt) {
            PtrClass pc;
            size_t nd = 0, hint = 0;
            const size_t a = count * t / nt, b = count * (t + 1) / nt;
            for (size_t i = a; i < b; ++i) {
                const bool d = !(have_maps && maps.host((uintptr_t)ptrs[i], &hint)) && pc.is_dev(ptrs[i]);
                if (kind) kind[i] = d ? 1 : 0;
                nd += d ? 1 : 0;
            }
            ndev += nd;
        },
        (int)std::max<size_t>(1, count >> 14));
    return ndev.load();
}

// rows of mixed kinds to a device staging area: the host rows through the pinned stage at h_tmp
// (copied on the pool's threads, then one DMA for the whole area), the device rows one copy each,
// queued after it on the same stream (host rows no longer take one pageable copy each)
int gather_rows_kind(DevCtx& c, unsigned char* const* ptrs, const uint8_t* kind, size_t count, int len, size_t pitch,
                     uint8_t* d_dst, uint8_t* h_tmp, HostPool& pool) {
    size_t nh = 0;
    for (size_t i = 0; i < count; ++i) nh += kind[i] ? 0 : 1;
    if (nh) {
        pool.run(
            [&](int t, int nt) {
                for (size_t i = count * t / nt, b = count * (t + 1) / nt; i < b; ++i)
                    if (!kind[i]) memcpy(h_tmp + i * pitch, ptrs[i], (size_t)len);
            },
            (int)std::max<size_t>(1, nh / 64));
        HIP_TRY(hipMemcpyAsync(d_dst, h_tmp, count * pitch, hipMemcpyHostToDevice, c.stream));
    }
    for (size_t i = 0; i < count; ++i)
        if (kind[i]) HIP_TRY(hipMemcpyAsync(d_dst + i * pitch, ptrs[i], (size_t)len, hipMemcpyDefault, c.stream));
    return QFEC_OK;
}

// the reverse, for the rows `only` marks (nullable: all); returns after every row is written
int scatter_rows_kind(DevCtx& c, unsigned char* const* ptrs, const uint8_t* kind, size_t count, int len,
                      size_t pitch, const uint8_t* d_src, uint8_t* h_tmp, const uint8_t* only, HostPool& pool) {
    size_t nh = 0;
    for (size_t i = 0; i < count; ++i) nh += (!kind[i] && (!only || only[i])) ? 1 : 0;
    if (nh) HIP_TRY(hipMemcpyAsync(h_tmp, d_src, count * pitch, hipMemcpyDeviceToHost, c.stream));
    for (size_t i = 0; i < count; ++i)
        if (kind[i] && (!only || only[i]))
            HIP_TRY(hipMemcpyAsync(ptrs[i], d_src + i * pitch, (size_t)len, hipMemcpyDefault, c.stream));
    HIP_TRY(hipStreamSynchronize(c.stream));
    if (nh)
        pool.run(
            [&](int t, int nt) {
                for (size_t i = count * t / nt, b = count * (t + 1) / nt; i < b; ++i)
                    if (!kind[i] && (!only || only[i])) memcpy(ptrs[i], h_tmp + i * pitch, (size_t)len);
            },
            (int)std::max<size_t>(1, nh / 64));
    return QFEC_OK;
}

// QFEC_RS_TRACE=1: where a host-pointer call's time goes (host gather, event waits, host scatter),
// printed per call to stderr
thread_local double t_rs_classify = 0;  // seconds the entry spent classifying the pointers
thread_local std::chrono::steady_clock::time_point t_rs_entry;  // when the ABI entry was called

struct RsTrace {
    bool on = getenv("QFEC_RS_TRACE") != nullptr;
    double gather = 0, wait = 0, scatter = 0;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    static double since(std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
    }
    void report(const char* what, long long chunks, int threads) const {
        if (on)
            fprintf(stderr,
                    "[qfec] %s: %.2f ms in the call (classify %.2f, pipeline %.2f: gather %.2f, wait %.2f, scatter %.2f "
                    "ms); %lld chunks, %d threads\n",
                    what, since(t_rs_entry) * 1e3, t_rs_classify * 1e3, since(t0) * 1e3, gather * 1e3, wait * 1e3,
                    scatter * 1e3, chunks, threads);
    }
};

// the staged (device or mixed pointer) paths under QFEC_RS_TRACE
void staged_report(const char* what, size_t ndev, size_t nptr) {
    if (getenv("QFEC_RS_TRACE"))
        fprintf(stderr, "[qfec] %s: %.2f ms in the call (classify %.2f ms); %zu of %zu pointers device memory\n", what,
                RsTrace::since(t_rs_entry) * 1e3, t_rs_classify * 1e3, ndev, nptr);
}

// bytes of caller shards per pipelined chunk of the host-pointer paths (tuning "host_chunk"
// overrides with groups per chunk)
constexpr size_t kRsPipeBytes = (size_t)16 << 20;

// the slot's device view: the pinned staging itself (zero copy) or the slot's device buffer
uint8_t* rs_slot_dev(DevCtx::HostSlot& h, bool zc) {
    uint8_t* z = nullptr;
    if (zc && host_dev(h.h_in, &z)) return z;
    return nullptr;
}

// a caller row into a pinned slot with streaming stores (tuning "host_nt"): the slot is read next by
// the device (DMA or zero-copy reads over PCIe), not by this CPU, so its lines need not be fetched
// for ownership first; the caller's thread fences (sfence) before the slot is handed over
inline void copy_row_nt(uint8_t* dst, const uint8_t* src, size_t len) {
    if (((uintptr_t)dst & 15) || len < 64) {
        memcpy(dst, src, len);
        return;
    }
    size_t i = 0;
    for (; i + 64 <= len; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    }
    if (i < len) memcpy(dst + i, src + i, len - i);
}

// one thread's run of row copies into a slot.  Streaming stores pay when the caller's rows follow one
// another in memory (the loads stream, and the stores' ownership reads are the traffic saved); on rows
// at scattered places the loads are latency-bound and the streaming stores lose (profiles/r06r).  So
// host_nt 2 (the default) streams a row only when it starts where the previous row of the same run
// ended (up to 4 KiB on); 1 streams every row, 0 none.
struct RowRun {
    int mode;
    size_t len;
    uintptr_t next = 0;
    void operator()(uint8_t* dst, const uint8_t* src) {
        const bool seq = (uintptr_t)src - next <= 4096;
        next = (uintptr_t)src + len;
        if (mode == 1 || (mode == 2 && seq)) copy_row_nt(dst, src, len);
        else memcpy(dst, src, len);
    }
    void fence() const {
        if (mode) _mm_sfence();
    }
};

// ---- where the host-pointer pipelines run their chunks: host_lanes slots on the calling thread's
// device (its context's own host slots; 4 by default: at config 2's shape, interleaved in one
// process, 2 / 4 / 6 / 8 slots 35.6 / 43.3 / 43.4 / 42.7 GiB/s, profiles/r06o), or two slots per entry of the list
// qfec_rs_host_devices set (own slots per entry, so a device may be listed more than once).  Chunk i takes lane i % lanes; a lane
// is one slot of one entry, with the entry's device, context and code tables.
struct RsLane {
    int device = 0;
    DevCtx* ctx = nullptr;
    DevCtx::HostSlot* h = nullptr;
    const uint32_t* tab = nullptr;  // encode tables on the lane's device
    const DevTables* d = nullptr;   // LUT and records on the lane's device
};

struct RsDevList {
    std::mutex mu;                                      // held by a call for its whole pipeline
    std::vector<int> devs;                              // empty: the current device
    std::vector<std::unique_ptr<DevCtx::HostSlot>> slots;  // 2 per entry
};
RsDevList& rs_devlist() {
    static RsDevList* l = new RsDevList();  // never destroyed: no slot freed after the runtime's exit
    return *l;
}

void free_slot(DevCtx::HostSlot& h) {
    if (h.stream) (void)hipStreamSynchronize(h.stream);
    if (h.d_buf) (void)hipFree(h.d_buf);
    if (h.h_in) (void)hipHostFree(h.h_in);
    if (h.h_out) (void)hipHostFree(h.h_out);
    if (h.done) (void)hipEventDestroy(h.done);
    if (h.stream) (void)hipStreamDestroy(h.stream);
    h = DevCtx::HostSlot();
    (void)hipGetLastError();
}

struct DeviceBack {  // the caller's current device, put back on every way out
    int prev = -1;
    DeviceBack() { if (hipGetDevice(&prev) != hipSuccess) prev = -1; }
    ~DeviceBack() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// the lanes of one call, each slot sized for `in_bytes` / `out_bytes` and the code's tables made
// current on its device (`enc`: encode tables, else LUT + records).  `lk` receives the lock that
// keeps the slots the call's until it returns.
int rs_lanes(DevCtx& cur, qfec_code* c, bool enc, size_t in_bytes, size_t out_bytes, std::vector<RsLane>& lanes,
             std::unique_lock<std::mutex>& lk) {
    RsDevList& L = rs_devlist();
    std::unique_lock<std::mutex> ll(L.mu);
    int rc = QFEC_OK;
    auto tables = [&](RsLane& ln) -> int {
        std::lock_guard<std::mutex> cl(c->mu);
        if (enc) {
            uint32_t* t = nullptr;
            const int r = ensure_enc(c, ln.device, &t);
            ln.tab = t;
            return r;
        }
        DevTables* d = nullptr;
        const int r = ensure_lut(c, ln.device, &d);
        ln.d = d;
        return r;
    };
    lanes.clear();
    if (L.devs.empty()) {
        ll.unlock();
        lk = std::unique_lock<std::mutex>(cur.host_mu);
        const int nl = std::max(2, std::min((int)tuning().host_lanes.load(), kMaxHostLanes));
        for (int sl = 0; sl < nl; ++sl) {
            DevCtx::HostSlot& h = cur.host[sl];
            if ((rc = ensure_host_slot(h, in_bytes, out_bytes))) return rc;
            RsLane ln;
            ln.device = cur.device;
            ln.ctx = &cur;
            ln.h = &h;
            if ((rc = tables(ln))) return rc;
            lanes.push_back(ln);
        }
        return QFEC_OK;
    }
    for (size_t e = 0; e < L.devs.size(); ++e) {
        HIP_TRY(hipSetDevice(L.devs[e]));
        DevCtx* ctx = nullptr;
        if ((rc = current_ctx(&ctx))) return rc;
        for (int sl = 0; sl < 2; ++sl) {
            DevCtx::HostSlot& h = *L.slots[e * 2 + sl];
            if ((rc = ensure_host_slot(h, in_bytes, out_bytes))) return rc;
            RsLane ln;
            ln.device = L.devs[e];
            ln.ctx = ctx;
            ln.h = &h;
            if ((rc = tables(ln))) return rc;
            lanes.push_back(ln);
        }
    }
    // slot sl of every entry first, so consecutive chunks land on different entries
    std::vector<RsLane> order;
    for (int sl = 0; sl < 2; ++sl)
        for (size_t e = 0; e < L.devs.size(); ++e) order.push_back(lanes[e * 2 + sl]);
    lanes.swap(order);
    lk = std::move(ll);
    return QFEC_OK;
}

// after an error: wait for whatever the lanes still have in flight
void quiesce_lanes(std::vector<RsLane>& lanes) {
    for (auto& ln : lanes) {
        (void)hipSetDevice(ln.device);
        if (ln.h->stream) (void)hipStreamSynchronize(ln.h->stream);
    }
    (void)hipGetLastError();
}

// reed_solomon_encode over host shard pointers: chunks of groups go round the lanes; the host
// threads gather a chunk's data rows into its lane's pinned slot while the devices encode the chunks
// before it (through the slot's device buffer), and scatter each chunk's parity rows once its event
// has fired -- the oldest chunk first, once every lane is busy.
int rs_encode_pipe(DevCtx& ctx, qfec_code* c, unsigned char** data, unsigned char** par, long long G, int B,
                   bool any_stale) {
    const int k = c->k, m = c->m;
    const size_t pitch = round_up((size_t)B, 16), dg = (size_t)k * pitch, pg = (size_t)m * pitch;
    long long per = tuning().host_chunk > 0 ? (long long)tuning().host_chunk
                                            : std::max<long long>(1, (long long)(kRsPipeBytes / (dg + pg)));
    per = std::min(per, G);
    const size_t slot_bytes = (size_t)per * (dg + pg);
    std::shared_ptr<HostPool> pool = host_pool();
    DeviceBack back;
    std::vector<RsLane> lanes;
    std::unique_lock<std::mutex> lk;
    int rc = rs_lanes(ctx, c, true, slot_bytes, 16, lanes, lk);
    if (rc) return rc;
    const size_t W = lanes.size();
    // staged: the DMA engines move the slot to the device and the parity back.  Reading the
    // freshly gathered slot in place over PCIe ran slower for the encode (26.4-26.9 against
    // 28.3-38.8 GiB/s in alternating processes, profiles/r05af); the reconstruct, which reads only
    // the survivors it needs and writes only the erased rows, stays in place (host_zero_copy)
    const bool zc = false;
    RsTrace tr;
    std::vector<long long> pending(W, -1);
    auto rows_job = [&](size_t nrows, const std::function<void(size_t)>& row) {
        pool->run(
            [&](int t, int nt) {
                const size_t a = nrows * t / nt, b = nrows * (t + 1) / nt;
                for (size_t i = a; i < b; ++i) row(i);
            },
            (int)std::max<size_t>(1, nrows / 64));
    };
    auto drain = [&](size_t ln) -> int {
        if (pending[ln] < 0) return QFEC_OK;
        DevCtx::HostSlot& h = *lanes[ln].h;
        auto tw = std::chrono::steady_clock::now();
        HIP_TRY(hipEventSynchronize(h.done));
        tr.wait += RsTrace::since(tw);
        tw = std::chrono::steady_clock::now();
        const long long g0 = pending[ln], gn = std::min(per, G - g0);
        const uint8_t* hp = h.h_in + (size_t)gn * dg;
        rows_job((size_t)gn * m, [&](size_t i) { memcpy(par[(size_t)g0 * m + i], hp + i * pitch, (size_t)B); });
        tr.scatter += RsTrace::since(tw);
        pending[ln] = -1;
        return QFEC_OK;
    };
    const long long nchunks = (G + per - 1) / per;
    for (long long i = 0; i < nchunks && !rc; ++i) {
        const size_t ln = (size_t)(i % (long long)W);
        if ((rc = drain(ln))) break;  // the lane's previous chunk (only when every lane is busy)
        RsLane& L = lanes[ln];
        DevCtx::HostSlot& h = *L.h;
        const long long g0 = i * per, gn = std::min(per, G - g0);
        uint8_t* hd = h.h_in;
        uint8_t* hp = h.h_in + (size_t)gn * dg;
        // data rows (and, when a parity row keeps its old bytes -- the rs.c quirk -- the parity rows)
        const size_t nd = (size_t)gn * k, np = any_stale ? (size_t)gn * m : 0;
        const auto tg = std::chrono::steady_clock::now();
        const int nt = tuning().host_nt;
        pool->run(
            [&](int t, int nth) {
                const size_t rows = nd + np, a = rows * t / nth, b = rows * (t + 1) / nth;
                RowRun put{nt, (size_t)B};
                for (size_t r = a; r < b; ++r) {
                    if (r < nd) put(hd + r * pitch, data[(size_t)g0 * k + r]);
                    else put(hp + (r - nd) * pitch, par[(size_t)g0 * m + (r - nd)]);
                }
                put.fence();
            },
            (int)std::max<size_t>(1, (nd + np) / 64));
        tr.gather += RsTrace::since(tg);
        if (hipSetDevice(L.device) != hipSuccess) { rc = hip_fail(hipGetLastError(), "reed_solomon_encode: device"); break; }
        uint8_t* z = rs_slot_dev(h, zc);
        uint8_t* dd = z ? z : h.d_buf;
        if (!z) {
            const hipError_t e = hipMemcpyAsync(dd, hd, (size_t)gn * dg + np * pitch, hipMemcpyHostToDevice, h.stream);
            if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_encode: H2D"); break; }
        }
        if ((rc = run_encode(*L.ctx, c, L.tab, m, dd, dd + (size_t)gn * dg, gn, B, (long long)pitch, h.stream))) break;
        if (!z) {
            const hipError_t e = hipMemcpyAsync(hp, dd + (size_t)gn * dg, (size_t)gn * pg, hipMemcpyDeviceToHost, h.stream);
            if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_encode: D2H"); break; }
        }
        const hipError_t e = hipEventRecord(h.done, h.stream);
        if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_encode: event"); break; }
        pending[ln] = g0;
        // the oldest chunk in flight, while this one runs (two lanes: the previous chunk)
        if (i + 1 >= (long long)W && (rc = drain((size_t)((i + 1) % (long long)W)))) break;
    }
    for (size_t j = 0; j < W && !rc; ++j) rc = drain((size_t)((nchunks + (long long)j) % (long long)W));  // oldest first
    if (rc) quiesce_lanes(lanes);  // nothing may still be writing into the slots
    tr.report("reed_solomon_encode (host)", nchunks, pool->threads());
    return rc;
}

// reed_solomon_reconstruct over host shard pointers (k + m <= QFEC_LUT_MAX_N): the same lanes.  Per
// group only what the decode reads is staged -- the surviving data rows and the first e surviving
// parity rows (rs.c:611-629), plus the erased rows where the pattern's record seeds a row from its
// old bytes (the rs.c quirk) -- with the chunk's marks in rs.c layout; the LUT kernel decodes and
// only the erased data rows of recoverable groups are scattered back.  Groups with more erased data
// than surviving parity are left untouched and counted (*nfail).
int rs_reconstruct_pipe(DevCtx& ctx, qfec_code* c, const uint8_t* seed, unsigned char** data, unsigned char** par,
                        const uint8_t* mk, long long G, int B, long long* nfail) {
    const int k = c->k, m = c->m, n = k + m;
    const size_t pitch = round_up((size_t)B, 16), dg = (size_t)k * pitch, pg = (size_t)m * pitch;
    long long per = tuning().host_chunk > 0 ? (long long)tuning().host_chunk
                                            : std::max<long long>(1, (long long)(kRsPipeBytes / (dg + pg)));
    per = std::min(per, G);
    const size_t mk_off = (size_t)per * (dg + pg), slot_bytes = round_up(mk_off + (size_t)per * n, 16);
    std::shared_ptr<HostPool> pool = host_pool();
    DeviceBack back;
    std::vector<RsLane> lanes;
    std::unique_lock<std::mutex> lk;
    int rc = rs_lanes(ctx, c, false, slot_bytes, 16, lanes, lk);
    if (rc) return rc;
    const size_t W = lanes.size();
    const bool zc = tuning().host_zero_copy != 0;
    RsTrace tr;
    std::vector<std::vector<uint8_t>> todo(W);  // per lane, per group: 1 = decoded (scatter its erased data rows)
    std::vector<long long> pending(W, -1);
    std::atomic<long long> fails{0};
    auto groups_job = [&](long long gn, const std::function<void(long long, long long)>& span) {
        pool->run(
            [&](int t, int nt) { span(gn * t / nt, gn * (t + 1) / nt); }, (int)std::max<long long>(1, gn / 16));
    };
    auto drain = [&](size_t ln) -> int {
        if (pending[ln] < 0) return QFEC_OK;
        DevCtx::HostSlot& h = *lanes[ln].h;
        auto tw = std::chrono::steady_clock::now();
        HIP_TRY(hipEventSynchronize(h.done));
        tr.wait += RsTrace::since(tw);
        tw = std::chrono::steady_clock::now();
        const long long g0 = pending[ln], gn = std::min(per, G - g0);
        const uint8_t* todo_s = todo[ln].data();
        const uint8_t* hd = h.h_in;
        groups_job(gn, [&](long long a, long long b) {
            for (long long g = a; g < b; ++g) {
                if (!todo_s[g]) continue;
                const uint8_t* dm = mk + (size_t)(g0 + g) * k;
                for (int i = 0; i < k; ++i)
                    if (dm[i]) memcpy(data[(size_t)(g0 + g) * k + i], hd + ((size_t)g * k + i) * pitch, (size_t)B);
            }
        });
        tr.scatter += RsTrace::since(tw);
        pending[ln] = -1;
        return QFEC_OK;
    };
    const long long nchunks = (G + per - 1) / per;
    for (long long i = 0; i < nchunks && !rc; ++i) {
        const size_t ln = (size_t)(i % (long long)W);
        if ((rc = drain(ln))) break;
        RsLane& L = lanes[ln];
        DevCtx::HostSlot& h = *L.h;
        const long long g0 = i * per, gn = std::min(per, G - g0);
        uint8_t* hd = h.h_in;
        uint8_t* hp = h.h_in + (size_t)gn * dg;
        uint8_t* hm = h.h_in + (size_t)gn * (dg + pg);
        todo[ln].assign((size_t)gn, 0);
        uint8_t* todo_s = todo[ln].data();
        const auto tg = std::chrono::steady_clock::now();
        const int nt = tuning().host_nt;
        groups_job(gn, [&](long long a, long long b) {
            RowRun put_d{nt, (size_t)B}, put_p{nt, (size_t)B};  // data rows and parity rows: two runs
            long long nf = 0;
            for (long long g = a; g < b; ++g) {
                const size_t gg = (size_t)(g0 + g);
                const uint8_t* dm = mk + gg * k;
                const uint8_t* pm = mk + (size_t)G * k + gg * m;
                memcpy(hm + (size_t)g * k, dm, (size_t)k);
                memcpy(hm + (size_t)gn * k + (size_t)g * m, pm, (size_t)m);
                uint32_t mask = 0;
                int e = 0;
                for (int x = 0; x < k; ++x)
                    if (dm[x]) { mask |= 1u << x; ++e; }
                if (!e) continue;
                for (int j = 0; j < m; ++j)
                    if (pm[j]) mask |= 1u << (k + j);
                int got = 0;
                for (int j = 0; j < m && got < e; ++j)
                    if (!pm[j]) {
                        put_p(hp + ((size_t)g * m + j) * pitch, par[gg * m + j]);
                        ++got;
                    }
                if (got < e) {  // under-determined: left as it is (rs.c:630-634)
                    ++nf;
                    continue;
                }
                const bool sd = seed[mask] != 0;
                for (int x = 0; x < k; ++x)
                    if (!dm[x] || sd) put_d(hd + ((size_t)g * k + x) * pitch, data[gg * k + x]);
                todo_s[g] = 1;
            }
            put_d.fence();
            fails += nf;
        });
        tr.gather += RsTrace::since(tg);
        if (hipSetDevice(L.device) != hipSuccess) {
            rc = hip_fail(hipGetLastError(), "reed_solomon_reconstruct: device");
            break;
        }
        uint8_t* z = rs_slot_dev(h, zc);
        uint8_t* dd = z ? z : h.d_buf;
        const size_t used = (size_t)gn * (dg + pg + n);
        if (!z) {
            const hipError_t e = hipMemcpyAsync(dd, h.h_in, used, hipMemcpyHostToDevice, h.stream);
            if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_reconstruct: H2D"); break; }
        }
        if ((rc = run_reconstruct(*L.ctx, c, L.d->d_lut, nullptr, L.d->d_rec, dd, dd + (size_t)gn * dg,
                                  dd + (size_t)gn * (dg + pg), gn, B, (long long)pitch, nullptr, h.stream)))
            break;
        if (!z) {
            const hipError_t e = hipMemcpyAsync(h.h_in, dd, (size_t)gn * dg, hipMemcpyDeviceToHost, h.stream);
            if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_reconstruct: D2H"); break; }
        }
        const hipError_t e = hipEventRecord(h.done, h.stream);
        if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_reconstruct: event"); break; }
        pending[ln] = g0;
        if (i + 1 >= (long long)W && (rc = drain((size_t)((i + 1) % (long long)W)))) break;
    }
    for (size_t j = 0; j < W && !rc; ++j) rc = drain((size_t)((nchunks + (long long)j) % (long long)W));
    if (rc) quiesce_lanes(lanes);
    *nfail = fails.load();
    tr.report("reed_solomon_reconstruct (host)", nchunks, pool->threads());
    return rc;
}

}  // namespace

// ====================================================================== module/rs.h ABI
namespace {

struct rs_handle {
    reed_solomon pub;  // must stay first: callers see only this prefix (rs.h:7-13)
    qfec_code* code;
};

std::atomic<int> g_rs_errno{0};
std::once_flag g_rs_init_once;

// pick up edits callers made to the public matrices since the last call: encode reads
// `parity` (rs.c:583), reconstruct reads `m` (rs.c:505, 536-548); the two are separate copies
void sync_rows(rs_handle* h) {
    qfec_code* c = h->code;
    std::lock_guard<std::mutex> lk(c->mu);
    if (memcmp(c->rows.data(), h->pub.parity, c->rows.size()) != 0) {
        memcpy(c->rows.data(), h->pub.parity, c->rows.size());
        ++c->version;
    }
    if (memcmp(c->full.data(), h->pub.m, c->full.size()) != 0) {
        memcpy(c->full.data(), h->pub.m, c->full.size());
        ++c->version;
    }
}

}  // namespace

extern "C" {

int qfec_rs_host_devices(const int* devices, int n) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        set_error("qfec_rs_host_devices: no HIP device available");
        return QFEC_ENODEV;
    }
    if (n < 0 || n > 64 || (n > 0 && !devices)) {
        set_error("qfec_rs_host_devices: invalid argument");
        return QFEC_EINVAL;
    }
    for (int i = 0; i < n; ++i)
        if (devices[i] < 0 || devices[i] >= count || devices[i] >= kMaxDevices) {
            set_error("qfec_rs_host_devices: device %d out of range (%d visible)", devices[i], count);
            return QFEC_EINVAL;
        }
    RsDevList& L = rs_devlist();
    std::lock_guard<std::mutex> lk(L.mu);  // no pipeline is using the slots
    DeviceBack back;
    for (size_t i = 0; i < L.slots.size(); ++i) {
        (void)hipSetDevice(L.devs[i / 2]);
        free_slot(*L.slots[i]);
    }
    L.devs.assign(devices, devices + n);
    L.slots.clear();
    for (int i = 0; i < 2 * n; ++i) L.slots.emplace_back(new DevCtx::HostSlot());
    return QFEC_OK;
}

int qfec_rs_host_devices_get(int* devices, int cap) {
    if (cap < 0 || (cap > 0 && !devices)) return QFEC_EINVAL;
    RsDevList& L = rs_devlist();
    std::lock_guard<std::mutex> lk(L.mu);
    for (int i = 0; i < cap && i < (int)L.devs.size(); ++i) devices[i] = L.devs[i];
    return (int)L.devs.size();
}

void reed_solomon_init(void) {
    std::call_once(g_rs_init_once, [] { (void)field(); });
}

reed_solomon* reed_solomon_new(int data_shards, int parity_shards) {
    reed_solomon_init();
    int err = 0;
    const int k = data_shards, m = parity_shards, n = k + m;
    rs_handle* h = nullptr;
    do {
        if (n > DATA_SHARDS_MAX || k <= 0 || m <= 0) { err = 1; break; }  // rs.c:404-407
        h = (rs_handle*)calloc(1, sizeof(rs_handle));
        if (!h) { err = 2; break; }
        h->pub.data_shards = k;
        h->pub.parity_shards = m;
        h->pub.shards = n;
        h->pub.m = (unsigned char*)calloc((size_t)n * k, 1);
        h->pub.parity = (unsigned char*)calloc((size_t)m * k, 1);
        if (!h->pub.m || !h->pub.parity) { err = 4; break; }
        std::vector<uint8_t> rows;
        if (!cauchy_rows(k, m, rows)) { err = 1; break; }
        for (int i = 0; i < k; ++i) h->pub.m[(size_t)i * k + i] = 1;
        memcpy(h->pub.m + (size_t)k * k, rows.data(), rows.size());
        memcpy(h->pub.parity, rows.data(), rows.size());
        h->code = make_code(k, m, std::move(rows), 1);
        if (!h->code) { err = 5; break; }
        h->code->full.assign(h->pub.m, h->pub.m + (size_t)n * k);
        g_rs_errno = 0;
        return &h->pub;
    } while (0);
    g_rs_errno = err;
    fprintf(stderr, "err=%d\n", err);  // rs.c:458
    if (h) {
        free(h->pub.m);
        free(h->pub.parity);
        free(h);
    }
    return nullptr;
}

void reed_solomon_release(reed_solomon* rs) {
    if (!rs) return;
    rs_handle* h = (rs_handle*)rs;
    free_code(h->code);
    free(h->pub.m);
    free(h->pub.parity);
    free(h);
}

int reed_solomon_error(void) { return g_rs_errno.load(); }

qfec_code* qfec_rs_code(reed_solomon* rs) {
    if (!rs) return nullptr;
    rs_handle* h = (rs_handle*)rs;
    sync_rows(h);
    return h->code;
}

int reed_solomon_encode(reed_solomon* rs, unsigned char** shards, int nr_shards, int block_size) {
    if (!rs || !shards) return 0;
    rs_handle* h = (rs_handle*)rs;
    const int k = rs->data_shards, m = rs->parity_shards, n = rs->shards;
    const long long G = nr_shards / n;
    if (G <= 0 || block_size <= 0) return 0;
    t_rs_entry = std::chrono::steady_clock::now();
    sync_rows(h);
    qfec_code* c = h->code;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) { fprintf(stderr, "[qfec] reed_solomon_encode: %s\n", qfec_last_error()); return rc; }
    uint32_t* tab = nullptr;
    bool any_stale = false;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        rc = ensure_enc(c, ctx->device, &tab);
        for (int r = 0; r < m; ++r) any_stale |= c->rows[(size_t)r * k] == 0;
    }
    if (rc) { fprintf(stderr, "[qfec] reed_solomon_encode: %s\n", qfec_last_error()); return rc; }
    unsigned char** data = shards;
    unsigned char** par = shards + G * k;
    // every shard pointer is classified: all host -> the pipelined host path, all device and
    // contiguous -> in place, otherwise staged by kind (host rows through the pinned stage, device
    // rows one copy each)
    const size_t nptr = (size_t)G * n;
    const auto tc = std::chrono::steady_clock::now();
    std::shared_ptr<HostPool> pool = host_pool();
    std::vector<uint8_t> kind(nptr);
    const size_t ndev = classify_ptrs(shards, nptr, *pool, kind.data());
    t_rs_classify = RsTrace::since(tc);
    if (ndev == 0) {
        rc = rs_encode_pipe(*ctx, c, data, par, G, block_size, any_stale);
        if (rc) fprintf(stderr, "[qfec] reed_solomon_encode: %s\n", qfec_last_error());
        return rc;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (ndev == nptr && contiguous(data, (size_t)G * k, block_size) && contiguous(par, (size_t)G * m, block_size)) {
        rc = run_encode(*ctx, c, tab, m, data[0], par[0], G, block_size, block_size, ctx->stream);
        if (!rc) rc = hipStreamSynchronize(ctx->stream) == hipSuccess ? 0 : QFEC_EHIP;
        if (rc) fprintf(stderr, "[qfec] reed_solomon_encode: %s\n", qfec_last_error());
        return rc;
    }
    const size_t pitch = round_up((size_t)block_size, 16);
    const long long per = tuning().host_chunk > 0 ? (long long)tuning().host_chunk
                                                  : std::max<long long>(1, (long long)(kChunkBytes / ((size_t)n * pitch)));
    for (long long g0 = 0; g0 < G && !rc; g0 += per) {
        const long long gn = std::min(per, G - g0);
        const size_t dbytes = (size_t)gn * k * pitch, pbytes = (size_t)gn * m * pitch;
        if ((rc = ensure_stage(*ctx, dbytes + pbytes, dbytes + pbytes))) break;
        uint8_t* d_d = ctx->d_stage;
        uint8_t* d_p = ctx->d_stage + dbytes;
        const uint8_t* kd = kind.data() + g0 * k;
        const uint8_t* kp = kind.data() + (size_t)G * k + g0 * m;
        if ((rc = gather_rows_kind(*ctx, data + g0 * k, kd, (size_t)gn * k, block_size, pitch, d_d, ctx->h_stage, *pool)))
            break;
        if (any_stale && (rc = gather_rows_kind(*ctx, par + g0 * m, kp, (size_t)gn * m, block_size, pitch, d_p,
                                                ctx->h_stage + dbytes, *pool)))
            break;
        if ((rc = run_encode(*ctx, c, tab, m, d_d, d_p, gn, block_size, (long long)pitch, ctx->stream))) break;
        rc = scatter_rows_kind(*ctx, par + g0 * m, kp, (size_t)gn * m, block_size, pitch, d_p, ctx->h_stage + dbytes,
                               nullptr, *pool);
    }
    if (rc) {
        (void)hipStreamSynchronize(ctx->stream);
        fprintf(stderr, "[qfec] reed_solomon_encode: %s\n", qfec_last_error());
    }
    staged_report("reed_solomon_encode (staged)", ndev, nptr);
    return rc;
}

int reed_solomon_reconstruct(reed_solomon* rs, unsigned char** shards, unsigned char* marks, int nr_shards,
                             int block_size) {
    if (!rs || !shards || !marks) return 0;
    rs_handle* h = (rs_handle*)rs;
    const int k = rs->data_shards, m = rs->parity_shards, n = rs->shards;
    const long long G = nr_shards / n;
    if (G <= 0 || block_size <= 0) return 0;
    t_rs_entry = std::chrono::steady_clock::now();
    sync_rows(h);
    qfec_code* c = h->code;
    const bool dev_marks = is_device_ptr(marks);
    std::vector<uint8_t> hmarks;
    const uint8_t* mk = marks;
    if (dev_marks) {
        hmarks.resize((size_t)G * n);
        if (hipMemcpy(hmarks.data(), marks, hmarks.size(), hipMemcpyDeviceToHost) != hipSuccess) {
            fprintf(stderr, "[qfec] reed_solomon_reconstruct: cannot read device marks\n");
            return QFEC_EHIP;
        }
        mk = hmarks.data();
    }
    unsigned char** data = shards;
    unsigned char** par = shards + G * k;
    DevCtx* ctx = nullptr;
    long long nfail_all = 0;
    int rc = QFEC_OK;
    bool any = false;
    for (size_t i = 0; i < (size_t)G * k && !any; ++i) any = mk[i] != 0;
    if (!any) return 0;  // nothing erased: nothing to do (rs.c:618-620)
    if ((rc = current_ctx(&ctx))) {
        fprintf(stderr, "[qfec] reed_solomon_reconstruct: %s\n", qfec_last_error());
        return rc;
    }
    const auto tc = std::chrono::steady_clock::now();
    std::shared_ptr<HostPool> pool = host_pool();
    std::vector<uint8_t> kind((size_t)G * n);
    const size_t ndev_all = classify_ptrs(shards, (size_t)G * n, *pool, kind.data());
    const bool all_host = ndev_all == 0;
    t_rs_classify = RsTrace::since(tc);
    // all shards in host memory and a pattern LUT in reach: the pipelined host path
    if (n <= QFEC_LUT_MAX_N && all_host) {
        DevTables* d = nullptr;
        std::shared_ptr<const std::vector<uint8_t>> seed;  // a reference, not a copy of the 2^n flags
        {
            std::lock_guard<std::mutex> lk(c->mu);
            rc = ensure_lut(c, ctx->device, &d);
            if (!rc) seed = c->lut_seed;
        }
        if (!rc) rc = rs_reconstruct_pipe(*ctx, c, seed->data(), data, par, mk, G, block_size, &nfail_all);
        if (rc) {
            fprintf(stderr, "[qfec] reed_solomon_reconstruct: %s\n", qfec_last_error());
            return rc;
        }
        return nfail_all ? -1 : 0;
    }
    // device or mixed pointers (or n > 24): chunks of ~kChunkBytes of staged shards, each with its
    // own decode records (built from that chunk's marks), so staging stays bounded whatever the
    // batch size; host rows through the pinned stage, device rows one copy each; groups left
    // under-determined -> -1 (rs.c:631-634), counted on the host by the kernel's rule
    const size_t pitch = round_up((size_t)block_size, 16);
    const long long per = tuning().host_chunk > 0 ? (long long)tuning().host_chunk  // knob: tests force several chunks
                                                  : std::max<long long>(1, (long long)(kChunkBytes / ((size_t)n * pitch)));
    std::vector<uint8_t> cmarks, only;
    std::vector<int32_t> grec;
    std::vector<uint32_t> recs;
    for (long long g0 = 0; g0 < G && !rc; g0 += per) {
        const long long gn = std::min(per, G - g0);
        cmarks.resize((size_t)gn * n);  // this chunk's marks in the rs.c layout
        memcpy(cmarks.data(), mk + (size_t)g0 * k, (size_t)gn * k);
        memcpy(cmarks.data() + (size_t)gn * k, mk + (size_t)G * k + (size_t)g0 * m, (size_t)gn * m);
        long long nfail = 0;
        {
            std::lock_guard<std::mutex> lk(c->mu);
            host_records(c, cmarks.data(), gn, grec, recs, &nfail);
        }
        nfail_all += nfail;
        if (recs.empty()) continue;  // nothing to recover in this chunk
        if (!ctx && (rc = current_ctx(&ctx))) break;
        only.resize((size_t)gn * k);
        for (size_t i = 0; i < only.size(); ++i) only[i] = cmarks[i] ? 1 : 0;
        std::lock_guard<std::mutex> lk(ctx->mu);
        // staged chunk: data | parity | group records | record words
        const size_t dbytes = (size_t)gn * k * pitch, pbytes = (size_t)gn * m * pitch;
        const size_t gbytes = round_up((size_t)gn * 4, 16), rbytes = round_up(recs.size() * 4, 16);
        const size_t tot = dbytes + pbytes + gbytes + rbytes;
        if ((rc = ensure_stage(*ctx, tot, tot))) break;
        uint8_t* d_d = ctx->d_stage;
        uint8_t* d_p = d_d + dbytes;
        int32_t* d_g = (int32_t*)(d_p + pbytes);
        uint32_t* d_r = (uint32_t*)((uint8_t*)d_g + gbytes);
        uint8_t* hs = ctx->h_stage;
        memcpy(hs + dbytes + pbytes, grec.data(), (size_t)gn * 4);
        memcpy(hs + dbytes + pbytes + gbytes, recs.data(), recs.size() * 4);
        const uint8_t* kd = kind.data() + g0 * k;
        const uint8_t* kp = kind.data() + (size_t)G * k + g0 * m;
        rc = gather_rows_kind(*ctx, data + g0 * k, kd, (size_t)gn * k, block_size, pitch, d_d, hs, *pool);
        if (!rc) rc = gather_rows_kind(*ctx, par + g0 * m, kp, (size_t)gn * m, block_size, pitch, d_p, hs + dbytes, *pool);
        if (!rc && hipMemcpyAsync(d_g, hs + dbytes + pbytes, gbytes + rbytes, hipMemcpyHostToDevice, ctx->stream) !=
                       hipSuccess)
            rc = hip_fail(hipGetLastError(), "reed_solomon_reconstruct: H2D");
        if (!rc) rc = run_reconstruct(*ctx, c, nullptr, d_g, d_r, d_d, d_p, nullptr, gn, block_size, (long long)pitch,
                                      nullptr, ctx->stream);
        if (!rc) rc = scatter_rows_kind(*ctx, data + g0 * k, kd, (size_t)gn * k, block_size, pitch, d_d, hs, only.data(),
                                        *pool);
        if (rc) (void)hipStreamSynchronize(ctx->stream);  // nothing left in flight into the staging
    }
    staged_report("reed_solomon_reconstruct (staged)", ndev_all, (size_t)G * n);
    if (rc) {
        fprintf(stderr, "[qfec] reed_solomon_reconstruct: %s\n", qfec_last_error());
        return rc;
    }
    return nfail_all ? -1 : 0;
}

}  // extern "C"

