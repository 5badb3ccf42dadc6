// qfec_runtime.cpp -- host runtime core of libqfec.so: device contexts, code objects, the batched
// device API (include/qfec.h, qfec_*), knobs and calibration probes.
//
// libqfec.so exports three ABIs (declared in include/):
//   qfec_fec.h  fec_new / fec_free / fec_encode / fec_decode      (system/fec.h:237-241; qfec_fec_abi.cpp)
//   qfec_rs.h   reed_solomon_init / new / release / encode /
//               reconstruct / error                                (module/rs.h:22-49; qfec_rs_abi.cpp)
//   qfec.h      the batched device API (qfec_*) both of the above are built on (here, qfec_pipe.cpp,
//               qfec_wire_api.cpp).  Shared internals: qfec_rt.hpp.
//
// Every GF multiply-accumulate runs in the HIP kernels of qfec_kernels.hip.  The host
// does what the reference's host code does outside its byte loops: build the parity
// matrices, shuffle packets, pick survivors, invert k x k matrices (cached per erasure
// pattern), and move bytes between the caller's buffers and the device.  There is no CPU
// arithmetic fallback: without a usable HIP device every entry point fails loudly.
//
// Threading: all entry points are thread-safe.  A device context (internal stream, pinned
// and device staging buffers) is created lazily and exactly once per device; codes keep
// their device tables per device.  No HIP state is visible to callers.
#include "qfec_rt.hpp"

#define QFEC_VERSION_STRING "qfec 0.1.0 (gfx950)"

using namespace qfec;

namespace qfec {

std::shared_ptr<HostPool> host_pool() {
    static std::mutex mu;
    static std::shared_ptr<HostPool> pool;
    static int made_with = -1;
    std::lock_guard<std::mutex> lk(mu);
    const int want = tuning().host_threads;
    if (!pool || want != made_with) {
        const int n = want > 0 ? std::min(want, 64) : std::min(usable_cpus(), 32);
        pool = std::make_shared<HostPool>(n);
        made_with = want;
    }
    return pool;
}

}  // namespace qfec

// ====================================================================== errors
namespace qfec {

thread_local std::string t_last_error;

void set_error(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    t_last_error = buf;
}

int hip_fail(hipError_t e, const char* what) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return QFEC_EHIP;
}

std::atomic<int> g_variant{QFEC_VARIANT_PERM};
std::atomic<int> g_percall_fast{1};  // qfec_tune "percall_fast": fec_encode / fec_decode via k_percall
std::atomic<unsigned long long> g_group_hits{0}, g_group_misses{0};  // fec_encode's group cache (all handles)

DevCtx g_ctx[kMaxDevices];
std::once_flag g_ctx_once[kMaxDevices];

int init_ctx(DevCtx& c, int dev) {
    c.device = dev;
    HIP_TRY(hipSetDevice(dev));
    HIP_TRY(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    const Field& f = field();
    HIP_TRY(hipMalloc(&c.d_gf, 768));
    HIP_TRY(hipMemcpy(c.d_gf, f.exp, 512, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c.d_gf + 512, f.log, 256, hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&c.d_counter, 256));
    std::vector<uint32_t> t256(256 * QFEC_TAB_STRIDE);
    for (int v = 0; v < 256; ++v) perm_entry((uint8_t)v, &t256[(size_t)v * QFEC_TAB_STRIDE]);
    HIP_TRY(hipMalloc(&c.d_t256, t256.size() * 4));
    HIP_TRY(hipMemcpy(c.d_t256, t256.data(), t256.size() * 4, hipMemcpyHostToDevice));
    return QFEC_OK;
}

// context of the calling thread's current device (created on first use)
int current_ctx(DevCtx** out) {
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) {
        set_error("no HIP device available (%s)", e == hipSuccess ? "0 devices" : hipGetErrorString(e));
        return QFEC_ENODEV;
    }
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDevices) {
        set_error("device %d out of range", dev);
        return QFEC_ENODEV;
    }
    DevCtx& c = g_ctx[dev];
    std::call_once(g_ctx_once[dev], [&] {
        int prev = 0;
        (void)hipGetDevice(&prev);
        c.init_rc = init_ctx(c, dev);
        (void)hipSetDevice(prev);
    });
    if (c.init_rc != QFEC_OK) {
        if (t_last_error.empty()) set_error("device %d context initialisation failed", dev);
        return c.init_rc;
    }
    *out = &c;
    return QFEC_OK;
}

int ensure_stage(DevCtx& c, size_t dbytes, size_t hbytes) {
    if (dbytes > c.d_cap) {
        if (c.d_stage) HIP_TRY(hipFree(c.d_stage));
        c.d_stage = nullptr;
        c.d_cap = 0;
        const size_t cap = round_up(std::max(dbytes, (size_t)1 << 20), 1 << 20);
        HIP_TRY(hipMalloc(&c.d_stage, cap));
        c.d_cap = cap;
    }
    if (hbytes > c.h_cap) {
        if (c.h_stage) HIP_TRY(hipHostFree(c.h_stage));
        c.h_stage = nullptr;
        c.h_cap = 0;
        const size_t cap = round_up(std::max(hbytes, (size_t)1 << 20), 1 << 20);
        HIP_TRY(hipHostMalloc(&c.h_stage, cap, hipHostMallocDefault));
        c.h_cap = cap;
    }
    return QFEC_OK;
}

int ensure_pc(DevCtx& c, size_t bytes) {
    if (!c.h_pc_done) {
        HIP_TRY(hipHostMalloc((void**)&c.h_pc_done, 256, hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(hipHostGetDevicePointer((void**)&c.d_pc_done, c.h_pc_done, 0));
        __atomic_store_n(c.h_pc_done, 0u, __ATOMIC_RELEASE);
    }
    if (bytes <= c.pc_cap) return QFEC_OK;
    if (c.h_pc) HIP_TRY(hipStreamSynchronize(c.stream));  // no launch may still use the old block
    if (c.h_pc) HIP_TRY(hipHostFree(c.h_pc));
    c.h_pc = c.d_pc = nullptr;
    c.pc_cap = 0;
    const size_t cap = round_up(std::max(bytes, (size_t)1 << 16), 1 << 16);
    HIP_TRY(hipHostMalloc(&c.h_pc, cap, hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer((void**)&c.d_pc, c.h_pc, 0));
    c.pc_cap = cap;
    return QFEC_OK;
}

int ensure_small(DevCtx& c, size_t words) {
    if (words <= c.small_cap) return QFEC_OK;
    if (c.d_small) HIP_TRY(hipFree(c.d_small));
    if (c.h_small) HIP_TRY(hipHostFree(c.h_small));
    c.d_small = nullptr;
    c.h_small = nullptr;
    c.small_cap = 0;
    const size_t cap = round_up(words, 4096);
    HIP_TRY(hipMalloc(&c.d_small, cap * 4));
    HIP_TRY(hipHostMalloc(&c.h_small, cap * 4, hipHostMallocDefault));
    c.small_cap = cap;
    return QFEC_OK;
}

// true if p is device (or managed) memory visible to the current device
// Plain (malloc'd, unregistered) host pointers this thread has probed, a small direct-mapped
// cache: the per-packet ABIs probe every packet pointer, and a probe costs a runtime lookup
// (tools/ptr_probe.cpp).  What the cache relies on: hipMalloc'd device memory comes from the GPU
// virtual-address apertures the runtime reserves, so a freed malloc block's address does not
// become device memory later.  The runtime does not promise that for every kind: an HMM-backed
// hipMallocManaged allocation is ordinary mmap'd memory and may reuse such an address, and then
// stays "host" here.  The bytes are still right (the CPU reaches managed memory; the copies go
// through the CPU), only the path is the host one.  Registering or pinning a block later leaves
// it host memory.
bool is_device_ptr(const void* p) {
    if (!p) return false;
    thread_local const void* plain[64] = {};
    const uintptr_t u = (uintptr_t)p;
    const void*& slot = plain[((u >> 4) ^ (u >> 10) ^ (u >> 16)) & 63u];
    if (slot == p) return false;
    hipPointerAttribute_t attr;
    hipError_t e = hipPointerGetAttributes(&attr, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // clear the sticky error of the probe
        slot = p;
        return false;
    }
    if (attr.type == hipMemoryTypeUnregistered) slot = p;
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

// host memory the DMA engines can read directly (hipHostMalloc'd or hipHostRegister'ed)
bool is_pinned_host(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t attr;
    hipError_t e = hipPointerGetAttributes(&attr, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

// the current device's address of pinned host memory (hipHostMalloc'd, or registered mapped):
// the kernels then read and write it directly over PCIe, with no staging copies ("zero copy")
bool host_dev(const void* h, uint8_t** d) {
    void* p = nullptr;
    if (!h || hipHostGetDevicePointer(&p, const_cast<void*>(h), 0) != hipSuccess || !p) {
        (void)hipGetLastError();
        return false;
    }
    *d = static_cast<uint8_t*>(p);
    return true;
}

int ensure_host_slot(DevCtx::HostSlot& h, size_t in_bytes, size_t out_bytes) {
    if (!h.stream) {
        HIP_TRY(hipStreamCreateWithFlags(&h.stream, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&h.done, hipEventDisableTiming));
    }
    if (in_bytes > h.in_cap || out_bytes > h.out_cap) {
        if (h.d_buf) HIP_TRY(hipFree(h.d_buf));
        if (h.h_in) HIP_TRY(hipHostFree(h.h_in));
        if (h.h_out) HIP_TRY(hipHostFree(h.h_out));
        h.d_buf = h.h_in = h.h_out = nullptr;
        h.in_cap = h.out_cap = 0;
        HIP_TRY(hipMalloc(&h.d_buf, in_bytes + out_bytes));
        HIP_TRY(hipHostMalloc(&h.h_in, in_bytes, hipHostMallocDefault));
        HIP_TRY(hipHostMalloc(&h.h_out, out_bytes, hipHostMallocDefault));
        h.in_cap = in_bytes;
        h.out_cap = out_bytes;
    }
    return QFEC_OK;
}

// after an error in the host-buffer pipelines: wait for whatever the slots still have in
// flight, so no DMA writes into caller memory after the call has returned
void quiesce_host_slots(DevCtx& c) {
    for (auto& h : c.host)
        if (h.stream) (void)hipStreamSynchronize(h.stream);
    (void)hipGetLastError();
}

// gather `count` rows of `len` bytes from ptrs[] into device rows of `pitch` at dst (device).
// dev_src: one copy per row, whatever memory each row is in (device, managed or host rows mixed:
// hipMemcpyDefault); else the rows are host memory, gathered through the pinned stage at h_tmp.
int gather_rows(DevCtx& c, unsigned char* const* ptrs, size_t count, int len, size_t pitch, uint8_t* d_dst,
                uint8_t* h_tmp, bool dev_src) {
    if (dev_src) {
        for (size_t i = 0; i < count; ++i)
            HIP_TRY(hipMemcpyAsync(d_dst + i * pitch, ptrs[i], (size_t)len, hipMemcpyDefault, c.stream));
        return QFEC_OK;
    }
    for (size_t i = 0; i < count; ++i) memcpy(h_tmp + i * pitch, ptrs[i], (size_t)len);
    HIP_TRY(hipMemcpyAsync(d_dst, h_tmp, count * pitch, hipMemcpyHostToDevice, c.stream));
    return QFEC_OK;
}

int scatter_rows(DevCtx& c, unsigned char* const* ptrs, size_t count, int len, size_t pitch, const uint8_t* d_src,
                 uint8_t* h_tmp, bool dev_dst, const uint8_t* only /* nullable: rows to write */) {
    if (dev_dst) {
        for (size_t i = 0; i < count; ++i)
            if (!only || only[i])
                HIP_TRY(hipMemcpyAsync(ptrs[i], d_src + i * pitch, (size_t)len, hipMemcpyDefault, c.stream));
        HIP_TRY(hipStreamSynchronize(c.stream));
        return QFEC_OK;
    }
    HIP_TRY(hipMemcpyAsync(h_tmp, d_src, count * pitch, hipMemcpyDeviceToHost, c.stream));
    HIP_TRY(hipStreamSynchronize(c.stream));
    for (size_t i = 0; i < count; ++i)
        if (!only || only[i]) memcpy(ptrs[i], h_tmp + i * pitch, (size_t)len);
    return QFEC_OK;
}

}  // namespace qfec


namespace qfec {

qfec_code* make_code(int k, int m, std::vector<uint8_t>&& rows, int quirk) {
    qfec_code* c = new (std::nothrow) qfec_code();
    if (!c) return nullptr;
    c->k = k;
    c->m = m;
    c->quirk = quirk;
    c->rows = std::move(rows);
    return c;
}

void free_code(qfec_code* c) {
    if (!c) return;
    int prev = 0;
    bool have = hipGetDevice(&prev) == hipSuccess;
    for (auto& kv : c->dev) {
        if (hipSetDevice(kv.first) != hipSuccess) continue;
        if (kv.second.d_enc) (void)hipFree(kv.second.d_enc);
        if (kv.second.d_lut) (void)hipFree(kv.second.d_lut);
        if (kv.second.d_rec) (void)hipFree(kv.second.d_rec);
    }
    if (have) (void)hipSetDevice(prev);
    delete c;
}

// module/rs.c decodes from rs->m (rs.c:505, 536-548); other codes from their parity rows
const uint8_t* full_of(const qfec_code* c) { return c->full.empty() ? nullptr : c->full.data(); }

void enc_table_host(const qfec_code* c, std::vector<uint32_t>& t) {
    const int k = c->k, m = c->m;
    t.assign((size_t)m * k * QFEC_TAB_STRIDE, 0);
    for (int r = 0; r < m; ++r) {
        for (int i = 0; i < k; ++i) perm_entry(c->rows[(size_t)r * k + i], &t[((size_t)r * k + i) * QFEC_TAB_STRIDE]);
        if (c->quirk && c->rows[(size_t)r * k] == 0) t[((size_t)r * k) * QFEC_TAB_STRIDE + 5] = 1;
    }
}

// encode tables of `c` on device `dev` (caller holds c->mu)
int ensure_enc(qfec_code* c, int dev, uint32_t** out) {
    DevTables& d = c->dev[dev];
    if (d.enc_version != c->version || !d.d_enc) {
        std::vector<uint32_t> t;
        enc_table_host(c, t);
        if (d.d_enc) HIP_TRY(hipFree(d.d_enc));
        d.d_enc = nullptr;
        HIP_TRY(hipMalloc(&d.d_enc, std::max<size_t>(t.size(), 8) * 4));
        if (!t.empty()) HIP_TRY(hipMemcpy(d.d_enc, t.data(), t.size() * 4, hipMemcpyHostToDevice));
        d.enc_version = c->version;
    }
    *out = d.d_enc;
    return QFEC_OK;
}

// key of the decode matrix a group-order erasure mask selects: erased data bits and
// the chosen parity bits (first e non-erased, ascending -- module/rs.c:620-629).
// Returns false when under-determined.  e == 0 -> key 0.
bool pattern_key(uint64_t mask, int k, int m, uint64_t* key, int* e_out) {
    const uint64_t dm = k >= 64 ? mask : (mask & ((1ull << k) - 1));
    const int e = __builtin_popcountll(dm);
    *e_out = e;
    if (e == 0) { *key = 0; return true; }
    uint64_t avail = ~(mask >> k) & (m >= 64 ? ~0ull : ((1ull << m) - 1));
    uint64_t chosen = 0;
    for (int i = 0; i < e; ++i) {
        if (!avail) return false;
        const uint64_t low = avail & (~avail + 1);
        chosen |= low;
        avail ^= low;
    }
    *key = dm | (chosen << k);
    return true;
}

int record_for_key(const qfec_code* c, uint64_t key, std::vector<uint32_t>& rec) {
    const int k = c->k, m = c->m, n = k + m;
    std::vector<uint8_t> marks(n, 0);
    for (int i = 0; i < k; ++i) marks[i] = (key >> i) & 1;
    // parity not chosen is treated as erased so decode_rows picks exactly `chosen`
    for (int j = 0; j < m; ++j) marks[k + j] = ((key >> (k + j)) & 1) ? 0 : 1;
    std::vector<uint8_t> rows;
    std::vector<int> surv, lost;
    const int e = decode_rows(c->rows.data(), k, m, marks.data(), rows, surv, lost, full_of(c));
    if (e <= 0) return -1;
    const RecordLayout L = record_layout(k, m);
    rec.assign(L.words(e, k), 0);
    build_record(L, k, e, rows.data(), surv.data(), lost.data(), c->quirk != 0, rec.data());
    return e;
}

// device LUT (2^n entries) + all decode records of `c` (caller holds c->mu)
int ensure_lut(qfec_code* c, int dev, DevTables** out) {
    DevTables& d = c->dev[dev];
    *out = &d;
    if (d.rec_version == c->version && d.d_lut) return QFEC_OK;
    const int k = c->k, m = c->m, n = k + m;
    if (n > QFEC_LUT_MAX_N) {
        set_error("qfec_reconstruct: k + m = %d > %d (use reed_solomon_reconstruct)", n, QFEC_LUT_MAX_N);
        return QFEC_EUNSUP;
    }
    const size_t nmask = (size_t)1 << n;
    std::vector<int32_t> lut(nmask);
    std::vector<uint8_t> seed(nmask, 0);
    std::unordered_map<uint64_t, int32_t> off_of;
    std::vector<uint32_t> recs, one;
    for (size_t mask = 0; mask < nmask; ++mask) {
        uint64_t key;
        int e;
        if (!pattern_key(mask, k, m, &key, &e)) { lut[mask] = QFEC_REC_FAIL; continue; }
        if (e == 0) { lut[mask] = QFEC_REC_NONE; continue; }
        auto it = off_of.find(key);
        if (it != off_of.end()) {
            lut[mask] = it->second;
            seed[mask] = recs[(size_t)it->second + 1] != 0;
            continue;
        }
        if (record_for_key(c, key, one) <= 0) { lut[mask] = QFEC_REC_FAIL; continue; }
        one.resize(record_layout(k, m).words(m, k), 0);  // pad to m rows (branch-free kernel)
        seed[mask] = one[1] != 0;  // record word 1: the rows the rs.c quirk seeds from the output
        const int32_t off = (int32_t)recs.size();
        recs.insert(recs.end(), one.begin(), one.end());
        off_of.emplace(key, off);
        lut[mask] = off;
    }
    if (d.d_lut) HIP_TRY(hipFree(d.d_lut));
    if (d.d_rec) HIP_TRY(hipFree(d.d_rec));
    d.d_lut = nullptr;
    d.d_rec = nullptr;
    HIP_TRY(hipMalloc(&d.d_lut, nmask * 4));
    HIP_TRY(hipMalloc(&d.d_rec, std::max<size_t>(recs.size(), 8) * 4));
    HIP_TRY(hipMemcpy(d.d_lut, lut.data(), nmask * 4, hipMemcpyHostToDevice));
    if (!recs.empty()) HIP_TRY(hipMemcpy(d.d_rec, recs.data(), recs.size() * 4, hipMemcpyHostToDevice));
    d.rec_version = c->version;
    c->lut_seed = std::make_shared<const std::vector<uint8_t>>(std::move(seed));
    c->lut_seed_version = c->version;
    return QFEC_OK;
}

bool vec16_ok(const void* a, const void* b, int block, long long pitch) {
    return ((uintptr_t)a % 16 == 0) && ((uintptr_t)b % 16 == 0) && (pitch % 16 == 0) &&
           (long long)round_up((size_t)block, 16) <= pitch;
}

// launch encode over `groups` groups with tables `tab` covering `m` rows
int run_encode(DevCtx& ctx, const qfec_code* c, const uint32_t* tab, int m, const uint8_t* d_data,
               uint8_t* d_par, long long groups, int block, long long pitch, hipStream_t s, long long dgs,
               long long pgs, bool host_mem) {
    EncodeArgs a{};
    a.tab = tab;
    a.gf_exp = ctx.d_gf;
    a.gf_log = ctx.d_gf + 512;
    a.k = c->k;
    a.m = m;
    a.pitch = (uint64_t)pitch;
    a.vec16 = vec16_ok(d_data, d_par, block, pitch) ? 1 : 0;
    a.impl = tuning().encode_impl;
    // a cap on resident waves (and the one-wave blocks held to 10 per CU) pays in HBM
    // (qfec_kernels.hip launch_encode), not over PCIe, where latency wants every wave the registers allow
    a.lds = host_mem ? 0 : tuning().encode_lds.load();
    a.block = host_mem ? 256 : tuning().encode_block.load();
    a.cols = a.vec16 ? (uint32_t)((block + 15) / 16) : (uint32_t)block;
    a.cols_div = make_div_magic(a.cols);
    a.dgs = dgs >= 0 ? (uint64_t)dgs : (uint64_t)c->k * pitch;
    a.pgs = pgs >= 0 ? (uint64_t)pgs : (uint64_t)m * pitch;
    if (a.vec16 && ((a.dgs | a.pgs) & 15)) {
        a.vec16 = 0;
        a.cols = (uint32_t)block;
        a.cols_div = make_div_magic(a.cols);
    }
    const long long per = std::max<long long>(1, (long long)(0x7FFFFFFFll / a.cols));
    for (long long g0 = 0; g0 < groups; g0 += per) {
        const long long gn = std::min(per, groups - g0);
        a.data = d_data + (size_t)g0 * a.dgs;
        a.parity = d_par + (size_t)g0 * a.pgs;
        a.work = (uint64_t)gn * a.cols;
        hipError_t e = launch_encode(a, g_variant.load(), s);
        if (e != hipSuccess) return hip_fail(e, "encode kernel launch");
    }
    return QFEC_OK;
}

int run_reconstruct(DevCtx& ctx, const qfec_code* c, const int32_t* lut, const int32_t* group_rec,
                    const uint32_t* recs, uint8_t* d_data, const uint8_t* d_par, const uint8_t* d_marks,
                    long long groups, int block, long long pitch, unsigned* d_failed, hipStream_t s,
                    long long dgs, long long pgs) {
    ReconArgs a{};
    const RecordLayout L = record_layout(c->k, c->m);
    a.data = d_data;
    a.parity = d_par;
    a.marks = d_marks;
    a.lut = lut;
    a.group_rec = group_rec;
    a.records = recs;
    a.failed = d_failed;
    a.groups = (uint64_t)groups;
    a.pitch = (uint64_t)pitch;
    a.k = c->k;
    a.m = c->m;
    a.surv_off = L.surv_off;
    a.lost_off = L.lost_off;
    a.hdr = L.hdr;
    a.coff = L.coff;
    a.t256 = ctx.d_t256;
    a.dgs = dgs >= 0 ? (uint64_t)dgs : (uint64_t)c->k * pitch;
    a.pgs = pgs >= 0 ? (uint64_t)pgs : (uint64_t)c->m * pitch;
    a.vec16 = vec16_ok(d_data, d_par, block, pitch) && !((a.dgs | a.pgs) & 15) ? 1 : 0;
    a.cols = a.vec16 ? (uint32_t)((block + 15) / 16) : (uint32_t)block;
    a.impl = tuning().recon_impl;
    a.wpg = (a.cols + 63) / 64;
    a.cols8 = (uint32_t)((block + 7) / 8);
    a.cols12 = (uint32_t)((block + 11) / 12);
    if (a.vec16 && c->k < 14) {
        // cover the 16-B columns' span, which the 16-B body writes anyway (it stays inside
        // the pitch): a row that ends part-way into a 64-B line costs a partial-line write
        // (B = 1400: 175 -> 176 8-B columns, rows end on 1408 = 22 lines).  It also reads the
        // extra 8 B of every survivor, and with k = 16 survivors per row written that costs
        // more than it saves: RS(16,4) B=1400 5 404 GB/s full against 5 508 partial, RS(10,3)
        // B=1024 6 009 against 5 949 (interleaved A/B, profiles/r03_recon/r03k_ab.txt)
        a.cols8 = 2u * a.cols;
        a.cols12 = std::max(a.cols12, a.cols * 16u / 12u);
    }
    a.wpg8 = (a.cols8 + 63) / 64;
    a.wpg12 = (a.cols12 + 63) / 64;
    hipError_t e = launch_reconstruct(a, s);
    if (e != hipSuccess) return hip_fail(e, "reconstruct kernel launch");
    return QFEC_OK;
}

// decode records for groups given host-side marks (rs.c layout); explicit mode
int host_records(qfec_code* c, const uint8_t* marks, long long groups, std::vector<int32_t>& grec,
                 std::vector<uint32_t>& recs, long long* nfail) {
    const int k = c->k, m = c->m;
    if (c->rec_cache_version != c->version) {
        c->rec_cache.clear();
        c->rec_cache_version = c->version;
    }
    std::unordered_map<uint64_t, int32_t> off_of;
    grec.assign((size_t)groups, QFEC_REC_NONE);
    recs.clear();
    *nfail = 0;
    std::vector<uint8_t> gm(k + m);
    for (long long g = 0; g < groups; ++g) {
        // group-order view of this group's marks (module/rs.c:611-639 walk)
        const uint8_t* dm = marks + (size_t)g * k;
        const uint8_t* pm = marks + (size_t)groups * k + (size_t)g * m;
        int e = 0;
        for (int i = 0; i < k; ++i) e += dm[i] ? 1 : 0;
        if (!e) continue;
        // chosen parity: first e non-erased, ascending
        uint64_t kd = 0;
        std::vector<int> chosen;
        for (int j = 0; j < m && (int)chosen.size() < e; ++j)
            if (!pm[j]) chosen.push_back(j);
        if ((int)chosen.size() < e) { grec[g] = QFEC_REC_FAIL; ++*nfail; continue; }
        // key over erased data + chosen parity; k + m may exceed 64 here, so hash the lists
        uint64_t h = 1469598103934665603ull;
        for (int i = 0; i < k; ++i) if (dm[i]) { h = (h ^ (uint64_t)i) * 1099511628211ull; }
        h = (h ^ 0xFFFFu) * 1099511628211ull;
        for (int j : chosen) h = (h ^ (uint64_t)j) * 1099511628211ull;
        kd = h;
        auto it = off_of.find(kd);
        if (it != off_of.end()) { grec[g] = it->second; continue; }
        auto ct = c->rec_cache.find(kd);
        if (ct == c->rec_cache.end()) {
            for (int i = 0; i < k; ++i) gm[i] = dm[i];
            for (int j = 0; j < m; ++j) gm[k + j] = 1;
            for (int j : chosen) gm[k + j] = 0;
            std::vector<uint8_t> rows;
            std::vector<int> surv, lost;
            const int ee = decode_rows(c->rows.data(), k, m, gm.data(), rows, surv, lost, full_of(c));
            if (ee <= 0) { grec[g] = QFEC_REC_FAIL; ++*nfail; continue; }
            const RecordLayout L = record_layout(k, m);
            std::vector<uint32_t> one(L.words(ee, k));
            build_record(L, k, ee, rows.data(), surv.data(), lost.data(), c->quirk != 0, one.data());
            ct = c->rec_cache.emplace(kd, std::move(one)).first;
        }
        const int32_t off = (int32_t)recs.size();
        recs.insert(recs.end(), ct->second.begin(), ct->second.end());
        off_of.emplace(kd, off);
        grec[g] = off;
    }
    return QFEC_OK;
}

// qfec_reconstruct for k + m above the LUT's reach (2^n entries): the group's n marks are
// read back (n bytes per group, after the caller's stream has produced them), the decode
// records are built per distinct pattern on the host (cached per code), and the explicit-
// record kernel runs on the caller's stream.  Synchronous: returns after the kernel.
int reconstruct_host_records(DevCtx& ctx, qfec_code* c, uint8_t* d_data, const uint8_t* d_par,
                             const uint8_t* d_marks, long long groups, int block_size, long long pitch,
                             unsigned* d_failed, hipStream_t s) {
    const int n = c->k + c->m;
    std::vector<uint8_t> hm((size_t)groups * n);
    HIP_TRY(hipMemcpyAsync(hm.data(), d_marks, hm.size(), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<int32_t> grec;
    std::vector<uint32_t> recs;
    long long nfail = 0;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        int rc = host_records(c, hm.data(), groups, grec, recs, &nfail);
        if (rc) return rc;
    }
    if (recs.empty() && (!nfail || !d_failed)) return QFEC_OK;  // nothing to recover or count
    recs.resize(std::max<size_t>(recs.size(), 8), 0);
    std::lock_guard<std::mutex> lk(ctx.mu);  // d_small is the context's: held until the kernel is done
    const size_t gw = round_up((size_t)groups, 4);
    int rc = ensure_small(ctx, gw + recs.size());
    if (rc) return rc;
    memcpy(ctx.h_small, grec.data(), (size_t)groups * 4);
    memcpy(ctx.h_small + gw, recs.data(), recs.size() * 4);
    HIP_TRY(hipMemcpyAsync(ctx.d_small, ctx.h_small, (gw + recs.size()) * 4, hipMemcpyHostToDevice, s));
    rc = run_reconstruct(ctx, c, nullptr, (const int32_t*)ctx.d_small, ctx.d_small + gw, d_data, d_par, nullptr,
                         groups, block_size, pitch, d_failed, s);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    return QFEC_OK;
}

}  // namespace qfec


// ====================================================================== batched device API
extern "C" {

const char* qfec_version(void) { return QFEC_VERSION_STRING; }

const char* qfec_last_error(void) { return t_last_error.c_str(); }

const char* qfec_strerror(int err) {
    switch (err) {
        case QFEC_OK: return "ok";
        case QFEC_EINVAL: return "invalid argument";
        case QFEC_ENODEV: return "no HIP device";
        case QFEC_EHIP: return "HIP runtime error";
        case QFEC_ENOMEM: return "out of memory";
        case QFEC_EUNSUP: return "unsupported shape for this entry point";
        default: return "unknown error";
    }
}

int qfec_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int qfec_set_kernel_variant(int v) {
    if (v != QFEC_VARIANT_PERM && v != QFEC_VARIANT_LDSLOG) return QFEC_EINVAL;
    g_variant.store(v);
    return QFEC_OK;
}

int qfec_get_kernel_variant(void) { return g_variant.load(); }

}  // extern "C"

// knobs: integration settings and A/B switches (include/qfec.h); every one an atomic int
namespace {
struct Knob {
    const char* key;
    std::atomic<int>* v;
    int lo, hi;
};
const std::vector<Knob>& knob_table() {
    static const std::vector<Knob> t = {
        {"recon_impl", &tuning().recon_impl, -1, 8},
        {"host_chunk", &tuning().host_chunk, 0, 0x7FFFFFFF},
        {"host_threads", &tuning().host_threads, 0, 64},
        {"encode_impl", &tuning().encode_impl, -1, 2},
        {"wire_fused", &tuning().wire_fused, 0, 1},
        {"wire_rx", &tuning().wire_rx, 0, 5},
        {"host_zero_copy", &tuning().host_zero_copy, 0, 1},
        {"host_lanes", &tuning().host_lanes, 2, 8},
        {"host_nt", &tuning().host_nt, 0, 2},
        {"percall_fast", &g_percall_fast, 0, 1},
        {"percall_group", &g_percall_group, 0, 1},
        {"percall_fault", &g_percall_fault, 0, 2},
        {"percall_timeout_us", &g_percall_timeout_us, 0, 0x7FFFFFFF},
        {"percall_stop_us", &g_percall_stop_us, 0, 0x7FFFFFFF},
        {"percall_idle_us", &g_percall_idle_us, 0, 1000000},
        {"percall_resident", &g_percall_resident, 0, 1},
        {"encode_lds", &tuning().encode_lds, -1, 163840},
        {"encode_block", &tuning().encode_block, -1, 256},
    };
    return t;
}

// percall_resident set to 1: a device whose server was abandoned (pc_server_abandon) sets up a new
// one at its next call (new buffers; the old ones stay with the abandoned block)
void retry_abandoned_servers() {
    for (DevCtx& c : g_ctx) {
        std::lock_guard<std::mutex> lk(c.mu);
        if (c.srv.usable == -2) c.srv.usable = 0;
    }
}

// a running per-call server keeps the settings it was launched with: stop it, the next call
// launches one with the new ones
void stop_percall_servers() {
    for (DevCtx& c : g_ctx) {
        std::lock_guard<std::mutex> lk(c.mu);
        if (c.srv.usable <= 0 || !c.srv.launched) continue;
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(c.device);
        (void)pc_server_stop(c);
        (void)hipSetDevice(prev);
    }
}
}  // namespace

extern "C" {

int qfec_tune(const char* key, int value) {
    if (!key) return QFEC_EINVAL;
    for (const Knob& kn : knob_table()) {
        if (strcmp(key, kn.key)) continue;
        if (value < kn.lo || value > kn.hi) break;
        if (!strcmp(key, "recon_impl") && value != -1 && value != 2 && value != 3 && value != 4 && value != 8) break;
        if (!strcmp(key, "encode_block") && value != -1 && value != 64 && value != 256) break;
        if (!strcmp(key, "encode_impl") && value == 1) break;
        kn.v->store(value);
        if (!strcmp(key, "percall_idle_us") || (!strcmp(key, "percall_resident") && !value)) stop_percall_servers();
        if (!strcmp(key, "percall_resident") && value) retry_abandoned_servers();
        return QFEC_OK;
    }
    set_error("qfec_tune: unknown key/value %s=%d", key, value);
    return QFEC_EINVAL;
}

int qfec_tune_get(const char* key, int* value) {
    if (!key || !value) return QFEC_EINVAL;
    for (const Knob& kn : knob_table())
        if (!strcmp(key, kn.key)) {
            *value = kn.v->load();
            return QFEC_OK;
        }
    set_error("qfec_tune_get: unknown key %s", key);
    return QFEC_EINVAL;
}

int qfec_percall_stats(unsigned long long out[5]) {
    if (!out) return QFEC_EINVAL;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    const DevCtx::PcServer& s = ctx->srv;
    out[0] = s.calls;
    out[1] = s.launches;
    out[2] = s.relaunches;
    out[3] = s.usable > 0 && pc_server_alive(s);
    out[4] = (unsigned long long)(long long)s.usable;
    return QFEC_OK;
}


int qfec_percall_counters(unsigned long long* out, int n) {
    if (!out || n < 0) return QFEC_EINVAL;
    unsigned long long v[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        const DevCtx::PcServer& s = ctx->srv;
        v[0] = s.calls;
        v[1] = s.launches;
        v[2] = s.relaunches;
        v[3] = s.usable > 0 && pc_server_alive(s);
        v[4] = (unsigned long long)(long long)s.usable;
        v[5] = s.timeouts;
        v[9] = s.abandoned;
    }
    v[6] = g_group_hits.load();
    v[7] = g_group_misses.load();
    v[8] = (unsigned long long)g_percall_idle_us.load();
    for (int i = 0; i < n && i < 10; ++i) out[i] = v[i];
    return std::min(n, 10);
}

qfec_code* qfec_code_new(int flavour, int k, int m) {
    std::vector<uint8_t> rows;
    bool ok = false;
    if (flavour == QFEC_CAUCHY) ok = cauchy_rows(k, m, rows);
    else if (flavour == QFEC_VANDERMONDE) ok = vandermonde_rows(k, m, rows);
    if (!ok) {
        set_error("qfec_code_new: invalid flavour/shape (%d, k=%d, m=%d)", flavour, k, m);
        return nullptr;
    }
    return make_code(k, m, std::move(rows), flavour == QFEC_CAUCHY ? 1 : 0);
}

qfec_code* qfec_code_from_rows(int k, int m, const unsigned char* parity_rows, int rs_stale_quirk) {
    if (k <= 0 || m < 0 || k > 256 || k + m > 256 || (m > 0 && !parity_rows)) {
        set_error("qfec_code_from_rows: bad shape k=%d m=%d", k, m);
        return nullptr;
    }
    std::vector<uint8_t> rows(parity_rows, parity_rows + (size_t)m * k);
    return make_code(k, m, std::move(rows), rs_stale_quirk ? 1 : 0);
}

void qfec_code_free(qfec_code* code) { free_code(code); }

int qfec_code_rows(const qfec_code* code, unsigned char* out) {
    if (!code || !out) return QFEC_EINVAL;
    memcpy(out, code->rows.data(), code->rows.size());
    return QFEC_OK;
}

int qfec_code_shape(const qfec_code* code, int* k, int* m) {
    if (!code) return QFEC_EINVAL;
    if (k) *k = code->k;
    if (m) *m = code->m;
    return QFEC_OK;
}

int qfec_encode(qfec_code* code, const unsigned char* d_data, unsigned char* d_parity, long long groups,
                int block_size, long long pitch, void* stream) {
    if (!code || groups < 0 || block_size < 1 || pitch < block_size || (groups > 0 && (!d_data || !d_parity))) {
        set_error("qfec_encode: invalid argument");
        return QFEC_EINVAL;
    }
    if (groups == 0 || code->m == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    uint32_t* tab = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_enc(code, ctx->device, &tab);
    }
    if (rc) return rc;
    return run_encode(*ctx, code, tab, code->m, d_data, d_parity, groups, block_size, pitch, (hipStream_t)stream);
}

int qfec_encode_host(qfec_code* code, const unsigned char* h_data, unsigned char* h_parity, long long groups,
                     int block_size, long long pitch) {
    if (!code || groups < 0 || block_size < 1 || pitch < block_size || (groups > 0 && (!h_data || !h_parity))) {
        set_error("qfec_encode_host: invalid argument");
        return QFEC_EINVAL;
    }
    if (groups == 0 || code->m == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    uint32_t* tab = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_enc(code, ctx->device, &tab);
    }
    if (rc) return rc;
    const int k = code->k, m = code->m;
    const size_t in_g = (size_t)k * (size_t)pitch, out_g = (size_t)m * (size_t)pitch;
    // chunk: ~32 MiB of data shards (tuning "host_chunk" = groups per chunk overrides)
    long long gc = tuning().host_chunk > 0 ? (long long)tuning().host_chunk
                                           : std::max<long long>(1, (long long)((size_t)32 << 20) / (long long)in_g);
    gc = std::min(gc, groups);
    const bool pin_in = is_pinned_host(h_data), pin_out = is_pinned_host(h_parity);
    std::lock_guard<std::mutex> lk(ctx->host_mu);
    uint8_t *z_in = nullptr, *z_out = nullptr;
    if (tuning().host_zero_copy && pin_in && pin_out && host_dev(h_data, &z_in) && host_dev(h_parity, &z_out)) {
        // zero copy: one launch reads the data and writes the parity in host memory
        if ((rc = ensure_host_slot(ctx->host[0], 0, 0))) return rc;
        hipStream_t st = ctx->host[0].stream;
        rc = run_encode(*ctx, code, tab, m, z_in, z_out, groups, block_size, pitch, st, -1, -1, true);
        const hipError_t e = hipStreamSynchronize(st);
        if (!rc && e != hipSuccess) rc = hip_fail(e, "qfec_encode_host: zero-copy encode");
        return rc;
    }
    for (int sl = 0; sl < 2; ++sl)
        if ((rc = ensure_host_slot(ctx->host[sl], (size_t)gc * in_g, (size_t)gc * out_g))) return rc;
    long long pending[2] = {-1, -1};  // chunk whose parity sits in the slot's staging
    auto drain = [&](int sl) -> int {
        if (pending[sl] < 0) return QFEC_OK;
        HIP_TRY(hipEventSynchronize(ctx->host[sl].done));
        if (!pin_out) {
            const long long g0 = pending[sl] * gc, gn = std::min(gc, groups - g0);
            memcpy(h_parity + (size_t)g0 * out_g, ctx->host[sl].h_out, (size_t)gn * out_g);
        }
        pending[sl] = -1;
        return QFEC_OK;
    };
    const long long nchunks = (groups + gc - 1) / gc;
    auto chunk = [&](long long i) -> int {
        const int sl = (int)(i & 1);
        DevCtx::HostSlot& h = ctx->host[sl];
        int r = drain(sl);  // the slot's previous chunk: copies done, parity out
        if (r) return r;
        const long long g0 = i * gc, gn = std::min(gc, groups - g0);
        const unsigned char* src = h_data + (size_t)g0 * in_g;
        if (!pin_in) {  // pageable: through pinned staging, overlapping the other slot's work
            memcpy(h.h_in, src, (size_t)gn * in_g);
            src = h.h_in;
        }
        uint8_t* d_in = h.d_buf;
        uint8_t* d_out = h.d_buf + (size_t)gc * in_g;
        HIP_TRY(hipMemcpyAsync(d_in, src, (size_t)gn * in_g, hipMemcpyHostToDevice, h.stream));
        if ((r = run_encode(*ctx, code, tab, m, d_in, d_out, gn, block_size, pitch, h.stream))) return r;
        unsigned char* dst = pin_out ? h_parity + (size_t)g0 * out_g : h.h_out;
        HIP_TRY(hipMemcpyAsync(dst, d_out, (size_t)gn * out_g, hipMemcpyDeviceToHost, h.stream));
        HIP_TRY(hipEventRecord(h.done, h.stream));
        pending[sl] = i;
        return QFEC_OK;
    };
    for (long long i = 0; i < nchunks && !rc; ++i) rc = chunk(i);
    if (!rc) rc = drain((int)(nchunks & 1));  // older slot first
    if (!rc) rc = drain((int)((nchunks + 1) & 1));
    if (rc) quiesce_host_slots(*ctx);  // no copy may still be writing into the caller's buffers
    return rc;
}

int qfec_reconstruct_host(qfec_code* code, unsigned char* h_data, const unsigned char* h_parity,
                          const unsigned char* h_marks, long long groups, int block_size, long long pitch,
                          long long* failed) {
    if (!code || groups < 0 || block_size < 1 || pitch < block_size ||
        (groups > 0 && (!h_data || !h_marks || (code->m > 0 && !h_parity)))) {
        set_error("qfec_reconstruct_host: invalid argument");
        return QFEC_EINVAL;
    }
    if (failed) *failed = 0;
    if (groups == 0) return QFEC_OK;
    const int k = code->k, m = code->m;
    if (k + m > QFEC_LUT_MAX_N) {
        set_error("qfec_reconstruct_host: k + m = %d > %d (use reed_solomon_reconstruct)", k + m, QFEC_LUT_MAX_N);
        return QFEC_EUNSUP;
    }
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    DevTables* d = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_lut(code, ctx->device, &d);
    }
    if (rc) return rc;
    // chunk slot layout, device and pinned alike: data [gc][k][pitch] | parity [gc][m][pitch]
    // | marks [gc*k data marks][gc*m parity marks] | failed counter (8 B)
    const size_t dg = (size_t)k * (size_t)pitch, pg = (size_t)m * (size_t)pitch;
    long long gc = tuning().host_chunk > 0 ? (long long)tuning().host_chunk
                                           : std::max<long long>(1, (long long)((size_t)32 << 20) / (long long)dg);
    gc = std::min(gc, groups);
    const size_t mk_off = (size_t)gc * (dg + pg), cnt_off = round_up(mk_off + (size_t)gc * (k + m), 16);
    const size_t slot_bytes = cnt_off + 16;
    std::lock_guard<std::mutex> lk(ctx->host_mu);
    uint8_t *z_data = nullptr, *z_par = nullptr;
    if (tuning().host_zero_copy && is_pinned_host(h_data) && host_dev(h_data, &z_data) &&
        (m == 0 || (is_pinned_host(h_parity) && host_dev(h_parity, &z_par)))) {
        // zero copy: the kernel reads the survivors and writes the erased data rows in host
        // memory (k + e rows per group over PCIe, not n in and k out); only the marks (one
        // byte per shard) and the failed counter are staged
        DevCtx::HostSlot& h = ctx->host[0];
        const size_t mbytes = (size_t)groups * (k + m), zc_cnt = round_up(mbytes, 16);
        if ((rc = ensure_host_slot(h, zc_cnt + 16, zc_cnt + 16))) return rc;
        memcpy(h.h_in, h_marks, mbytes);
        memset(h.h_in + zc_cnt, 0, 16);
        HIP_TRY(hipMemcpyAsync(h.d_buf, h.h_in, zc_cnt + 16, hipMemcpyHostToDevice, h.stream));
        rc = run_reconstruct(*ctx, code, d->d_lut, nullptr, d->d_rec, z_data, z_par, h.d_buf, groups, block_size, pitch,
                             reinterpret_cast<unsigned*>(h.d_buf + zc_cnt), h.stream);
        if (!rc) {
            const hipError_t e1 = hipMemcpyAsync(h.h_out, h.d_buf + zc_cnt, 16, hipMemcpyDeviceToHost, h.stream);
            if (e1 != hipSuccess) rc = hip_fail(e1, "qfec_reconstruct_host: counter");
        }
        const hipError_t e = hipStreamSynchronize(h.stream);
        if (!rc && e != hipSuccess) rc = hip_fail(e, "qfec_reconstruct_host: zero-copy reconstruct");
        if (!rc && failed) *failed = *reinterpret_cast<const unsigned*>(h.h_out);
        return rc;
    }
    for (int sl = 0; sl < 2; ++sl)
        if ((rc = ensure_host_slot(ctx->host[sl], slot_bytes, slot_bytes))) return rc;
    long long pending[2] = {-1, -1};
    long long nfail = 0;
    auto drain = [&](int sl) -> int {
        if (pending[sl] < 0) return QFEC_OK;
        DevCtx::HostSlot& h = ctx->host[sl];
        HIP_TRY(hipEventSynchronize(h.done));
        const long long g0 = pending[sl] * gc, gn = std::min(gc, groups - g0);
        memcpy(h_data + (size_t)g0 * dg, h.h_out, (size_t)gn * dg);
        nfail += *reinterpret_cast<const unsigned*>(h.h_out + cnt_off);
        pending[sl] = -1;
        return QFEC_OK;
    };
    const long long nchunks = (groups + gc - 1) / gc;
    auto chunk = [&](long long i) -> int {
        const int sl = (int)(i & 1);
        DevCtx::HostSlot& h = ctx->host[sl];
        int r = drain(sl);
        if (r) return r;
        const long long g0 = i * gc, gn = std::min(gc, groups - g0);
        // stage the chunk: data, parity, then its marks in rs.c layout for gn groups
        memcpy(h.h_in, h_data + (size_t)g0 * dg, (size_t)gn * dg);
        if (m) memcpy(h.h_in + (size_t)gn * dg, h_parity + (size_t)g0 * pg, (size_t)gn * pg);
        uint8_t* hm = h.h_in + (size_t)gn * (dg + pg);
        memcpy(hm, h_marks + (size_t)g0 * k, (size_t)gn * k);
        memcpy(hm + (size_t)gn * k, h_marks + (size_t)groups * k + (size_t)g0 * m, (size_t)gn * m);
        memset(h.h_in + cnt_off, 0, 16);
        const size_t used = (size_t)gn * (dg + pg + k + m);
        uint8_t* dd = h.d_buf;
        HIP_TRY(hipMemcpyAsync(dd, h.h_in, used, hipMemcpyHostToDevice, h.stream));
        HIP_TRY(hipMemcpyAsync(dd + cnt_off, h.h_in + cnt_off, 16, hipMemcpyHostToDevice, h.stream));
        if ((r = run_reconstruct(*ctx, code, d->d_lut, nullptr, d->d_rec, dd, dd + (size_t)gn * dg,
                                 dd + (size_t)gn * (dg + pg), gn, block_size, pitch,
                                 reinterpret_cast<unsigned*>(dd + cnt_off), h.stream)))
            return r;
        HIP_TRY(hipMemcpyAsync(h.h_out, dd, (size_t)gn * dg, hipMemcpyDeviceToHost, h.stream));
        HIP_TRY(hipMemcpyAsync(h.h_out + cnt_off, dd + cnt_off, 16, hipMemcpyDeviceToHost, h.stream));
        HIP_TRY(hipEventRecord(h.done, h.stream));
        pending[sl] = i;
        return QFEC_OK;
    };
    for (long long i = 0; i < nchunks && !rc; ++i) rc = chunk(i);
    if (!rc) rc = drain((int)(nchunks & 1));
    if (!rc) rc = drain((int)((nchunks + 1) & 1));
    if (rc) {
        quiesce_host_slots(*ctx);
        return rc;
    }
    if (failed) *failed = nfail;
    return QFEC_OK;
}

int qfec_prepare_reconstruct(qfec_code* code) {
    if (!code) return QFEC_EINVAL;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    DevTables* d = nullptr;
    std::lock_guard<std::mutex> lk(code->mu);
    return ensure_lut(code, ctx->device, &d);
}

int qfec_reconstruct(qfec_code* code, unsigned char* d_data, const unsigned char* d_parity,
                     const unsigned char* d_marks, long long groups, int block_size, long long pitch,
                     unsigned int* d_failed, void* stream) {
    if (!code || groups < 0 || block_size < 1 || pitch < block_size ||
        (groups > 0 && (!d_data || !d_marks || (code->m > 0 && !d_parity)))) {
        set_error("qfec_reconstruct: invalid argument");
        return QFEC_EINVAL;
    }
    if (groups == 0) return QFEC_OK;
    if (groups > 0x7FFFFFFFll * 4) {
        set_error("qfec_reconstruct: too many groups per call");
        return QFEC_EINVAL;
    }
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    if (code->k + code->m > QFEC_LUT_MAX_N) return reconstruct_host_records(*ctx, code, d_data, d_parity, d_marks,
                                                                           groups, block_size, pitch, d_failed,
                                                                           (hipStream_t)stream);
    DevTables* d = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_lut(code, ctx->device, &d);
    }
    if (rc) return rc;
    return run_reconstruct(*ctx, code, d->d_lut, nullptr, d->d_rec, d_data, d_parity, d_marks, groups, block_size,
                           pitch, d_failed, (hipStream_t)stream);
}

int qfec_decode_rows(const qfec_code* code, const unsigned char* marks_n, unsigned char* rows_out,
                     int* survivors_out, int* erased_out) {
    if (!code || !marks_n) return QFEC_EINVAL;
    std::vector<uint8_t> rows;
    std::vector<int> surv, lost;
    const int e = decode_rows(code->rows.data(), code->k, code->m, marks_n, rows, surv, lost, full_of(code));
    if (e > 0) {
        if (rows_out) memcpy(rows_out, rows.data(), rows.size());
        if (survivors_out) memcpy(survivors_out, surv.data(), surv.size() * sizeof(int));
        if (erased_out) memcpy(erased_out, lost.data(), lost.size() * sizeof(int));
    }
    return e;
}

int qfec_synth_fill(unsigned char* d_ptr, long long nbytes, unsigned long long seed, void* stream) {
    if (nbytes < 0 || (nbytes > 0 && !d_ptr)) return QFEC_EINVAL;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    hipError_t e = launch_synth_fill(d_ptr, (uint64_t)nbytes, seed, (hipStream_t)stream);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "synth fill launch");
}

// streaming probe with the encode's traffic shape (XOR only, not a codec): calibration
int qfec_probe_stream(const unsigned char* d_data, unsigned char* d_parity, long long groups, int k, int m,
                      int block_size, long long pitch, void* stream) {
    if (groups <= 0 || k <= 0 || m <= 0 || !vec16_ok(d_data, d_parity, block_size, pitch)) return QFEC_EINVAL;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    EncodeArgs a{};
    a.data = d_data;
    a.parity = d_parity;
    a.k = k;
    a.m = m;
    a.pitch = (uint64_t)pitch;
    a.vec16 = 1;
    a.cols = (uint32_t)((block_size + 15) / 16);
    a.cols_div = make_div_magic(a.cols);
    a.work = (uint64_t)groups * a.cols;
    a.dgs = (uint64_t)k * pitch;
    a.pgs = (uint64_t)m * pitch;
    a.lds = tuning().encode_lds.load();
    a.block = tuning().encode_block.load();
    if (a.work >= 0x80000000ull) return QFEC_EINVAL;
    hipError_t e = launch_probe_xor(a, (hipStream_t)stream);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "probe launch");
}

// the reconstruct's memory skeleton (XOR only, not a codec): calibration of the reconstruct's
// own access pattern, as qfec_probe_stream is of the encode's
int qfec_probe_reconstruct(unsigned char* d_data, const unsigned char* d_parity, const unsigned char* d_marks,
                           long long groups, int k, int m, int block_size, long long pitch, int lds_cap,
                           void* stream) {
    if (groups <= 0 || !d_marks || lds_cap < 0 || lds_cap > 163840 || !vec16_ok(d_data, d_parity, block_size, pitch))
        return QFEC_EINVAL;
    if (!((k == 10 && m == 3) || (k == 16 && m == 4))) return QFEC_EUNSUP;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    ReconArgs a{};
    a.data = d_data;
    a.parity = d_parity;
    a.marks = d_marks;
    a.groups = (uint64_t)groups;
    a.pitch = (uint64_t)pitch;
    a.k = k;
    a.m = m;
    a.dgs = (uint64_t)k * pitch;
    a.pgs = (uint64_t)m * pitch;
    a.cols = (uint32_t)((block_size + 15) / 16);
    a.cols8 = k < 14 ? 2u * a.cols : (uint32_t)((block_size + 7) / 8);  // as run_reconstruct sets them
    a.wpg8 = (a.cols8 + 63) / 64;
    a.rlds = lds_cap;
    hipError_t e = launch_probe_recon(a, (hipStream_t)stream);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "reconstruct probe launch");
}

}  // extern "C"

