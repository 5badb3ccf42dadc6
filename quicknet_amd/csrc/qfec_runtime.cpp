// qfec_runtime.cpp -- host runtime and C ABI of libqfec.so.
//
// Exports three ABIs (declared in include/):
//   qfec_fec.h  fec_new / fec_free / fec_encode / fec_decode      (system/fec.h:237-241)
//   qfec_rs.h   reed_solomon_init / new / release / encode /
//               reconstruct / error                                (module/rs.h:22-49)
//   qfec.h      the batched device API (qfec_*) both of the above are built on.
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
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/qfec.h"
#include "../../include/qfec_fec.h"
#include "../../include/qfec_rs.h"
#include "qfec_internal.hpp"
#include "qfec_maps.hpp"
#include "qfec_percall.hpp"
#include "qfec_pool.hpp"

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
namespace {

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

#define HIP_TRY(expr)                                       \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return hip_fail(_e, #expr);   \
    } while (0)

std::atomic<int> g_variant{QFEC_VARIANT_PERM};
std::atomic<int> g_percall_fast{1};  // qfec_tune "percall_fast": fec_encode / fec_decode via k_percall

inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ====================================================================== device contexts
constexpr int kMaxDevices = 64;

struct DevCtx {
    int device = 0;
    std::mutex mu;  // serialises use of the staging buffers and the internal stream
    hipStream_t stream = nullptr;
    uint8_t* d_stage = nullptr;
    size_t d_cap = 0;
    uint8_t* h_stage = nullptr;  // pinned
    size_t h_cap = 0;
    uint8_t* d_gf = nullptr;     // exp[512] | log[256] for the LDS variant
    uint32_t* d_t256 = nullptr;  // perm tables of all 256 coefficient values (compact reconstruct)
    uint32_t* d_small = nullptr; // per-call tables (fec_encode row, fec_decode matrix)
    size_t small_cap = 0;
    uint32_t* h_small = nullptr; // pinned mirror
    unsigned* d_counter = nullptr;
    // per-packet calls (fec_encode / fec_decode): pinned, device-mapped staging the
    // k_percall kernel reads and writes directly (qfec_percall.hpp)
    uint8_t* h_pc = nullptr;
    uint8_t* d_pc = nullptr;  // the device address of h_pc
    size_t pc_cap = 0;
    uint32_t* h_pc_done = nullptr;  // k_percall's completion word (coherent pinned)
    uint32_t* d_pc_done = nullptr;
    uint32_t pc_seq = 0;
    uint32_t pc_unsynced = 0;       // spin-completed launches since the last stream query
    // the resident per-call server (qfec_percall.hpp): set up on first use
    struct PcServer {
        int usable = 0;              // 0 not tried, 1 ready, -1 unavailable on this device
        hipStream_t stream = nullptr;
        PcBell* bell = nullptr;      // fine-grained device memory the CPU stores into
        uint8_t* in = nullptr;       // ditto: kPcMaxCoef rows of kPcMaxChunks * 16 bytes
        uint8_t* h_out = nullptr;    // coherent pinned host memory, same shape
        uint8_t* d_out = nullptr;
        PcStatus* h_st = nullptr;    // coherent pinned host memory
        PcStatus* d_st = nullptr;
        uint32_t req = 0;            // the last request number stored into the bell word
        uint32_t tab_last[kPcTabWords];  // the tables the bell holds (tab_bytes of them)
        size_t tab_bytes = 0;
        uint32_t gen = 0;            // the last launch's generation
        bool launched = false;
        unsigned long long calls = 0, launches = 0, relaunches = 0, timeouts = 0;
        // QFEC_PERCALL_TRACE sums: loads, compute, fence (shader clocks), host wait (ns), n, clocks and
        // wall ticks over the traced span (the clock calibration)
        unsigned long long tr[7] = {0, 0, 0, 0, 0, 0, 0};
    } srv;
    int init_rc = QFEC_ENODEV;
    // qfec_encode_host: two chunk slots, each with its own stream, event, device buffers
    // and pinned staging (created on first use)
    struct HostSlot {
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
        uint8_t* d_buf = nullptr;  // data chunk | parity chunk
        uint8_t* h_in = nullptr;   // pinned
        uint8_t* h_out = nullptr;  // pinned
        size_t in_cap = 0, out_cap = 0;
    } host[2];
    std::mutex host_mu;
};

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

// ---- the resident per-call server (qfec_percall.hpp)
std::atomic<int> g_percall_resident{1};  // qfec_tune "percall_resident"
std::atomic<int> g_percall_idle_us{(int)kPcIdleUsDefault};  // qfec_tune "percall_idle_us": the block's idle exit
std::atomic<int> g_percall_timeout_us{2000000};  // qfec_tune "percall_timeout_us": give up spinning, wait instead
std::atomic<int> g_percall_fault{0};     // qfec_tune "percall_fault" (tests): 1 = requests are never handed to a server
std::atomic<int> g_percall_group{1};     // qfec_tune "percall_group": fec_encode computes a group's m rows at once
constexpr size_t kPcSrvBytes = (size_t)kPcMaxCoef * kPcMaxChunks * 16;

// true if [p, p + n) lies inside one readable, writable mapping of this process.  Fine-grained
// device memory is mapped for the CPU through the PCIe BAR where the BAR spans all of HBM (as on
// the MI355X); elsewhere its range is reserved without access and a store would fault.
bool cpu_mapped(const void* p, size_t n) {
    FILE* f = fopen("/proc/self/maps", "r");
    if (!f) return false;
    const unsigned long a = (unsigned long)p, b = a + n;
    char line[512];
    bool ok = false;
    while (fgets(line, sizeof line, f)) {
        unsigned long lo = 0, hi = 0;
        char perm[8] = {0};
        if (sscanf(line, "%lx-%lx %7s", &lo, &hi, perm) != 3) continue;
        if (lo <= a && a < hi) {
            ok = b <= hi && perm[0] == 'r' && perm[1] == 'w';
            break;
        }
    }
    fclose(f);
    return ok;
}

void pc_server_stop_all();

// allocate the server's buffers once; on any failure the device keeps the launch-per-call path
int pc_server_setup(DevCtx& c) {
    DevCtx::PcServer& s = c.srv;
    if (s.usable) return s.usable > 0 ? QFEC_OK : QFEC_EHIP;
    s.usable = -1;
    auto release = [&]() {  // nothing stays allocated on a device that keeps the launch-per-call path
        if (s.stream) (void)hipStreamDestroy(s.stream);
        if (s.bell) (void)hipFree(s.bell);
        if (s.in) (void)hipFree(s.in);
        if (s.h_out) (void)hipHostFree(s.h_out);
        if (s.h_st) (void)hipHostFree(s.h_st);
        s.stream = nullptr;
        s.bell = nullptr;
        s.in = s.h_out = s.d_out = nullptr;
        s.h_st = s.d_st = nullptr;
        (void)hipGetLastError();
    };
    auto fail = [&](hipError_t e, const char* what) {
        (void)hipGetLastError();
        fprintf(stderr, "[qfec] per-call server unavailable (%s: %s); launching per call\n", what,
                hipGetErrorString(e));
        release();
        return QFEC_EHIP;
    };
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess) return fail(e, "stream");
    if ((e = hipExtMallocWithFlags((void**)&s.bell, sizeof(PcBell), hipDeviceMallocFinegrained)) != hipSuccess)
        return fail(e, "bell");
    if ((e = hipExtMallocWithFlags((void**)&s.in, kPcSrvBytes, hipDeviceMallocFinegrained)) != hipSuccess)
        return fail(e, "input rows");
    if ((e = hipHostMalloc((void**)&s.h_out, kPcSrvBytes, hipHostMallocMapped | hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&s.d_out, s.h_out, 0)) != hipSuccess)
        return fail(e, "output rows");
    if ((e = hipHostMalloc((void**)&s.h_st, sizeof(PcStatus), hipHostMallocMapped | hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&s.d_st, s.h_st, 0)) != hipSuccess)
        return fail(e, "status word");
    if (!cpu_mapped(s.bell, sizeof(PcBell)) || !cpu_mapped(s.in, kPcSrvBytes)) {
        fprintf(stderr, "[qfec] per-call server unavailable (device memory not CPU-mapped); launching per call\n");
        release();
        return QFEC_EHIP;
    }
    memset(s.bell, 0, sizeof(PcBell));
    memset(s.h_st, 0, sizeof(PcStatus));
    __builtin_ia32_sfence();
    static std::once_flag once;
    std::call_once(once, [] { atexit(pc_server_stop_all); });  // after the runtime's own handlers
    s.usable = 1;
    return QFEC_OK;
}

bool pc_server_alive(const DevCtx::PcServer& s) {
    return s.launched && __atomic_load_n(&s.h_st->state, __ATOMIC_ACQUIRE) != (s.gen << 1);
}

// stop the server and wait for it (a few microseconds: it polls `stop`)
hipError_t pc_server_stop(DevCtx& c) {
    DevCtx::PcServer& s = c.srv;
    if (s.usable <= 0 || !s.launched) return hipSuccess;
    __atomic_store_n(&s.bell->stop, 1u, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    hipError_t e = hipStreamSynchronize(s.stream);
    __atomic_store_n(&s.bell->stop, 0u, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    s.launched = false;
    return e;
}

// pc_server_call's answer when the request was not served: the caller runs it another way
constexpr int kPcNotServed = 1;

// CPU work a per-call path runs while the device serves the request (once, in every path)
struct Overlap {
    void (*fn)(void*) = nullptr;
    void* arg = nullptr;
    bool done = false;
    void run() {
        if (fn && !done) {
            done = true;
            fn(arg);
        }
    }
};

// one call through the server: QFEC_OK, kPcNotServed (the server is stopped and the request is
// still the caller's to serve), or an error (the server then is stopped)
int pc_server_call(DevCtx& c, const std::vector<uint32_t>& tab, int k, int e, unsigned char* const* in,
                   unsigned char* const* out, int sz, size_t pitch, Overlap* ov = nullptr) {
    DevCtx::PcServer& s = c.srv;
    PcBell* b = s.bell;
    uint8_t* rows = s.in;  // fine-grained device memory the CPU stores into (reading the rows from
                           // write-combined host memory instead cost 0.9 us more per call, r03)
    for (int r = 0; r < k; ++r) memcpy(rows + (size_t)r * pitch, in[r], (size_t)sz);
    // the tables go out only when they differ from the last call's (fec_encode of one parity
    // index, or a repeated loss pattern, sends none)
    const size_t tb = (size_t)k * e * 8 * sizeof(uint32_t);
    uint32_t t5[kPcTabWords];
    for (int i = 0; i < k * e; ++i) {
        memcpy(&t5[i * 8], &tab[(size_t)i * QFEC_TAB_STRIDE], 5 * sizeof(uint32_t));
        t5[i * 8 + 5] = t5[i * 8 + 6] = t5[i * 8 + 7] = 0;
    }
    if (tb != s.tab_bytes || memcmp(s.tab_last, t5, tb)) {
        memcpy(b->tab, t5, tb);
        memcpy(s.tab_last, t5, tb);
        s.tab_bytes = tb;
    }
    // the device memory is write-combined for the CPU: the rows and tables must be out of the
    // write-combining buffers before the request word is
    __builtin_ia32_sfence();
    const uint32_t prev = s.req;
    uint32_t req = prev + 1;
    if (req == 0) req = 1;
    s.req = req;
    __atomic_store_n(&b->bell, pc_bell(req, (uint32_t)k, (uint32_t)e, (uint32_t)(pitch / 16)), __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    auto launch = [&]() {
        ++s.gen;
        s.launched = true;
        ++s.launches;
        static const uint32_t trace = getenv("QFEC_PERCALL_TRACE") && atoi(getenv("QFEC_PERCALL_TRACE")) ? 1u : 0u;
        const uint64_t idle = (uint64_t)std::max(0, g_percall_idle_us.load()) * 100u;  // 100 MHz wall clock
        const uint32_t flags = trace;  // bit 0: QFEC_PERCALL_TRACE (qfec_percall.hip)
        return launch_percall_server(b, s.in, s.d_out, s.d_st, prev, s.gen, flags, idle,
                                     s.stream);
    };
    hipError_t he = hipSuccess;
    const bool fault = g_percall_fault.load() != 0;  // test hook: as if no server ever got a CU
    if (fault) (void)pc_server_stop(c);
    else if (!pc_server_alive(s)) he = launch();
    if (ov) ov->run();  // the caller's CPU work, while the request crosses PCIe
    const auto t0 = std::chrono::steady_clock::now();
    const auto limit = std::chrono::microseconds(g_percall_timeout_us.load());
    for (uint32_t it = 1; he == hipSuccess; ++it) {
        if (__atomic_load_n(&s.h_st->done, __ATOMIC_ACQUIRE) == req) {
            ++s.calls;
            if (s.h_st->ts[0]) {  // QFEC_PERCALL_TRACE: sum the device stage times (shader clocks)
                s.tr[0] += s.h_st->ts[1] - s.h_st->ts[0];
                s.tr[1] += s.h_st->ts[2] - s.h_st->ts[1];
                s.tr[2] += s.h_st->ts[3] - s.h_st->ts[2];
                s.tr[5] += s.h_st->ts[3] - s.h_st->ts[0];
                s.tr[6] += s.h_st->rt;
                s.tr[3] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
                ++s.tr[4];
            }
            for (int j = 0; j < e; ++j) memcpy(out[j], s.h_out + (size_t)j * pitch, (size_t)sz);
            return QFEC_OK;
        }
        __builtin_ia32_pause();
        if (!fault && (it & 63) == 0 && __atomic_load_n(&s.h_st->state, __ATOMIC_ACQUIRE) == (s.gen << 1)) {
            // the server went idle and exited just before the request arrived: its exit is
            // published after its last completion, so the request is not served -- relaunch
            if (__atomic_load_n(&s.h_st->done, __ATOMIC_ACQUIRE) == req) continue;
            ++s.relaunches;
            he = launch();
        }
        if ((it & 63) == 0 && std::chrono::steady_clock::now() - t0 > limit) {
            // not served in time: the block may be waiting for a CU that other streams hold.
            // Stop it and wait for it, like the launch path waits for its kernel: once it runs
            // it serves the pending request before it sees `stop`.  A request it never saw is
            // handed back to the caller, which launches it on its own.
            ++s.timeouts;
            const hipError_t se = pc_server_stop(c);
            if (se != hipSuccess) return hip_fail(se, "per-call server: stop after a timeout");
            if (__atomic_load_n(&s.h_st->done, __ATOMIC_ACQUIRE) == req) {
                ++s.calls;
                for (int j = 0; j < e; ++j) memcpy(out[j], s.h_out + (size_t)j * pitch, (size_t)sz);
                return QFEC_OK;
            }
            return kPcNotServed;
        }
    }
    (void)pc_server_stop(c);
    return hip_fail(he, "per-call server launch");
}

void pc_server_stop_all() {
    for (DevCtx& c : g_ctx) {
        if (c.srv.tr[4]) {  // QFEC_PERCALL_TRACE
            const double n = (double)c.srv.tr[4], ghz = c.srv.tr[6] ? c.srv.tr[5] / (c.srv.tr[6] * 10.0) : 2.4;
            fprintf(stderr, "[qfec] per-call server, device %d, %llu traced calls (shader clock %.2f GHz): seen -> "
                    "inputs and tables in %.2f us, compute -> outputs issued %.2f us, system fence %.2f us, host "
                    "request -> completion seen %.2f us\n", c.device, c.srv.tr[4], ghz, c.srv.tr[0] / n / ghz * 1e-3,
                    c.srv.tr[1] / n / ghz * 1e-3, c.srv.tr[2] / n / ghz * 1e-3, c.srv.tr[3] * 1e-3 / n);
        }
        if (c.srv.usable <= 0 || !c.srv.launched) continue;
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(c.device);
        (void)pc_server_stop(c);
        (void)hipSetDevice(prev);
    }
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

}  // namespace

// ====================================================================== code objects
struct DevTables {
    uint32_t* d_enc = nullptr;  // [m][k][8]
    uint64_t enc_version = ~0ull;
    int32_t* d_lut = nullptr;    // [2^n]
    uint32_t* d_rec = nullptr;   // decode records
    uint64_t rec_version = ~0ull;
};

struct qfec_code {
    int k = 0, m = 0;
    int quirk = 0;  // module/rs.c column-0 zero-coefficient behaviour
    std::mutex mu;
    std::vector<uint8_t> rows;  // m x k
    std::vector<uint8_t> full;  // n x k decode matrix of a reed_solomon handle (rs->m), else empty
    uint64_t version = 0;
    std::map<int, DevTables> dev;
    // host-side decode cache: pattern key -> (record words); for explicit mode
    std::unordered_map<uint64_t, std::vector<uint32_t>> rec_cache;
    uint64_t rec_cache_version = ~0ull;
    // per LUT mask: 1 if its record seeds a row from the output's old bytes (the rs.c quirk), so a
    // host-pointer reconstruct must stage the erased rows too (filled with the LUT)
    std::vector<uint8_t> lut_seed;
    uint64_t lut_seed_version = ~0ull;
};

namespace {

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
    c->lut_seed.swap(seed);
    c->lut_seed_version = c->version;
    return QFEC_OK;
}

bool vec16_ok(const void* a, const void* b, int block, long long pitch) {
    return ((uintptr_t)a % 16 == 0) && ((uintptr_t)b % 16 == 0) && (pitch % 16 == 0) &&
           (long long)round_up((size_t)block, 16) <= pitch;
}

// launch encode over `groups` groups with tables `tab` covering `m` rows
int run_encode(DevCtx& ctx, const qfec_code* c, const uint32_t* tab, int m, const uint8_t* d_data,
               uint8_t* d_par, long long groups, int block, long long pitch, hipStream_t s,
               long long dgs = -1, long long pgs = -1, bool host_mem = false) {
    EncodeArgs a{};
    a.tab = tab;
    a.gf_exp = ctx.d_gf;
    a.gf_log = ctx.d_gf + 512;
    a.k = c->k;
    a.m = m;
    a.pitch = (uint64_t)pitch;
    a.vec16 = vec16_ok(d_data, d_par, block, pitch) ? 1 : 0;
    a.impl = tuning().encode_impl;
    // a cap on resident waves pays in HBM (qfec_kernels.hip launch_encode), not over PCIe, where
    // latency wants every wave the registers allow
    a.lds = host_mem ? 0 : tuning().encode_lds.load();
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
                    long long dgs = -1, long long pgs = -1) {
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

}  // namespace

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
        {"percall_fast", &g_percall_fast, 0, 1},
        {"percall_group", &g_percall_group, 0, 1},
        {"percall_fault", &g_percall_fault, 0, 1},
        {"percall_timeout_us", &g_percall_timeout_us, 0, 0x7FFFFFFF},
        {"percall_idle_us", &g_percall_idle_us, 0, 1000000},
        {"percall_resident", &g_percall_resident, 0, 1},
        {"encode_lds", &tuning().encode_lds, -1, 163840},
    };
    return t;
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
        if (!strcmp(key, "encode_impl") && value == 1) break;
        kn.v->store(value);
        if (!strcmp(key, "percall_idle_us") || (!strcmp(key, "percall_resident") && !value)) stop_percall_servers();
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

static std::atomic<unsigned long long> g_group_hits{0}, g_group_misses{0};  // fec_encode's group cache (all handles)

int qfec_percall_counters(unsigned long long* out, int n) {
    if (!out || n < 0) return QFEC_EINVAL;
    unsigned long long v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
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
    }
    v[6] = g_group_hits.load();
    v[7] = g_group_misses.load();
    v[8] = (unsigned long long)g_percall_idle_us.load();
    for (int i = 0; i < n && i < 9; ++i) out[i] = v[i];
    return std::min(n, 9);
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
    for (auto& h : ctx->host)
        if ((rc = ensure_host_slot(h, (size_t)gc * in_g, (size_t)gc * out_g))) return rc;
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
    for (auto& h : ctx->host)
        if ((rc = ensure_host_slot(h, slot_bytes, slot_bytes))) return rc;
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
    if (a.work >= 0x80000000ull) return QFEC_EINVAL;
    hipError_t e = launch_probe_xor(a, (hipStream_t)stream);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "probe launch");
}

}  // extern "C"

// ====================================================================== host streaming pipe
// BASELINE config 5: batches that start and end in (pinned) host memory, streamed over
// several HIP streams per device and several devices.  Each slot = (device, stream, event,
// device staging, failed counter).  A piece of a batch takes the next slot round-robin
// (devices interleaved), waits for that slot's previous piece, and queues H2D -> kernel ->
// D2H on the slot's stream, so one piece's copies overlap the other slots' kernels and
// copies.  The caller's buffers must be pinned (DMA'd directly, no host memcpy) and stay
// untouched until qfec_pipe_wait.
struct qfec_pipe {
    struct Slot {
        int device = 0;
        DevCtx* ctx = nullptr;
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
        uint8_t* d_buf = nullptr;
        unsigned* d_failed = nullptr;  // accumulated under-determined groups (reconstruct)
        unsigned* h_failed = nullptr;  // pinned read-back
        bool busy = false;
    };
    std::mutex mu;
    std::vector<Slot> slots;
    size_t next = 0;
    size_t cap = 0;  // staging bytes per slot
};

namespace {

// wait for every queued piece (errors are reported after all slots are drained, so no DMA
// is left in flight into caller memory when an error returns)
int pipe_drain(qfec_pipe* p) {
    int rc = QFEC_OK;
    for (auto& s : p->slots) {
        if (!s.busy) continue;
        hipError_t e = hipEventSynchronize(s.done);
        if (e != hipSuccess) {
            (void)hipSetDevice(s.device);
            (void)hipStreamSynchronize(s.stream);
            if (!rc) rc = hip_fail(e, "qfec_pipe: piece failed");
        }
        s.busy = false;
    }
    return rc;
}

struct DeviceRestore {
    int prev = -1;
    DeviceRestore() { if (hipGetDevice(&prev) != hipSuccess) prev = -1; }
    ~DeviceRestore() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// the next slot, with its previous piece finished
int pipe_take(qfec_pipe* p, qfec_pipe::Slot** out) {
    qfec_pipe::Slot& s = p->slots[p->next++ % p->slots.size()];
    HIP_TRY(hipSetDevice(s.device));
    if (s.busy) {
        HIP_TRY(hipEventSynchronize(s.done));
        s.busy = false;
    }
    *out = &s;
    return QFEC_OK;
}

// groups per piece: fits a slot, and a batch spreads over all slots
long long pipe_piece(const qfec_pipe* p, long long groups, size_t per_group) {
    long long fit = (long long)(p->cap / per_group);
    long long even = (groups + (long long)p->slots.size() - 1) / (long long)p->slots.size();
    return std::max<long long>(1, std::min(fit, std::max<long long>(even, 64)));
}

}  // namespace

extern "C" {

qfec_pipe* qfec_pipe_new(const int* devices, int ndev, int nstreams, long long slot_bytes) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        set_error("qfec_pipe_new: no HIP device available");
        return nullptr;
    }
    if (nstreams < 1 || nstreams > 16 || slot_bytes < (1 << 16) || ndev < 0 || ndev > 64 || (ndev > 0 && !devices)) {
        set_error("qfec_pipe_new: invalid argument");
        return nullptr;
    }
    std::vector<int> devs;
    if (ndev == 0)
        for (int d = 0; d < count; ++d) devs.push_back(d);
    else
        devs.assign(devices, devices + ndev);
    for (int d : devs)
        if (d < 0 || d >= count || d >= kMaxDevices) {
            set_error("qfec_pipe_new: device %d out of range (%d visible)", d, count);
            return nullptr;
        }
    DeviceRestore restore;
    qfec_pipe* p = new (std::nothrow) qfec_pipe();
    if (!p) return nullptr;
    p->cap = round_up((size_t)slot_bytes, 4096);
    p->slots.resize((size_t)nstreams * devs.size());
    int rc = QFEC_OK;
    for (size_t i = 0; i < p->slots.size() && !rc; ++i) {
        qfec_pipe::Slot& s = p->slots[i];
        s.device = devs[i % devs.size()];  // devices interleaved: consecutive pieces land on different GPUs
        if (hipSetDevice(s.device) != hipSuccess) { rc = QFEC_EHIP; break; }
        if ((rc = current_ctx(&s.ctx))) break;
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess ||
            hipMalloc(&s.d_buf, p->cap) != hipSuccess || hipMalloc(&s.d_failed, 16) != hipSuccess ||
            hipMemset(s.d_failed, 0, 16) != hipSuccess ||
            hipHostMalloc(&s.h_failed, 16, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            set_error("qfec_pipe_new: allocation on device %d failed", s.device);
            rc = QFEC_ENOMEM;
        }
    }
    if (rc) {
        qfec_pipe_free(p);
        return nullptr;
    }
    return p;
}

void qfec_pipe_free(qfec_pipe* p) {
    if (!p) return;
    DeviceRestore restore;
    {
        std::lock_guard<std::mutex> lk(p->mu);
        (void)pipe_drain(p);
        for (auto& s : p->slots) {
            if (hipSetDevice(s.device) != hipSuccess) continue;
            if (s.d_buf) (void)hipFree(s.d_buf);
            if (s.d_failed) (void)hipFree(s.d_failed);
            if (s.h_failed) (void)hipHostFree(s.h_failed);
            if (s.done) (void)hipEventDestroy(s.done);
            if (s.stream) (void)hipStreamDestroy(s.stream);
        }
    }
    delete p;
}

int qfec_pipe_encode(qfec_pipe* p, qfec_code* code, const unsigned char* h_data, unsigned char* h_parity,
                     long long groups, int block_size, long long pitch) {
    if (!p || !code || groups < 0 || block_size < 1 || pitch < block_size || (groups > 0 && (!h_data || !h_parity))) {
        set_error("qfec_pipe_encode: invalid argument");
        return QFEC_EINVAL;
    }
    if (groups == 0 || code->m == 0) return QFEC_OK;
    const int k = code->k, m = code->m;
    const size_t in_g = (size_t)k * (size_t)pitch, out_g = (size_t)m * (size_t)pitch;
    if (in_g + out_g > p->cap) {
        set_error("qfec_pipe_encode: one group (%zu B) exceeds the slot staging (%zu B)", in_g + out_g, p->cap);
        return QFEC_EINVAL;
    }
    if (!is_pinned_host(h_data) || !is_pinned_host(h_parity)) {
        set_error("qfec_pipe_encode: host buffers must be pinned (hipHostMalloc / hipHostRegister)");
        return QFEC_EINVAL;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    DeviceRestore restore;
    const long long gp = pipe_piece(p, groups, in_g + out_g);
    int rc = QFEC_OK;
    for (long long g0 = 0; g0 < groups && !rc; g0 += gp) {
        const long long gn = std::min(gp, groups - g0);
        qfec_pipe::Slot* s = nullptr;
        if ((rc = pipe_take(p, &s))) break;
        uint32_t* tab = nullptr;
        {
            std::lock_guard<std::mutex> ck(code->mu);
            rc = ensure_enc(code, s->device, &tab);
        }
        if (rc) break;
        uint8_t *z_in = nullptr, *z_out = nullptr;
        if (tuning().host_zero_copy && host_dev(h_data, &z_in) && host_dev(h_parity, &z_out)) {
            // zero copy: the piece's kernel reads and writes the pinned host buffers directly
            s->busy = true;
            if ((rc = run_encode(*s->ctx, code, tab, m, z_in + (size_t)g0 * in_g, z_out + (size_t)g0 * out_g, gn,
                                 block_size, pitch, s->stream, -1, -1, true)))
                break;
            if (hipEventRecord(s->done, s->stream) != hipSuccess) { rc = hip_fail(hipGetLastError(), "event"); break; }
            continue;
        }
        uint8_t* d_in = s->d_buf;
        uint8_t* d_out = s->d_buf + (size_t)gn * in_g;
        if (hipMemcpyAsync(d_in, h_data + (size_t)g0 * in_g, (size_t)gn * in_g, hipMemcpyHostToDevice, s->stream) !=
            hipSuccess) { rc = hip_fail(hipGetLastError(), "qfec_pipe_encode: H2D"); break; }
        s->busy = true;
        if ((rc = run_encode(*s->ctx, code, tab, m, d_in, d_out, gn, block_size, pitch, s->stream))) break;
        if (hipMemcpyAsync(h_parity + (size_t)g0 * out_g, d_out, (size_t)gn * out_g, hipMemcpyDeviceToHost,
                           s->stream) != hipSuccess) { rc = hip_fail(hipGetLastError(), "qfec_pipe_encode: D2H"); break; }
        if (hipEventRecord(s->done, s->stream) != hipSuccess) { rc = hip_fail(hipGetLastError(), "event"); break; }
    }
    if (rc) {
        const std::string err = t_last_error;
        (void)pipe_drain(p);
        t_last_error = err;
    }
    return rc;
}

int qfec_pipe_reconstruct(qfec_pipe* p, qfec_code* code, unsigned char* h_data, const unsigned char* h_parity,
                          const unsigned char* h_marks, long long groups, int block_size, long long pitch) {
    if (!p || !code || groups < 0 || block_size < 1 || pitch < block_size ||
        (groups > 0 && (!h_data || !h_marks || (code->m > 0 && !h_parity)))) {
        set_error("qfec_pipe_reconstruct: invalid argument");
        return QFEC_EINVAL;
    }
    if (groups == 0) return QFEC_OK;
    const int k = code->k, m = code->m;
    if (k + m > QFEC_LUT_MAX_N) {
        set_error("qfec_pipe_reconstruct: k + m = %d > %d", k + m, QFEC_LUT_MAX_N);
        return QFEC_EUNSUP;
    }
    const size_t dg = (size_t)k * (size_t)pitch, pg = (size_t)m * (size_t)pitch;
    const size_t per_group = dg + pg + (size_t)(k + m);
    if (per_group + 64 > p->cap) {
        set_error("qfec_pipe_reconstruct: one group exceeds the slot staging (%zu B)", p->cap);
        return QFEC_EINVAL;
    }
    if (!is_pinned_host(h_data) || (m && !is_pinned_host(h_parity)) || !is_pinned_host(h_marks)) {
        set_error("qfec_pipe_reconstruct: host buffers must be pinned (hipHostMalloc / hipHostRegister)");
        return QFEC_EINVAL;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    DeviceRestore restore;
    const long long gp = pipe_piece(p, groups, per_group + 1);
    int rc = QFEC_OK;
    for (long long g0 = 0; g0 < groups && !rc; g0 += gp) {
        const long long gn = std::min(gp, groups - g0);
        qfec_pipe::Slot* s = nullptr;
        if ((rc = pipe_take(p, &s))) break;
        DevTables* d = nullptr;
        {
            std::lock_guard<std::mutex> ck(code->mu);
            rc = ensure_lut(code, s->device, &d);
        }
        if (rc) break;
        // slot layout: data [gn][k][pitch] | parity [gn][m][pitch] | marks in rs.c layout
        // for the piece: gn*k data marks, then gn*m parity marks (module/rs.c:609-612)
        uint8_t *z_data = nullptr, *z_par = nullptr;
        if (tuning().host_zero_copy && host_dev(h_data, &z_data) && (m == 0 || host_dev(h_parity, &z_par))) {
            // zero copy: survivors read and erased rows written in host memory; the piece's
            // marks (rs.c layout for gn groups) staged into the slot
            uint8_t* dm = s->d_buf;
            s->busy = true;
            if (hipMemcpyAsync(dm, h_marks + (size_t)g0 * k, (size_t)gn * k, hipMemcpyHostToDevice, s->stream) ||
                (m && hipMemcpyAsync(dm + (size_t)gn * k, h_marks + (size_t)groups * k + (size_t)g0 * m, (size_t)gn * m,
                                     hipMemcpyHostToDevice, s->stream))) {
                rc = hip_fail(hipGetLastError(), "qfec_pipe_reconstruct: marks H2D");
                break;
            }
            if ((rc = run_reconstruct(*s->ctx, code, d->d_lut, nullptr, d->d_rec, z_data + (size_t)g0 * dg,
                                      m ? z_par + (size_t)g0 * pg : nullptr, dm, gn, block_size, pitch, s->d_failed,
                                      s->stream)))
                break;
            if (hipEventRecord(s->done, s->stream) != hipSuccess) { rc = hip_fail(hipGetLastError(), "event"); break; }
            continue;
        }
        uint8_t* dd = s->d_buf;
        uint8_t* dp = dd + (size_t)gn * dg;
        uint8_t* dm = dp + (size_t)gn * pg;
        s->busy = true;
        if (hipMemcpyAsync(dd, h_data + (size_t)g0 * dg, (size_t)gn * dg, hipMemcpyHostToDevice, s->stream) ||
            (m && hipMemcpyAsync(dp, h_parity + (size_t)g0 * pg, (size_t)gn * pg, hipMemcpyHostToDevice, s->stream)) ||
            hipMemcpyAsync(dm, h_marks + (size_t)g0 * k, (size_t)gn * k, hipMemcpyHostToDevice, s->stream) ||
            (m && hipMemcpyAsync(dm + (size_t)gn * k, h_marks + (size_t)groups * k + (size_t)g0 * m, (size_t)gn * m,
                                 hipMemcpyHostToDevice, s->stream))) {
            rc = hip_fail(hipGetLastError(), "qfec_pipe_reconstruct: H2D");
            break;
        }
        if ((rc = run_reconstruct(*s->ctx, code, d->d_lut, nullptr, d->d_rec, dd, dp, dm, gn, block_size, pitch,
                                  s->d_failed, s->stream)))
            break;
        if (hipMemcpyAsync(h_data + (size_t)g0 * dg, dd, (size_t)gn * dg, hipMemcpyDeviceToHost, s->stream) !=
            hipSuccess) { rc = hip_fail(hipGetLastError(), "qfec_pipe_reconstruct: D2H"); break; }
        if (hipEventRecord(s->done, s->stream) != hipSuccess) { rc = hip_fail(hipGetLastError(), "event"); break; }
    }
    if (rc) {
        const std::string err = t_last_error;
        (void)pipe_drain(p);
        t_last_error = err;
    }
    return rc;
}

int qfec_pipe_wait(qfec_pipe* p, long long* failed) {
    if (!p) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(p->mu);
    DeviceRestore restore;
    int rc = pipe_drain(p);
    long long nf = 0;
    for (auto& s : p->slots) {  // read back and reset the slots' failed counters
        if (hipSetDevice(s.device) != hipSuccess ||
            hipMemcpyAsync(s.h_failed, s.d_failed, 4, hipMemcpyDeviceToHost, s.stream) != hipSuccess ||
            hipMemsetAsync(s.d_failed, 0, 4, s.stream) != hipSuccess || hipStreamSynchronize(s.stream) != hipSuccess) {
            if (!rc) rc = hip_fail(hipGetLastError(), "qfec_pipe_wait");
            continue;
        }
        nf += *s.h_failed;
    }
    if (failed) *failed = nf;
    return rc;
}

int qfec_pipe_slots(const qfec_pipe* p) { return p ? (int)p->slots.size() : QFEC_EINVAL; }

}  // extern "C"

// ====================================================================== FEC datagram batches
namespace {

int wire_check(const qfec_code* c, long long groups, int checksum, long long pitch, long long wire_pitch,
               const void* shards, const void* wire) {
    if (!c || groups < 0 || (checksum != 0 && checksum != 1)) return QFEC_EINVAL;
    if (c->k + c->m > 15 || c->k < 1) {
        set_error("FEC datagrams carry 4-bit n and k (network/FecCodecBuf.cpp:290-299): n = %d > 15", c->k + c->m);
        return QFEC_EUNSUP;
    }
    if (pitch < 16 || pitch % 16 || wire_pitch % 16 || wire_pitch < (long long)round_up((size_t)pitch + 13, 16) ||
        ((uintptr_t)shards | (uintptr_t)wire) % 16) {
        set_error("datagram batch: shard pitch and wire pitch must be multiples of 16, wire >= shard + 13, 16-B aligned");
        return QFEC_EINVAL;
    }
    return QFEC_OK;
}

// frame rows: a 16-B multiple pitch that holds prefix + 13 + shard pitch
int frame_check(const qfec_code* c, long long groups, int checksum, long long pitch, long long frame_pitch, int fp,
                const void* shards, const void* frames) {
    const int rc = wire_check(c, groups, checksum, pitch, (long long)round_up((size_t)pitch + 13, 16), shards, frames);
    if (rc) return rc;
    if (frame_pitch % 16 || frame_pitch < pitch + 13 + fp) {
        set_error("frames: frame pitch must be a multiple of 16 and >= prefix (%d) + 13 + shard pitch", fp);
        return QFEC_EINVAL;
    }
    return QFEC_OK;
}

}  // namespace

extern "C" {

int qfec_pack_datagrams(qfec_code* code, const unsigned char* d_payload, const long long* d_offsets,
                        const int* d_sizes, const unsigned int* d_seq, long long groups, int checksum,
                        unsigned char* d_shards, long long shard_pitch, unsigned char* d_wire, long long wire_pitch,
                        int* d_wire_len, void* stream) {
    int rc = wire_check(code, groups, checksum, shard_pitch, wire_pitch, d_shards, d_wire);
    if (rc) return rc;
    if (groups == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    if ((rc = current_ctx(&ctx))) return rc;
    uint32_t* tab = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_enc(code, ctx->device, &tab);
    }
    if (rc) return rc;
    const int k = code->k, m = code->m, n = k + m;
    hipStream_t s = (hipStream_t)stream;
    WireArgs a{};
    a.payload = d_payload;
    a.offsets = (const int64_t*)d_offsets;
    a.sizes = d_sizes;
    a.seq = d_seq;
    a.shards = d_shards;
    a.pitch = (uint64_t)shard_pitch;
    a.group_stride = (uint64_t)n * shard_pitch;
    a.wire = d_wire;
    a.wire_pitch = (uint64_t)wire_pitch;
    a.wire_len = d_wire_len;
    a.groups = (uint64_t)groups;
    a.k = k;
    a.m = m;
    a.checksum = checksum;
    a.store_nt = 3;  // non-temporal datagram stores, body and head
    if (tuning().wire_fused) {
        bool launched = false;
        // the fused path never materialises shards; their buffer holds its partial sums
        // ((wire_pitch + 63) / 256 + 2) * 8 u32 per group  <<  n * pitch bytes
        hipError_t e = launch_pack_fused(a, tab, reinterpret_cast<uint32_t*>(d_shards), s, &launched);
        if (e != hipSuccess) return hip_fail(e, "pack_fused launch");
        if (launched) return QFEC_OK;
    }
    hipError_t e = launch_build_shards(a, s);
    if (e != hipSuccess) return hip_fail(e, "build_shards launch");
    // check shards: fec_encode(.., groupMax) over the k data shards (FecCodecBuf.cpp:151);
    // bytes past a group's groupMax are zero in every data shard, hence in the parity.
    if (m > 0 && (rc = run_encode(*ctx, code, tab, m, d_shards, d_shards + (size_t)k * shard_pitch, groups,
                                  (int)shard_pitch, shard_pitch, s, (long long)a.group_stride, (long long)a.group_stride)))
        return rc;
    e = launch_emit_wire(a, s);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "emit_wire launch");
}

int qfec_unpack_datagrams(qfec_code* code, const unsigned char* d_wire, long long wire_pitch, const int* d_wire_len,
                          long long groups, int checksum, int dec_pkt_size, unsigned char* d_shards,
                          long long shard_pitch, unsigned char* d_marks, int* d_rx_size, int* d_status, int* d_psize,
                          void* stream) {
    int rc = wire_check(code, groups, checksum, shard_pitch, wire_pitch, d_shards, d_wire);
    if (rc) return rc;
    if (groups == 0) return QFEC_OK;
    if (!d_marks || !d_status || !d_psize || !d_wire_len) return QFEC_EINVAL;
    DevCtx* ctx = nullptr;
    if ((rc = current_ctx(&ctx))) return rc;
    DevTables* d = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_lut(code, ctx->device, &d);
    }
    if (rc) return rc;
    const int k = code->k, m = code->m, n = k + m;
    hipStream_t s = (hipStream_t)stream;
    WireArgs a{};
    a.shards = d_shards;
    a.pitch = (uint64_t)shard_pitch;
    a.group_stride = (uint64_t)n * shard_pitch;
    a.wire = const_cast<uint8_t*>(d_wire);
    a.wire_pitch = (uint64_t)wire_pitch;
    a.wire_len = const_cast<int32_t*>(d_wire_len);
    a.marks = d_marks;
    a.rx_size = d_rx_size;
    a.status = d_status;
    a.psize = d_psize;
    a.groups = (uint64_t)groups;
    a.k = k;
    a.m = m;
    a.checksum = checksum;
    a.dec_pkt_size = dec_pkt_size;
    if (tuning().wire_rx && d->d_lut) {
        bool launched = false;
        const hipError_t ef =
            launch_unpack_fused(a, d->d_lut, d->d_rec, (uint32_t)record_layout(k, m).hdr, s, &launched);
        if (ef != hipSuccess) return hip_fail(ef, "unpack_fused launch");
        if (launched) return QFEC_OK;
    }
    hipError_t e = launch_parse_wire(a, s);
    if (e != hipSuccess) return hip_fail(e, "parse_wire launch");
    // decode the missing data shards from the first k valid ones in group order
    // (network/NetFecCodec.cpp:504-528 == module/rs.c:620-629)
    if ((rc = run_reconstruct(*ctx, code, d->d_lut, nullptr, d->d_rec, d_shards, d_shards + (size_t)k * shard_pitch,
                              d_marks, groups, (int)shard_pitch, shard_pitch, nullptr, s, (long long)a.group_stride,
                              (long long)a.group_stride)))
        return rc;
    e = launch_check_payloads(a, s);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "check_payloads launch");
}


// ---- datagrams straight to / from ProtocolUdp frames (one pass where a kernel instance exists)
int qfec_pack_frames(qfec_code* code, const unsigned char* d_payload, const long long* d_offsets, const int* d_sizes,
                     const unsigned int* d_seq, long long groups, int checksum, unsigned char* d_shards,
                     long long shard_pitch, const unsigned char* d_mask, const unsigned int* d_conv_hid, int gmask,
                     int cmd, int protocol, unsigned char* d_frames, long long frame_pitch, int* d_frame_len,
                     void* stream) {
    const int fp = d_conv_hid ? 12 : 4;
    int rc = frame_check(code, groups, checksum, shard_pitch, frame_pitch, fp, d_shards, d_frames);
    if (rc) return rc;
    if (!d_mask || !d_frame_len) return QFEC_EINVAL;
    if (groups == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    if ((rc = current_ctx(&ctx))) return rc;
    uint32_t* tab = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_enc(code, ctx->device, &tab);
    }
    if (rc) return rc;
    const int k = code->k, m = code->m, n = k + m;
    hipStream_t s = (hipStream_t)stream;
    if (tuning().wire_fused) {
        WireArgs a{};
        a.payload = d_payload;
        a.offsets = (const int64_t*)d_offsets;
        a.sizes = d_sizes;
        a.seq = d_seq;
        a.pitch = (uint64_t)shard_pitch;
        a.group_stride = (uint64_t)n * shard_pitch;
        a.wire = d_frames;
        a.wire_pitch = (uint64_t)frame_pitch;
        a.wire_len = d_frame_len;
        a.groups = (uint64_t)groups;
        a.k = k;
        a.m = m;
        a.checksum = checksum;
        a.store_nt = 3;  // non-temporal datagram stores, body and head
        FrameSend fs{d_mask, d_conv_hid, (uint32_t)gmask & 0xFFu, (uint32_t)cmd, (uint32_t)protocol};
        bool launched = false;
        const hipError_t e = launch_pack_frames(a, fs, fp, tab, s, &launched);
        if (e != hipSuccess) return hip_fail(e, "pack_frames launch");
        if (launched) return QFEC_OK;
    }
    // two passes: datagrams into stream-ordered scratch, then qfec_frame_udp over them
    const long long wp = (long long)round_up((size_t)shard_pitch + 13, 16);
    const size_t rows = (size_t)groups * n, wbytes = rows * (size_t)wp;
    uint8_t* scratch = nullptr;
    if (hipMallocAsync((void**)&scratch, wbytes + rows * 4, s) != hipSuccess)
        return hip_fail(hipGetLastError(), "pack_frames scratch");
    int* wlen = reinterpret_cast<int*>(scratch + wbytes);
    rc = qfec_pack_datagrams(code, d_payload, d_offsets, d_sizes, d_seq, groups, checksum, d_shards, shard_pitch,
                             scratch, wp, wlen, stream);
    if (!rc)
        rc = qfec_frame_udp(scratch, wp, wlen, (long long)rows, d_mask, d_conv_hid, gmask, cmd, protocol, d_frames,
                            frame_pitch, d_frame_len, stream);
    (void)hipFreeAsync(scratch, s);
    return rc;
}

int qfec_unpack_frames(qfec_code* code, const unsigned char* d_frames, long long frame_pitch, const int* d_frame_len,
                       long long groups, int gmask, int session, int checksum, int dec_pkt_size,
                       unsigned char* d_shards, long long shard_pitch, unsigned char* d_marks, int* d_rx_size,
                       int* d_status, int* d_psize, int* d_frame_status, unsigned int* d_conv_hid, void* stream) {
    if (session != 0 && session != 1) return QFEC_EINVAL;
    const int fp = session ? 12 : 4;
    int rc = frame_check(code, groups, checksum, shard_pitch, frame_pitch, fp, d_shards, d_frames);
    if (rc) return rc;
    if (groups == 0) return QFEC_OK;
    if (!d_marks || !d_status || !d_psize || !d_frame_len) return QFEC_EINVAL;
    DevCtx* ctx = nullptr;
    if ((rc = current_ctx(&ctx))) return rc;
    DevTables* d = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_lut(code, ctx->device, &d);
    }
    if (rc) return rc;
    const int k = code->k, m = code->m, n = k + m;
    hipStream_t s = (hipStream_t)stream;
    if (tuning().wire_rx && d->d_lut) {
        WireArgs a{};
        a.shards = d_shards;
        a.pitch = (uint64_t)shard_pitch;
        a.group_stride = (uint64_t)n * shard_pitch;
        a.wire = const_cast<uint8_t*>(d_frames);
        a.wire_pitch = (uint64_t)frame_pitch;
        a.wire_len = const_cast<int32_t*>(d_frame_len);
        a.marks = d_marks;
        a.rx_size = d_rx_size;
        a.status = d_status;
        a.psize = d_psize;
        a.groups = (uint64_t)groups;
        a.k = k;
        a.m = m;
        a.checksum = checksum;
        a.dec_pkt_size = dec_pkt_size;
        FrameRecv fr{(uint32_t)gmask & 0xFFu, d_frame_status, session ? d_conv_hid : nullptr};
        bool launched = false;
        const hipError_t e = launch_unpack_frames(a, fr, fp, d->d_lut, d->d_rec, (uint32_t)record_layout(k, m).hdr, s,
                                                  &launched);
        if (e != hipSuccess) return hip_fail(e, "unpack_frames launch");
        if (launched) return QFEC_OK;
    }
    // two passes: qfec_unframe_udp into stream-ordered scratch (rows RecvPacket rejects count as
    // not received), then qfec_unpack_datagrams
    const long long wp = (long long)round_up((size_t)frame_pitch, 16);
    const size_t rows = (size_t)groups * n, wbytes = rows * (size_t)wp;
    uint8_t* scratch = nullptr;
    if (hipMallocAsync((void**)&scratch, wbytes + rows * 8, s) != hipSuccess)
        return hip_fail(hipGetLastError(), "unpack_frames scratch");
    int* wlen = reinterpret_cast<int*>(scratch + wbytes);
    int* fst = d_frame_status ? d_frame_status : wlen + rows;
    rc = qfec_unframe_udp(d_frames, frame_pitch, d_frame_len, (long long)rows, gmask, session, scratch, wp, wlen, fst,
                          nullptr, session ? d_conv_hid : nullptr, stream);
    if (!rc) {
        const hipError_t e = launch_len_by_status(wlen, fst, rows, s);
        if (e != hipSuccess) rc = hip_fail(e, "len_by_status launch");
    }
    if (!rc)
        rc = qfec_unpack_datagrams(code, scratch, wp, wlen, groups, checksum, dec_pkt_size, d_shards, shard_pitch,
                                   d_marks, d_rx_size, d_status, d_psize, stream);
    (void)hipFreeAsync(scratch, s);
    return rc;
}

int qfec_gather_rows(const unsigned char* d_base, const unsigned long long* d_off, const int* d_len, long long rows,
                     int wrap_n, int wrap_k, unsigned char* d_out, long long out_pitch, int* d_out_len, void* stream) {
    if (rows < 0 || (rows && (!d_base || !d_off || !d_len || !d_out || !d_out_len)) || out_pitch < 16 || out_pitch % 16 ||
        (uintptr_t)d_out % 16 || wrap_n < 0 || wrap_n > 15 || (wrap_n && (wrap_k < 1 || wrap_k >= wrap_n))) {
        set_error("gather_rows: out_pitch a multiple of 16, 16-B aligned output, 0 < wrap_k < wrap_n <= 15");
        return QFEC_EINVAL;
    }
    if (rows == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    const int rc = current_ctx(&ctx);
    if (rc) return rc;
    const hipError_t e = launch_gather_rows(d_base, (const uint64_t*)d_off, d_len, (uint64_t)rows, wrap_n, wrap_k, d_out,
                                            (uint64_t)out_pitch, d_out_len, (hipStream_t)stream);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "gather_rows launch");
}

int qfec_frame_udp(const unsigned char* d_in, long long in_pitch, const int* d_len, long long rows,
                   const unsigned char* d_mask, const unsigned int* d_conv_hid, int gmask, int cmd, int protocol,
                   unsigned char* d_out, long long out_pitch, int* d_out_len, void* stream) {
    if (rows < 0 || !d_len || !d_mask || !d_out_len || in_pitch < 16 || out_pitch < 16 || in_pitch % 16 ||
        out_pitch % 16 || ((uintptr_t)d_in | (uintptr_t)d_out) % 16) {
        set_error("frame_udp: pitches must be multiples of 16 and rows 16-B aligned");
        return QFEC_EINVAL;
    }
    if (rows == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    FrameArgs a{};
    a.in = d_in;
    a.in_len = d_len;
    a.out = d_out;
    a.out_len = d_out_len;
    a.mask = d_mask;
    a.conv_hid = const_cast<uint32_t*>(d_conv_hid);
    a.rows = (uint64_t)rows;
    a.in_pitch = (uint64_t)in_pitch;
    a.out_pitch = (uint64_t)out_pitch;
    a.gmask = (uint32_t)gmask & 0xFFu;
    a.cmd = (uint32_t)cmd;
    a.protocol = (uint32_t)protocol;
    a.session = d_conv_hid != nullptr;
    const hipError_t e = launch_frame_udp(a, (hipStream_t)stream);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "frame_udp launch");
}

int qfec_unframe_udp(const unsigned char* d_in, long long in_pitch, const int* d_len, long long rows, int gmask,
                     int session, unsigned char* d_out, long long out_pitch, int* d_out_len, int* d_status,
                     unsigned char* d_info, unsigned int* d_conv_hid, void* stream) {
    if (rows < 0 || !d_len || !d_out_len || !d_status || (session != 0 && session != 1) || in_pitch < 16 ||
        out_pitch < 16 || in_pitch % 16 || out_pitch % 16 || ((uintptr_t)d_in | (uintptr_t)d_out) % 16) {
        set_error("unframe_udp: pitches must be multiples of 16 and rows 16-B aligned");
        return QFEC_EINVAL;
    }
    if (rows == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    FrameArgs a{};
    a.in = d_in;
    a.in_len = d_len;
    a.out = d_out;
    a.out_len = d_out_len;
    a.conv_hid = d_conv_hid;
    a.status = d_status;
    a.info = d_info;
    a.rows = (uint64_t)rows;
    a.in_pitch = (uint64_t)in_pitch;
    a.out_pitch = (uint64_t)out_pitch;
    a.gmask = (uint32_t)gmask & 0xFFu;
    a.session = session;
    const hipError_t e = launch_unframe_udp(a, (hipStream_t)stream);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "unframe_udp launch");
}

}  // extern "C"

// ====================================================================== host-buffer paths
namespace {

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
    std::vector<std::pair<uintptr_t, uintptr_t>> dev;  // device allocation ranges [lo, hi)
    std::vector<uintptr_t> host_win;                   // 64 KiB windows with a host verdict
    uintptr_t last_win = ~(uintptr_t)0;
    size_t last_dev = 0;
    bool is_dev(const void* p) {
        const uintptr_t u = (uintptr_t)p, w = u >> 16;
        if (last_dev < dev.size() && u >= dev[last_dev].first && u < dev[last_dev].second) return true;
        for (size_t i = 0; i < dev.size(); ++i)
            if (u >= dev[i].first && u < dev[i].second) {
                last_dev = i;
                return true;
            }
        if (w == last_win) return false;
        for (uintptr_t x : host_win)
            if (x == w) {
                last_win = w;
                return false;
            }
        hipPointerAttribute_t attr;
        const hipError_t e = hipPointerGetAttributes(&attr, p);
        if (e == hipSuccess && (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged)) {
            void* base = nullptr;
            size_t size = 0;
            if (hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) == hipSuccess && base && size) {
                dev.emplace_back((uintptr_t)base, (uintptr_t)base + size);
                last_dev = dev.size() - 1;
            } else {
                (void)hipGetLastError();
                dev.emplace_back(u, u + 1);  // this pointer only
            }
            return true;
        }
        if (e != hipSuccess) (void)hipGetLastError();
        if (host_win.size() < 4096) host_win.push_back(w);
        last_win = w;
        return false;
    }
};


constexpr size_t kMapsMinPointers = 4096;

// number of device pointers among ptrs[0 .. count), classified on the host pool's threads
size_t count_device_ptrs(unsigned char* const* ptrs, size_t count, HostPool& pool) {
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
                if (have_maps && maps.host((uintptr_t)ptrs[i], &hint)) continue;
                nd += pc.is_dev(ptrs[i]) ? 1 : 0;
            }
            ndev += nd;
        },
        (int)std::max<size_t>(1, count >> 14));
    return ndev.load();
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

// bytes of caller shards per pipelined chunk of the host-pointer paths (tuning "host_chunk"
// overrides with groups per chunk)
constexpr size_t kRsPipeBytes = (size_t)16 << 20;

// the slot's device view: the pinned staging itself (zero copy) or the slot's device buffer
uint8_t* rs_slot_dev(DevCtx::HostSlot& h, bool zc) {
    uint8_t* z = nullptr;
    if (zc && host_dev(h.h_in, &z)) return z;
    return nullptr;
}

// reed_solomon_encode over host shard pointers: chunks of groups alternate between two pinned
// slots; the host threads gather a chunk's data rows into one slot while the device encodes the
// previous chunk out of the other (reading and writing the pinned slot in place, or through the
// slot's device buffer), and scatter each chunk's parity rows once its event has fired.
int rs_encode_pipe(DevCtx& ctx, const qfec_code* c, const uint32_t* tab, unsigned char** data, unsigned char** par,
                   long long G, int B, bool any_stale) {
    const int k = c->k, m = c->m;
    const size_t pitch = round_up((size_t)B, 16), dg = (size_t)k * pitch, pg = (size_t)m * pitch;
    long long per = tuning().host_chunk > 0 ? (long long)tuning().host_chunk
                                            : std::max<long long>(1, (long long)(kRsPipeBytes / (dg + pg)));
    per = std::min(per, G);
    const size_t slot_bytes = (size_t)per * (dg + pg);
    std::shared_ptr<HostPool> pool = host_pool();
    std::lock_guard<std::mutex> lk(ctx.host_mu);
    int rc = QFEC_OK;
    for (auto& h : ctx.host)
        if ((rc = ensure_host_slot(h, slot_bytes, 16))) return rc;
    // staged: the DMA engines move the slot to the device and the parity back.  Reading the
    // freshly gathered slot in place over PCIe ran slower for the encode (26.4-26.9 against
    // 28.3-38.8 GiB/s in alternating processes, profiles/r05af); the reconstruct, which reads only
    // the survivors it needs and writes only the erased rows, stays in place (host_zero_copy)
    const bool zc = false;
    RsTrace tr;
    long long pending[2] = {-1, -1};
    auto rows_job = [&](size_t nrows, const std::function<void(size_t)>& row) {
        pool->run(
            [&](int t, int nt) {
                const size_t a = nrows * t / nt, b = nrows * (t + 1) / nt;
                for (size_t i = a; i < b; ++i) row(i);
            },
            (int)std::max<size_t>(1, nrows / 64));
    };
    auto drain = [&](int sl) -> int {
        if (pending[sl] < 0) return QFEC_OK;
        DevCtx::HostSlot& h = ctx.host[sl];
        auto tw = std::chrono::steady_clock::now();
        HIP_TRY(hipEventSynchronize(h.done));
        tr.wait += RsTrace::since(tw);
        tw = std::chrono::steady_clock::now();
        const long long g0 = pending[sl], gn = std::min(per, G - g0);
        const uint8_t* hp = h.h_in + (size_t)gn * dg;
        rows_job((size_t)gn * m, [&](size_t i) { memcpy(par[(size_t)g0 * m + i], hp + i * pitch, (size_t)B); });
        tr.scatter += RsTrace::since(tw);
        pending[sl] = -1;
        return QFEC_OK;
    };
    const long long nchunks = (G + per - 1) / per;
    for (long long i = 0; i < nchunks && !rc; ++i) {
        const int sl = (int)(i & 1);
        DevCtx::HostSlot& h = ctx.host[sl];
        const long long g0 = i * per, gn = std::min(per, G - g0);
        uint8_t* hd = h.h_in;
        uint8_t* hp = h.h_in + (size_t)gn * dg;
        // data rows (and, when a parity row keeps its old bytes -- the rs.c quirk -- the parity rows)
        const size_t nd = (size_t)gn * k, np = any_stale ? (size_t)gn * m : 0;
        const auto tg = std::chrono::steady_clock::now();
        rows_job(nd + np, [&](size_t r) {
            if (r < nd) memcpy(hd + r * pitch, data[(size_t)g0 * k + r], (size_t)B);
            else memcpy(hp + (r - nd) * pitch, par[(size_t)g0 * m + (r - nd)], (size_t)B);
        });
        tr.gather += RsTrace::since(tg);
        uint8_t* z = rs_slot_dev(h, zc);
        uint8_t* dd = z ? z : h.d_buf;
        if (!z) {
            const hipError_t e = hipMemcpyAsync(dd, hd, (size_t)gn * dg + np * pitch, hipMemcpyHostToDevice, h.stream);
            if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_encode: H2D"); break; }
        }
        if ((rc = run_encode(ctx, c, tab, m, dd, dd + (size_t)gn * dg, gn, B, (long long)pitch, h.stream))) break;
        if (!z) {
            const hipError_t e = hipMemcpyAsync(hp, dd + (size_t)gn * dg, (size_t)gn * pg, hipMemcpyDeviceToHost, h.stream);
            if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_encode: D2H"); break; }
        }
        const hipError_t e = hipEventRecord(h.done, h.stream);
        if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_encode: event"); break; }
        pending[sl] = g0;
        if (i > 0 && (rc = drain(sl ^ 1))) break;  // the previous chunk, while this one runs
    }
    if (!rc) rc = drain((int)((nchunks - 1) & 1));
    if (rc) quiesce_host_slots(ctx);  // nothing may still be writing into the slots
    tr.report("reed_solomon_encode (host)", nchunks, pool->threads());
    return rc;
}

// reed_solomon_reconstruct over host shard pointers (k + m <= QFEC_LUT_MAX_N): the same two-slot
// pipeline.  Per group only what the decode reads is staged -- the surviving data rows and the
// first e surviving parity rows (rs.c:611-629), plus the erased rows where the pattern's record
// seeds a row from its old bytes (the rs.c quirk) -- with the chunk's marks in rs.c layout; the
// LUT kernel decodes and only the erased data rows of recoverable groups are scattered back.
// Groups with more erased data than surviving parity are left untouched and counted (*nfail).
int rs_reconstruct_pipe(DevCtx& ctx, qfec_code* c, const DevTables* d, const uint8_t* seed, unsigned char** data,
                        unsigned char** par, const uint8_t* mk, long long G, int B, long long* nfail) {
    const int k = c->k, m = c->m, n = k + m;
    const size_t pitch = round_up((size_t)B, 16), dg = (size_t)k * pitch, pg = (size_t)m * pitch;
    long long per = tuning().host_chunk > 0 ? (long long)tuning().host_chunk
                                            : std::max<long long>(1, (long long)(kRsPipeBytes / (dg + pg)));
    per = std::min(per, G);
    const size_t mk_off = (size_t)per * (dg + pg), slot_bytes = round_up(mk_off + (size_t)per * n, 16);
    std::shared_ptr<HostPool> pool = host_pool();
    std::lock_guard<std::mutex> lk(ctx.host_mu);
    int rc = QFEC_OK;
    for (auto& h : ctx.host)
        if ((rc = ensure_host_slot(h, slot_bytes, 16))) return rc;
    const bool zc = tuning().host_zero_copy != 0;
    RsTrace tr;
    std::vector<uint8_t> todo[2];  // per slot, per group: 1 = decoded (scatter its erased data rows)
    long long pending[2] = {-1, -1};
    std::atomic<long long> fails{0};
    auto groups_job = [&](long long gn, const std::function<void(long long, long long)>& span) {
        pool->run(
            [&](int t, int nt) { span(gn * t / nt, gn * (t + 1) / nt); }, (int)std::max<long long>(1, gn / 16));
    };
    auto drain = [&](int sl) -> int {
        if (pending[sl] < 0) return QFEC_OK;
        DevCtx::HostSlot& h = ctx.host[sl];
        auto tw = std::chrono::steady_clock::now();
        HIP_TRY(hipEventSynchronize(h.done));
        tr.wait += RsTrace::since(tw);
        tw = std::chrono::steady_clock::now();
        const long long g0 = pending[sl], gn = std::min(per, G - g0);
        const uint8_t* todo_s = todo[sl].data();
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
        pending[sl] = -1;
        return QFEC_OK;
    };
    const long long nchunks = (G + per - 1) / per;
    for (long long i = 0; i < nchunks && !rc; ++i) {
        const int sl = (int)(i & 1);
        DevCtx::HostSlot& h = ctx.host[sl];
        const long long g0 = i * per, gn = std::min(per, G - g0);
        uint8_t* hd = h.h_in;
        uint8_t* hp = h.h_in + (size_t)gn * dg;
        uint8_t* hm = h.h_in + (size_t)gn * (dg + pg);
        todo[sl].assign((size_t)gn, 0);
        uint8_t* todo_s = todo[sl].data();
        const auto tg = std::chrono::steady_clock::now();
        groups_job(gn, [&](long long a, long long b) {
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
                        memcpy(hp + ((size_t)g * m + j) * pitch, par[gg * m + j], (size_t)B);
                        ++got;
                    }
                if (got < e) {  // under-determined: left as it is (rs.c:630-634)
                    ++nf;
                    continue;
                }
                const bool sd = seed[mask] != 0;
                for (int x = 0; x < k; ++x)
                    if (!dm[x] || sd) memcpy(hd + ((size_t)g * k + x) * pitch, data[gg * k + x], (size_t)B);
                todo_s[g] = 1;
            }
            fails += nf;
        });
        tr.gather += RsTrace::since(tg);
        uint8_t* z = rs_slot_dev(h, zc);
        uint8_t* dd = z ? z : h.d_buf;
        const size_t used = (size_t)gn * (dg + pg + n);
        if (!z) {
            const hipError_t e = hipMemcpyAsync(dd, h.h_in, used, hipMemcpyHostToDevice, h.stream);
            if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_reconstruct: H2D"); break; }
        }
        if ((rc = run_reconstruct(ctx, c, d->d_lut, nullptr, d->d_rec, dd, dd + (size_t)gn * dg,
                                  dd + (size_t)gn * (dg + pg), gn, B, (long long)pitch, nullptr, h.stream)))
            break;
        if (!z) {
            const hipError_t e = hipMemcpyAsync(h.h_in, dd, (size_t)gn * dg, hipMemcpyDeviceToHost, h.stream);
            if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_reconstruct: D2H"); break; }
        }
        const hipError_t e = hipEventRecord(h.done, h.stream);
        if (e != hipSuccess) { rc = hip_fail(e, "reed_solomon_reconstruct: event"); break; }
        pending[sl] = g0;
        if (i > 0 && (rc = drain(sl ^ 1))) break;
    }
    if (!rc) rc = drain((int)((nchunks - 1) & 1));
    if (rc) quiesce_host_slots(ctx);
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
    // every shard pointer is classified: all device -> in place (or device gathers), all host ->
    // the pipelined host path, a mix -> one copy per row, whatever memory each row is in
    const size_t nptr = (size_t)G * n;
    const auto tc = std::chrono::steady_clock::now();
    const size_t ndev = count_device_ptrs(shards, nptr, *host_pool());
    t_rs_classify = RsTrace::since(tc);
    if (ndev == 0) {
        rc = rs_encode_pipe(*ctx, c, tab, data, par, G, block_size, any_stale);
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
        if ((rc = gather_rows(*ctx, data + g0 * k, (size_t)gn * k, block_size, pitch, d_d, ctx->h_stage, true))) break;
        if (any_stale &&
            (rc = gather_rows(*ctx, par + g0 * m, (size_t)gn * m, block_size, pitch, d_p, ctx->h_stage + dbytes, true)))
            break;
        if ((rc = run_encode(*ctx, c, tab, m, d_d, d_p, gn, block_size, (long long)pitch, ctx->stream))) break;
        rc = scatter_rows(*ctx, par + g0 * m, (size_t)gn * m, block_size, pitch, d_p, ctx->h_stage + dbytes, true,
                          nullptr);
    }
    if (rc) {
        (void)hipStreamSynchronize(ctx->stream);
        fprintf(stderr, "[qfec] reed_solomon_encode: %s\n", qfec_last_error());
    }
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
    // all shards in host memory and a pattern LUT in reach: the pipelined host path
    if (n <= QFEC_LUT_MAX_N) {
        bool any = false;
        for (size_t i = 0; i < (size_t)G * k && !any; ++i) any = mk[i] != 0;
        if (!any) return 0;  // nothing erased: nothing to do (rs.c:618-620)
        if ((rc = current_ctx(&ctx))) {
            fprintf(stderr, "[qfec] reed_solomon_reconstruct: %s\n", qfec_last_error());
            return rc;
        }
        const auto tc = std::chrono::steady_clock::now();
        const bool all_host = count_device_ptrs(shards, (size_t)G * n, *host_pool()) == 0;
        t_rs_classify = RsTrace::since(tc);
        if (all_host) {
            DevTables* d = nullptr;
            std::vector<uint8_t> seed;
            {
                std::lock_guard<std::mutex> lk(c->mu);
                rc = ensure_lut(c, ctx->device, &d);
                if (!rc) seed = c->lut_seed;
            }
            if (!rc) rc = rs_reconstruct_pipe(*ctx, c, d, seed.data(), data, par, mk, G, block_size, &nfail_all);
            if (rc) {
                fprintf(stderr, "[qfec] reed_solomon_reconstruct: %s\n", qfec_last_error());
                return rc;
            }
            return nfail_all ? -1 : 0;
        }
    }
    // device or mixed pointers (or n > 24): chunks of ~kChunkBytes of staged shards, each with its
    // own decode records (built from that chunk's marks), so staging stays bounded whatever the
    // batch size; one copy per row, whatever memory it is in; groups left under-determined -> -1
    // (rs.c:631-634), counted on the host by the kernel's rule
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
        rc = gather_rows(*ctx, data + g0 * k, (size_t)gn * k, block_size, pitch, d_d, hs, true);
        if (!rc) rc = gather_rows(*ctx, par + g0 * m, (size_t)gn * m, block_size, pitch, d_p, hs + dbytes, true);
        if (!rc && hipMemcpyAsync(d_g, hs + dbytes + pbytes, gbytes + rbytes, hipMemcpyHostToDevice, ctx->stream) !=
                       hipSuccess)
            rc = hip_fail(hipGetLastError(), "reed_solomon_reconstruct: H2D");
        if (!rc) rc = run_reconstruct(*ctx, c, nullptr, d_g, d_r, d_d, d_p, nullptr, gn, block_size, (long long)pitch,
                                      nullptr, ctx->stream);
        if (!rc) rc = scatter_rows(*ctx, data + g0 * k, (size_t)gn * k, block_size, pitch, d_d, hs, true, only.data());
        if (rc) (void)hipStreamSynchronize(ctx->stream);  // nothing left in flight into the staging
    }
    if (rc) {
        fprintf(stderr, "[qfec] reed_solomon_reconstruct: %s\n", qfec_last_error());
        return rc;
    }
    return nfail_all ? -1 : 0;
}

}  // extern "C"

// ====================================================================== system/fec.h ABI
namespace {

struct fec_handle {
    int k, n;
    qfec_code* code;
    std::vector<uint8_t> full;  // n x k systematic matrix (identity on top)
    // per-call tables, built once (the reference rebuilds its decode matrix on every call,
    // fec.c:778-808; here only the first call with a given pattern pays for the inversion)
    std::mutex mu;
    std::vector<std::vector<uint32_t>> enc_tab;  // [index] perm tables of parity row `index`
    struct Dec {
        std::vector<int> idx;    // the shuffled index[] this entry is for
        std::vector<int> slots;  // slots holding parity: the rows to recover
        std::vector<uint32_t> tab;
    };
    std::unordered_map<uint64_t, std::shared_ptr<const Dec>> dec;  // keyed by a hash of the shuffled index[]
    // fec_encode's group cache.  The network layer asks for a group's check packets one index at
    // a time over the same inputs (get_fec_encoded_pkt for ik = k .. n-1, network/NetFecCodec.cpp:
    // 133-166, network/FecCodecBuf.cpp:137-156).  The first such call computes all n - k rows in
    // one request; the next ones are served from here when the src[] pointers, sz and every input
    // byte (kept as a host copy, compared in full) are unchanged.  Any difference recomputes.
    std::vector<uint32_t> enc_all;  // [n - k][k] perm tables of every parity row
    std::mutex grp_mu;              // held across a group's compute: one computation per group
    std::vector<unsigned char*> grp_src;
    int grp_sz = -1;
    std::vector<uint8_t> grp_in;    // k x sz: the inputs the rows were computed from
    std::vector<uint8_t> grp_out;   // (n - k) x sz
};
constexpr size_t kFecDecCacheMax = 4096;

// run `rows` (e x k coefficient rows) over k input packets of sz bytes -> e outputs.  in_dev /
// out_dev: whether in[0] / out[0] are device memory (-1: find out here)
int apply_rows(const std::vector<uint32_t>& tab, int k, int e, unsigned char* const* in, unsigned char* const* out,
               int sz, int in_dev = -1, int out_dev = -1, Overlap* ov = nullptr) {
    struct RunOnExit {  // the overlap work runs in every path, at the latest on the way out
        Overlap* o;
        ~RunOnExit() {
            if (o) o->run();
        }
    } run_on_exit{ov};
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    const bool dev = in_dev < 0 ? is_device_ptr(in[0]) : in_dev != 0;
    const size_t pitch = round_up((size_t)sz, 16);
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!dev && k * e <= kPcMaxCoef && g_percall_fast.load() && !(out_dev < 0 ? is_device_ptr(out[0]) : out_dev != 0)) {
        // the resident server (packets of up to 4 KiB)
        if (pitch <= (size_t)kPcMaxChunks * 16 && k <= 16 && k * e <= kPcSrvMaxCoef && g_percall_resident.load() &&
            pc_server_setup(*ctx) == QFEC_OK) {
            rc = pc_server_call(*ctx, tab, k, e, in, out, sz, pitch, ov);
            if (rc != kPcNotServed) return rc;
            // not served within percall_timeout_us: the launch path below serves it
        }
        // host packets: CPU staging into mapped pinned memory, one launch, one synchronise
        if ((rc = ensure_pc(*ctx, (size_t)(k + e) * pitch))) return rc;
        for (int c = 0; c < k; ++c) memcpy(ctx->h_pc + (size_t)c * pitch, in[c], (size_t)sz);
        PcArgs a;
        a.in = ctx->d_pc;
        a.out = ctx->d_pc + (size_t)k * pitch;
        a.pitch = (uint32_t)pitch;
        a.chunks = (uint32_t)(pitch / 16);
        a.k = (uint32_t)k;
        a.e = (uint32_t)e;
        for (int i = 0; i < k * e; ++i) memcpy(&a.tab[i * 5], &tab[(size_t)i * QFEC_TAB_STRIDE], 5 * sizeof(uint32_t));
        // one block: wait on the kernel's completion word (its outputs are visible in host
        // memory once it is stored), not on the runtime's completion signal
        const bool spin = a.chunks <= 256;
        a.done = spin ? ctx->d_pc_done : nullptr;
        a.seq = spin ? ++ctx->pc_seq : 0;
        if (spin && a.seq == 0) a.seq = ++ctx->pc_seq;  // 0 is the word's initial value
        hipError_t he = launch_percall(a, ctx->stream);
        bool seen = false;
        if (he == hipSuccess && spin) {
            const auto t0 = std::chrono::steady_clock::now();
            for (uint32_t it = 1;; ++it) {
                if (__atomic_load_n(ctx->h_pc_done, __ATOMIC_ACQUIRE) == a.seq) {
                    seen = true;
                    break;
                }
                __builtin_ia32_pause();
                // after 2 s the stream synchronise below reports what happened
                if ((it & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
            }
            // let the runtime retire finished launches now and then (nothing to wait for)
            if (seen && ++ctx->pc_unsynced >= 256) {
                ctx->pc_unsynced = 0;
                (void)hipStreamQuery(ctx->stream);
            }
        }
        if (he == hipSuccess && !seen) he = hipStreamSynchronize(ctx->stream);
        if (he != hipSuccess) return hip_fail(he, "per-call kernel");
        for (int j = 0; j < e; ++j) memcpy(out[j], ctx->h_pc + (size_t)(k + j) * pitch, (size_t)sz);
        return QFEC_OK;
    }
    if ((rc = ensure_small(*ctx, tab.size()))) return rc;
    const size_t ib = (size_t)k * pitch, ob = (size_t)e * pitch;
    if ((rc = ensure_stage(*ctx, ib + ob, ib + ob))) return rc;
    memcpy(ctx->h_small, tab.data(), tab.size() * 4);
    HIP_TRY(hipMemcpyAsync(ctx->d_small, ctx->h_small, tab.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    if ((rc = gather_rows(*ctx, in, (size_t)k, sz, pitch, ctx->d_stage, ctx->h_stage, dev))) return rc;
    qfec_code tmp;
    tmp.k = k;
    tmp.m = e;
    if ((rc = run_encode(*ctx, &tmp, ctx->d_small, e, ctx->d_stage, ctx->d_stage + ib, 1, sz, (long long)pitch,
                         ctx->stream)))
        return rc;
    return scatter_rows(*ctx, out, (size_t)e, sz, pitch, ctx->d_stage + ib, ctx->h_stage + ib,
                        out_dev < 0 ? is_device_ptr(out[0]) : out_dev != 0, nullptr);
}

std::once_flag g_fec_init_once;

}  // namespace

extern "C" {

void* fec_new(int k, int n) {
    std::call_once(g_fec_init_once, [] { (void)field(); });  // init_fec (fec.c:612-625), once
    if (k > 256 || n > 256 || k > n) {  // fec.c:664-668
        fprintf(stderr, "Invalid parameters k %d n %d GF_SIZE %d\n", k, n, 255);
        return nullptr;
    }
    std::vector<uint8_t> rows;
    if (!vandermonde_rows(k, n - k, rows)) {
        fprintf(stderr, "Invalid parameters k %d n %d GF_SIZE %d\n", k, n, 255);
        return nullptr;
    }
    fec_handle* h = new (std::nothrow) fec_handle();
    if (!h) {
        fprintf(stderr, "-- malloc failure allocating new_code\n");
        exit(1);  // my_malloc (fec.c:238-247)
    }
    h->k = k;
    h->n = n;
    h->full.assign((size_t)n * k, 0);
    for (int i = 0; i < k; ++i) h->full[(size_t)i * k + i] = 1;
    memcpy(h->full.data() + (size_t)k * k, rows.data(), rows.size());
    h->code = make_code(k, n - k, std::move(rows), 0);
    h->enc_tab.resize((size_t)n);
    return h;
}

void fec_free(void* p) {
    if (!p) {
        fprintf(stderr, "bad parameters to fec_free\n");  // fec.c:641-643
        return;
    }
    fec_handle* h = (fec_handle*)p;
    free_code(h->code);
    delete h;
}

qfec_code* qfec_fec_code(void* p) { return p ? ((fec_handle*)p)->code : nullptr; }

int qfec_fec_matrix(void* p, unsigned char* out_full) {
    if (!p || !out_full) return QFEC_EINVAL;
    fec_handle* h = (fec_handle*)p;
    memcpy(out_full, h->full.data(), h->full.size());
    return QFEC_OK;
}

void fec_encode(void* code, unsigned char** src, unsigned char* dst, int index, int sz) {
    fec_handle* h = (fec_handle*)code;
    if (!h) return;
    const int k = h->k;
    if (index >= 0 && index < k) {  // fec.c:723-724: a copy
        if (sz <= 0) return;
        if (is_device_ptr(src[index]) || is_device_ptr(dst)) {
            if (hipMemcpy(dst, src[index], (size_t)sz, hipMemcpyDefault) != hipSuccess)
                fprintf(stderr, "[qfec] fec_encode: copy failed\n");
        } else {
            memcpy(dst, src[index], (size_t)sz);
        }
        return;
    }
    if (index < 0 || index >= h->n) {  // fec.c:730-732
        fprintf(stderr, "Invalid index %d (max %d)\n", index, h->n - 1);
        return;
    }
    if (sz <= 0) return;
    const int m = h->n - k;
    if (g_percall_group.load() && m > 1 && k <= 16 && k * m <= kPcSrvMaxCoef &&
        round_up((size_t)sz, 16) <= (size_t)kPcMaxChunks * 16) {
        // the whole group at once (see fec_handle::grp_*); host packets only
        if (!is_device_ptr(dst) && !is_device_ptr(src[0])) {  // the kinds apply_rows checks
            std::lock_guard<std::mutex> gl(h->grp_mu);
            const size_t szz = (size_t)sz;
            bool hit = h->grp_sz == sz && std::equal(src, src + k, h->grp_src.begin());
            for (int i = 0; i < k && hit; ++i) hit = !memcmp(h->grp_in.data() + (size_t)i * szz, src[i], szz);
            if (!hit) {
                h->grp_sz = -1;
                h->grp_src.assign(src, src + k);
                h->grp_in.resize((size_t)k * szz);
                h->grp_out.resize((size_t)m * szz);
                {
                    std::lock_guard<std::mutex> lk(h->mu);
                    if (h->enc_all.empty()) {
                        h->enc_all.resize((size_t)m * k * QFEC_TAB_STRIDE);
                        for (int r = 0; r < m; ++r)
                            for (int i = 0; i < k; ++i)
                                perm_entry(h->full[(size_t)(k + r) * k + i], &h->enc_all[((size_t)r * k + i) * QFEC_TAB_STRIDE]);
                    }
                }
                unsigned char* outs[256];
                for (int r = 0; r < m; ++r) outs[r] = h->grp_out.data() + (size_t)r * szz;
                // the inputs are staged for the device from the caller's packets, and the host copy
                // that later calls compare against is taken while the device computes (the packets
                // are the caller's and unchanged for the duration of the call)
                struct Keep {
                    fec_handle* h;
                    unsigned char** src;
                    int k;
                    size_t sz;
                    static void copy(void* p) {
                        const Keep& q = *static_cast<const Keep*>(p);
                        for (int i = 0; i < q.k; ++i) memcpy(q.h->grp_in.data() + (size_t)i * q.sz, q.src[i], q.sz);
                    }
                } keep{h, src, k, szz};
                Overlap ov;
                ov.fn = &Keep::copy;
                ov.arg = &keep;
                const int rc = apply_rows(h->enc_all, k, m, src, outs, sz, 0, 0, &ov);  // host packets, host rows
                if (rc) {
                    fprintf(stderr, "[qfec] fec_encode: %s\n", qfec_last_error());
                    return;
                }
                h->grp_sz = sz;
                ++g_group_misses;
            } else {
                ++g_group_hits;
            }
            memcpy(dst, h->grp_out.data() + (size_t)(index - k) * szz, szz);
            return;
        }
    }
    const std::vector<uint32_t>* tab = nullptr;
    {
        std::lock_guard<std::mutex> lk(h->mu);
        std::vector<uint32_t>& t = h->enc_tab[(size_t)index];
        if (t.empty()) {
            t.resize((size_t)k * QFEC_TAB_STRIDE);
            for (int i = 0; i < k; ++i) perm_entry(h->full[(size_t)index * k + i], &t[(size_t)i * QFEC_TAB_STRIDE]);
        }
        tab = &t;  // never resized again: stable after the lock is released
    }
    unsigned char* outs[1] = {dst};
    int rc = apply_rows(*tab, k, 1, src, outs, sz);
    if (rc) fprintf(stderr, "[qfec] fec_encode: %s\n", qfec_last_error());
}

int fec_decode(void* code, unsigned char** pkt, int* index, int sz) {
    fec_handle* h = (fec_handle*)code;
    if (!h) return 1;
    const int k = h->k, n = h->n;
    // shuffle (fec.c:738-771): data packets move to the slot of their index
    for (int i = 0; i < k;) {
        const int c = index[i];
        if (c >= k || c == i) { ++i; continue; }
        if (c < 0) return 1;           // undefined in the reference; rejected
        if (index[c] == c) return 1;   // conflict
        std::swap(index[i], index[c]);
        std::swap(pkt[i], pkt[c]);
    }
    for (int r = 0; r < k; ++r)
        if (index[r] >= n) {
            fprintf(stderr, "decode: invalid index %d (max %d)\n", index[r], n - 1);
            return 1;
        }
    // the pattern's recovery rows, cached per shuffled index[]
    uint64_t key = 1469598103934665603ull;  // FNV-1a over the indices
    for (int r = 0; r < k; ++r) key = (key ^ (uint64_t)(uint32_t)index[r]) * 1099511628211ull;
    std::shared_ptr<const fec_handle::Dec> d;  // held for the call: a cache clear on another thread does not free it
    {
        std::lock_guard<std::mutex> lk(h->mu);
        auto it = h->dec.find(key);
        if (it != h->dec.end() && std::equal(index, index + k, it->second->idx.begin())) d = it->second;
    }
    if (!d) {
        // build_decode_matrix (fec.c:778-808)
        std::vector<uint8_t> dm((size_t)k * k, 0);
        for (int r = 0; r < k; ++r) {
            if (index[r] < k) dm[(size_t)r * k + r] = 1;
            else memcpy(&dm[(size_t)r * k], &h->full[(size_t)index[r] * k], (size_t)k);
        }
        if (!gf_invert(dm.data(), k)) {
            fprintf(stderr, "singular matrix\n");
            return 1;
        }
        auto fresh = std::make_shared<fec_handle::Dec>();
        fresh->idx.assign(index, index + k);
        // rows to recover: slots holding parity (fec.c:840-858)
        for (int r = 0; r < k; ++r)
            if (index[r] >= k) fresh->slots.push_back(r);
        const int e = (int)fresh->slots.size();
        fresh->tab.resize((size_t)e * k * QFEC_TAB_STRIDE);
        for (int j = 0; j < e; ++j)
            for (int c = 0; c < k; ++c)
                perm_entry(dm[(size_t)fresh->slots[j] * k + c], &fresh->tab[((size_t)j * k + c) * QFEC_TAB_STRIDE]);
        std::lock_guard<std::mutex> lk(h->mu);
        if (h->dec.size() >= kFecDecCacheMax) h->dec.clear();
        h->dec[key] = fresh;  // a hash collision replaces the older pattern
        d = std::move(fresh);
    }
    if (sz <= 0 || d->slots.empty()) return 0;
    const int e = (int)d->slots.size();
    unsigned char* outs[256];
    for (int j = 0; j < e; ++j) outs[j] = pkt[d->slots[j]];
    const int rc = apply_rows(d->tab, k, e, pkt, outs, sz);
    if (rc) {
        fprintf(stderr, "[qfec] fec_decode: %s\n", qfec_last_error());
        return 1;
    }
    return 0;
}

}  // extern "C"
