// qfec_fec_abi.cpp -- system/fec.h on the GPU: fec_new / fec_free / fec_encode / fec_decode
// (system/fec.h:237-241, module/fec.c:612-862), served per packet by the resident per-call server
// (qfec_percall.hpp) or a per-call launch; qfec_fec_code / qfec_fec_matrix expose the handle's code.
#include "qfec_rt.hpp"

using namespace qfec;

namespace qfec {

// ---- the resident per-call server (qfec_percall.hpp)
std::atomic<int> g_percall_resident{1};  // qfec_tune "percall_resident"
std::atomic<int> g_percall_idle_us{(int)kPcIdleUsDefault};  // qfec_tune "percall_idle_us": the block's idle exit
std::atomic<int> g_percall_timeout_us{2000000};  // qfec_tune "percall_timeout_us": give up spinning, wait instead
std::atomic<int> g_percall_fault{0};     // qfec_tune "percall_fault" (tests): 1 = requests are never handed to a server
std::atomic<int> g_percall_group{1};     // qfec_tune "percall_group": fec_encode computes a group's m rows at once
std::atomic<int> g_percall_stop_us{2000000};  // qfec_tune "percall_stop_us": the bounded wait for a stopped server
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

// stop the server and wait for it (a few microseconds: it polls `stop`); limit_us >= 0: wait at
// most that long, hipErrorNotReady if the block has not exited by then (it is still queued or
// running, `stop` stays set, the caller abandons it)
hipError_t pc_server_stop(DevCtx& c, long long limit_us) {
    DevCtx::PcServer& s = c.srv;
    if (s.usable <= 0 || !s.launched) return hipSuccess;
    __atomic_store_n(&s.bell->stop, 1u, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    hipError_t e;
    if (limit_us < 0) {
        e = hipStreamSynchronize(s.stream);
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        while ((e = hipStreamQuery(s.stream)) == hipErrorNotReady &&
               std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(limit_us))
            __builtin_ia32_pause();
        if (e == hipErrorNotReady) {
            (void)hipGetLastError();
            return hipErrorNotReady;
        }
    }
    __atomic_store_n(&s.bell->stop, 0u, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    s.launched = false;
    return e;
}

// give up on a server that did not exit within percall_stop_us after `stop`: its block may still
// run one day and write its own buffers, so they stay allocated (leaked) and are never touched
// again; the device takes the one-launch path until percall_resident is set to 1 again
void pc_server_abandon(DevCtx& c) {
    DevCtx::PcServer& s = c.srv;
    s.usable = -2;
    s.launched = false;
    s.stream = nullptr;
    s.bell = nullptr;
    s.in = s.h_out = s.d_out = nullptr;
    s.h_st = s.d_st = nullptr;
    s.tab_bytes = 0;
    ++s.abandoned;
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
            // handed back to the caller, which launches it on its own.  That wait is bounded by
            // percall_stop_us: a block still not done then is abandoned and the request fails
            // (fec_encode leaves dst as it was, fec_decode returns 1)
            ++s.timeouts;
            hipError_t se = pc_server_stop(c, (long long)g_percall_stop_us.load());
            if (g_percall_fault.load() == 2 && se == hipSuccess) se = hipErrorNotReady;  // test hook
            if (se == hipErrorNotReady) {
                pc_server_abandon(c);
                set_error("per-call server: not served within percall_timeout_us and not stopped within "
                          "percall_stop_us (%d us); request abandoned", g_percall_stop_us.load());
                return QFEC_EHIP;
            }
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

}  // namespace qfec

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
