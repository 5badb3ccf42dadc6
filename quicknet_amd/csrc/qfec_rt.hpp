// qfec_rt.hpp -- internals shared by the host runtime's translation units:
//   qfec_runtime.cpp   errors, device contexts, code objects and their device tables, the batched
//                      device API (qfec_*), knobs, calibration probes, row staging
//   qfec_fec_abi.cpp   system/fec.h (fec_new / fec_encode / fec_decode) and the resident per-call
//                      server behind it
//   qfec_rs_abi.cpp    module/rs.h (reed_solomon_*) with its host-pointer pipelines and the
//                      classification of caller shard pointers
//   qfec_pipe.cpp      qfec_pipe_* (host batches streamed over several streams and devices)
//   qfec_wire_api.cpp  the datagram / framing entry points (qfec_pack_*, qfec_unpack_*, ...)
#pragma once

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
#include <unordered_set>
#include <vector>

#include "../../include/qfec.h"
#include "../../include/qfec_fec.h"
#include "../../include/qfec_rs.h"
#include "qfec_internal.hpp"
#include "qfec_maps.hpp"
#include "qfec_percall.hpp"
#include "qfec_pool.hpp"

namespace qfec {

// ---- errors (qfec_runtime.cpp): the thread's last error text, qfec_last_error()
extern thread_local std::string t_last_error;
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
int hip_fail(hipError_t e, const char* what);  // sets the error text, returns QFEC_EHIP

#define HIP_TRY(expr)                                       \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return hip_fail(_e, #expr);   \
    } while (0)

inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- settings (qfec_tune keys outside Tuning; qfec_runtime.cpp / qfec_fec_abi.cpp)
extern std::atomic<int> g_variant;
extern std::atomic<int> g_percall_fast, g_percall_resident, g_percall_idle_us, g_percall_timeout_us,
    g_percall_fault, g_percall_group, g_percall_stop_us;
extern std::atomic<unsigned long long> g_group_hits, g_group_misses;

// ---- device contexts (qfec_runtime.cpp)
constexpr int kMaxDevices = 64;
constexpr int kMaxHostLanes = 8;  // host-buffer chunk slots per device context

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
        int usable = 0;              // 0 not tried, 1 ready, -1 unavailable on this device, -2 abandoned
                                     // (did not stop within percall_stop_us; percall_resident 1 retries)
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
        unsigned long long calls = 0, launches = 0, relaunches = 0, timeouts = 0, abandoned = 0;
        // QFEC_PERCALL_TRACE sums: loads, compute, fence (shader clocks), host wait (ns), n, clocks and
        // wall ticks over the traced span (the clock calibration)
        unsigned long long tr[7] = {0, 0, 0, 0, 0, 0, 0};
    } srv;
    int init_rc = QFEC_ENODEV;
    // host-buffer chunk slots, each with its own stream, event, device buffers and pinned staging
    // (created on first use): qfec_encode_host / qfec_reconstruct_host alternate host[0] and host[1];
    // module/rs.h's host-pointer pipelines take the first tuning "host_lanes" of them
    struct HostSlot {
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
        uint8_t* d_buf = nullptr;  // data chunk | parity chunk
        uint8_t* h_in = nullptr;   // pinned
        uint8_t* h_out = nullptr;  // pinned
        size_t in_cap = 0, out_cap = 0;
    } host[kMaxHostLanes];
    std::mutex host_mu;
};

extern DevCtx g_ctx[kMaxDevices];

int current_ctx(DevCtx** out);  // the calling thread's current device (created on first use)
int ensure_stage(DevCtx& c, size_t dbytes, size_t hbytes);
int ensure_pc(DevCtx& c, size_t bytes);
int ensure_small(DevCtx& c, size_t words);
bool is_device_ptr(const void* p);
bool is_pinned_host(const void* p);
bool host_dev(const void* h, uint8_t** d);
int ensure_host_slot(DevCtx::HostSlot& h, size_t in_bytes, size_t out_bytes);
void quiesce_host_slots(DevCtx& c);
// rows of caller memory to / from a device staging area (qfec_runtime.cpp)
int gather_rows(DevCtx& c, unsigned char* const* ptrs, size_t count, int len, size_t pitch, uint8_t* d_dst,
                uint8_t* h_tmp, bool dev_src);
int scatter_rows(DevCtx& c, unsigned char* const* ptrs, size_t count, int len, size_t pitch, const uint8_t* d_src,
                 uint8_t* h_tmp, bool dev_dst, const uint8_t* only);

// ---- the resident per-call server (qfec_fec_abi.cpp)
bool pc_server_alive(const DevCtx::PcServer& s);
hipError_t pc_server_stop(DevCtx& c, long long limit_us = -1);  // limit_us >= 0: bounded wait

}  // namespace qfec

// ---- code objects (qfec_runtime.cpp); qfec_code is the C ABI's opaque type
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
    std::shared_ptr<const std::vector<uint8_t>> lut_seed;  // replaced whole on a rebuild; readers keep a reference
    uint64_t lut_seed_version = ~0ull;
};

namespace qfec {

qfec_code* make_code(int k, int m, std::vector<uint8_t>&& rows, int quirk);
void free_code(qfec_code* c);
const uint8_t* full_of(const qfec_code* c);  // module/rs.c's rs->m, or nullptr
int ensure_enc(qfec_code* c, int dev, uint32_t** out);    // caller holds c->mu
int ensure_lut(qfec_code* c, int dev, DevTables** out);   // caller holds c->mu
bool vec16_ok(const void* a, const void* b, int block, long long pitch);
int run_encode(DevCtx& ctx, const qfec_code* c, const uint32_t* tab, int m, const uint8_t* d_data, uint8_t* d_par,
               long long groups, int block, long long pitch, hipStream_t s, long long dgs = -1, long long pgs = -1,
               bool host_mem = false);
int run_reconstruct(DevCtx& ctx, const qfec_code* c, const int32_t* lut, const int32_t* group_rec,
                    const uint32_t* recs, uint8_t* d_data, const uint8_t* d_par, const uint8_t* d_marks,
                    long long groups, int block, long long pitch, unsigned* d_failed, hipStream_t s,
                    long long dgs = -1, long long pgs = -1);
int host_records(qfec_code* c, const uint8_t* marks, long long groups, std::vector<int32_t>& grec,
                 std::vector<uint32_t>& recs, long long* nfail);
int reconstruct_host_records(DevCtx& ctx, qfec_code* c, uint8_t* d_data, const uint8_t* d_par,
                             const uint8_t* d_marks, long long groups, int block_size, long long pitch,
                             unsigned* d_failed, hipStream_t s);

}  // namespace qfec
