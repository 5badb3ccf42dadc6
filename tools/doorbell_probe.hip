// tools/doorbell_probe.hip -- latency probe for the per-packet ABI (measurement aid, not the
// product).  Where does a fec_encode-sized call (k = 10 input rows of 1 KiB in, one row out,
// host buffers on both sides) spend its time, and how low can it go?
//   A  launch per call, inputs in pinned host memory (the current per-call path's shape)
//   B  launch per call, inputs written by the CPU into device memory (fine-grained, host-mapped)
//   C  a resident kernel that polls a doorbell word in device memory (the CPU writes the inputs
//      and the doorbell there; the kernel writes the output and a completion word into pinned
//      host memory, the CPU spins on it).  The kernel exits by itself after 2 ms without a
//      request, or at once when the stop word is set; the host waits for it before exiting.
// Prints microseconds per call (median of 2000) for each.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                          \
        }                                                                      \
    } while (0)

constexpr int K = 10, ROW = 1024, CH = ROW / 16;

struct Bell {             // in device memory (CPU-written)
    uint32_t req;         // request sequence number
    uint32_t stop;        // 1: exit now
    uint32_t pad[62];
};

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one block of 64 lanes: lane = one 16-B column of the k rows
__device__ __forceinline__ void xor_rows(const uint8_t* in, uint8_t* out, int lane) {
    uint4 acc = make_uint4(0, 0, 0, 0), x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = *reinterpret_cast<const uint4*>(in + c * ROW + lane * 16);
#pragma unroll
    for (int c = 0; c < K; ++c) {
        acc.x ^= x[c].x;
        acc.y ^= x[c].y;
        acc.z ^= x[c].z;
        acc.w ^= x[c].w;
    }
    *reinterpret_cast<uint4*>(out + lane * 16) = acc;
}

__global__ void k_once(const uint8_t* in, uint8_t* out, uint32_t* done, uint32_t seq) {
    xor_rows(in, out, threadIdx.x);
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_resident(Bell* bell, const uint8_t* in, uint8_t* out, uint32_t* done, uint32_t served0,
                           uint64_t idle_ticks) {
    __shared__ uint32_t s_req, s_quit;
    uint32_t served = served0;
    uint64_t t0 = wall_clock64();
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t r;
            for (;;) {
                r = ld_sys(&bell->req);
                if (r != served || ld_sys(&bell->stop) || wall_clock64() - t0 > idle_ticks) break;
                __builtin_amdgcn_s_sleep(1);
            }
            s_req = r;
            s_quit = r == served;
        }
        __syncthreads();
        if (s_quit) break;
        const uint32_t r = s_req;
        xor_rows(in, out, threadIdx.x);
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(done, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        served = r;
        t0 = wall_clock64();
        __syncthreads();
    }
}

static double median(std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const int N = 2000;
    std::vector<uint8_t> src(K * ROW), dst(ROW);
    for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 7 + 3);
    uint8_t *h_in, *h_out;
    uint32_t* h_done;
    CK(hipHostMalloc((void**)&h_in, K * ROW, hipHostMallocMapped));
    CK(hipHostMalloc((void**)&h_out, ROW, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc((void**)&h_done, 64, hipHostMallocMapped | hipHostMallocCoherent));
    *h_done = 0;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t seq = 0;
    auto spin = [&](uint32_t want) {
        const auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(h_done, __ATOMIC_ACQUIRE) != want) {
            __builtin_ia32_pause();
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) return false;
        }
        return true;
    };
    // ---- A: pinned host inputs, launch per call
    {
        std::vector<double> t;
        for (int i = 0; i < N; ++i) {
            const auto a = std::chrono::steady_clock::now();
            memcpy(h_in, src.data(), src.size());
            hipLaunchKernelGGL(k_once, dim3(1), dim3(64), 0, s, h_in, h_out, h_done, ++seq);
            if (!spin(seq)) { fprintf(stderr, "A: timeout\n"); return 1; }
            memcpy(dst.data(), h_out, ROW);
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
        }
        CK(hipStreamSynchronize(s));
        printf("A launch per call, inputs in pinned host memory:            %6.2f us\n", median(t));
    }
    // ---- device memory the CPU can write: fine-grained device allocation
    uint8_t* d_in = nullptr;
    Bell* bell = nullptr;
    CK(hipExtMallocWithFlags((void**)&d_in, K * ROW, hipDeviceMallocFinegrained));
    CK(hipExtMallocWithFlags((void**)&bell, sizeof(Bell), hipDeviceMallocFinegrained));
    hipPointerAttribute_t attr;
    CK(hipPointerGetAttributes(&attr, d_in));
    printf("fine-grained device memory: device %p host %p type %d\n", attr.devicePointer, attr.hostPointer,
           (int)attr.type);
    fflush(stdout);
    // the CPU writes into it (a large-BAR mapping); if that is not possible this faults here
    memset(d_in, 0, K * ROW);
    memset(bell, 0, sizeof(Bell));
    printf("host writes into device memory: ok\n");
    fflush(stdout);
    {
        std::vector<double> t;
        for (int i = 0; i < N; ++i) {
            const auto a = std::chrono::steady_clock::now();
            memcpy(d_in, src.data(), src.size());
            hipLaunchKernelGGL(k_once, dim3(1), dim3(64), 0, s, d_in, h_out, h_done, ++seq);
            if (!spin(seq)) { fprintf(stderr, "B: timeout\n"); return 1; }
            memcpy(dst.data(), h_out, ROW);
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
        }
        CK(hipStreamSynchronize(s));
        printf("B launch per call, inputs written into device memory:       %6.2f us\n", median(t));
    }
    // ---- C: resident kernel on a doorbell
    {
        hipStream_t rs;
        CK(hipStreamCreateWithFlags(&rs, hipStreamNonBlocking));
        const uint64_t idle = 200000;  // 2 ms at the 100 MHz wall clock
        uint32_t served = seq;
        __atomic_store_n(&bell->req, served, __ATOMIC_RELEASE);
        hipLaunchKernelGGL(k_resident, dim3(1), dim3(64), 0, rs, bell, d_in, h_out, h_done, served, idle);
        std::vector<double> t;
        int lost = 0;
        for (int i = 0; i < N; ++i) {
            const auto a = std::chrono::steady_clock::now();
            memcpy(d_in, src.data(), src.size());
            ++seq;
            __atomic_store_n(&bell->req, seq, __ATOMIC_RELEASE);
            if (!spin(seq)) {
                ++lost;
                break;
            }
            memcpy(dst.data(), h_out, ROW);
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
        }
        if (lost || t.empty()) {
            __atomic_store_n(&bell->stop, 1u, __ATOMIC_RELEASE);
            CK(hipStreamSynchronize(rs));
            printf("C resident kernel: a request was not answered within 2 s\n");
            return 1;
        }
        printf("C resident kernel on a doorbell in device memory:           %6.2f us\n", median(t));
        // C2: the same with fresh input bytes every call (one byte of every row changes), each
        // output checked: stale cached input lines would show up here
        t.clear();
        int wrong = 0;
        std::vector<uint8_t> ref(ROW);
        for (int i = 0; i < N && !lost; ++i) {
            for (int c = 0; c < K; ++c) src[c * ROW + (i * 67 + c) % ROW] ^= (uint8_t)(1 + i);
            const auto a = std::chrono::steady_clock::now();
            memcpy(d_in, src.data(), src.size());
            ++seq;
            __atomic_store_n(&bell->req, seq, __ATOMIC_RELEASE);
            if (!spin(seq)) {
                ++lost;
                break;
            }
            memcpy(dst.data(), h_out, ROW);
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
            memset(ref.data(), 0, ROW);
            for (int c = 0; c < K; ++c)
                for (int b2 = 0; b2 < ROW; ++b2) ref[b2] ^= src[c * ROW + b2];
            wrong += memcmp(ref.data(), dst.data(), ROW) != 0;
        }
        __atomic_store_n(&bell->stop, 1u, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(rs));
        if (!t.empty())
            printf("C2 the same, fresh inputs every call:                         %6.2f us  (%d of %zu outputs wrong)\n",
                   median(t), wrong, t.size());
        else
            printf("C2: a request was not answered within 2 s\n");
        // after an idle gap the kernel has exited by itself: a new launch then serves the request
        CK(hipStreamDestroy(rs));
    }
    uint8_t ref[ROW];
    memset(ref, 0, ROW);
    for (int c = 0; c < K; ++c)
        for (int b = 0; b < ROW; ++b) ref[b] ^= src[c * ROW + b];
    printf("output correct: %s\n", memcmp(ref, dst.data(), ROW) == 0 ? "yes" : "NO");
    CK(hipFree(d_in));
    CK(hipFree(bell));
    CK(hipStreamDestroy(s));
    return 0;
}
