// tools/launch_lat.hip -- where a per-call launch's time goes on this box (measurement only).
// Variants, each timed over N back-to-back calls from one host thread:
//   sync      empty kernel, hipStreamSynchronize
//   spin      empty kernel that stores a sequence word into coherent pinned memory; host spins
//   spin_rd   one block reads k rows of mapped pinned memory (like k_percall), writes 3 rows
//             back, then stores the word
//   spin_big  spin with a 3.2 KB kernel argument block (k_percall's table size)
//   d_spin    spin_rd but the rows are in device memory (no PCIe reads by the kernel)
// build: hipcc --offload-arch=gfx950 -O3 -o tools/launch_lat tools/launch_lat.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Big { uint32_t t[800]; };

__global__ void k_empty() {}
__global__ void k_flag(uint32_t* done, uint32_t seq) {
    if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_flag_big(uint32_t* done, uint32_t seq, Big b) {
    if (threadIdx.x == 0) __hip_atomic_store(done, seq + (b.t[799] & 0), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_rows(const uint8_t* in, uint8_t* out, int k, int chunks, uint32_t* done, uint32_t seq) {
    const int c = threadIdx.x;
    if (c < chunks) {
        uint4 acc = make_uint4(0, 0, 0, 0);
        for (int i = 0; i < k; ++i) {
            const uint4 x = reinterpret_cast<const uint4*>(in + (size_t)i * chunks * 16)[c];
            acc.x ^= x.x; acc.y ^= x.y; acc.z ^= x.z; acc.w ^= x.w;
        }
        for (int j = 0; j < 3; ++j) reinterpret_cast<uint4*>(out + (size_t)j * chunks * 16)[c] = acc;
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static void spin(volatile uint32_t* w, uint32_t seq) {
    while (__atomic_load_n(w, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
}

int main() {
    const int N = 4000, k = 10, chunks = 65;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *hw, *dw;
    CK(hipHostMalloc((void**)&hw, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&dw, hw, 0));
    *hw = 0;
    uint8_t *hp, *dp, *dd;
    CK(hipHostMalloc((void**)&hp, 1 << 16, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void**)&dp, hp, 0));
    CK(hipMalloc((void**)&dd, 1 << 16));
    memset(hp, 1, 1 << 16);
    Big b;
    memset(&b, 0, sizeof(b));
    uint32_t seq = 0;
    for (int rep = 0; rep < 3; ++rep) {
        double t0 = now_us();
        for (int i = 0; i < N; ++i) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); CK(hipStreamSynchronize(s)); }
        const double t_sync = (now_us() - t0) / N;
        t0 = now_us();
        for (int i = 0; i < N; ++i) { ++seq; hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, dw, seq); spin(hw, seq); }
        const double t_spin = (now_us() - t0) / N;
        t0 = now_us();
        double t_launch = 0;
        for (int i = 0; i < N; ++i) {
            ++seq;
            const double a = now_us();
            hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, dw, seq);
            t_launch += now_us() - a;
            spin(hw, seq);
        }
        t_launch /= N;
        t0 = now_us();
        for (int i = 0; i < N; ++i) { ++seq; hipLaunchKernelGGL(k_flag_big, dim3(1), dim3(64), 0, s, dw, seq, b); spin(hw, seq); }
        const double t_big = (now_us() - t0) / N;
        t0 = now_us();
        for (int i = 0; i < N; ++i) { ++seq; hipLaunchKernelGGL(k_rows, dim3(1), dim3(128), 0, s, dp, dp + 32768, k, chunks, dw, seq); spin(hw, seq); }
        const double t_rd = (now_us() - t0) / N;
        t0 = now_us();
        for (int i = 0; i < N; ++i) { ++seq; hipLaunchKernelGGL(k_rows, dim3(1), dim3(128), 0, s, dd, dd + 32768, k, chunks, dw, seq); spin(hw, seq); }
        const double t_drd = (now_us() - t0) / N;
        CK(hipStreamSynchronize(s));
        printf("rep %d: sync %.2f us | spin %.2f us (launch call %.2f) | spin_big %.2f | spin_rd %.2f | d_spin %.2f\n", rep, t_sync,
               t_spin, t_launch, t_big, t_rd, t_drd);
    }
    return 0;
}
