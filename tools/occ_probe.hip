// occ_probe.hip -- does the streaming rate of a k-rows-in, m-rows-out shape depend on how many
// waves each CU holds?  One wave per group, lane = 16-B column of 1 KiB rows (the encode's map),
// XOR only; residency capped by a dynamic LDS allocation per one-wave block (160 KiB per CU:
// 40 KiB -> 4 waves per CU, 27 -> 5, 20 -> 8, 14 -> 11, 10 -> 16, 0 -> as many as the registers
// allow).
//   hipcc --offload-arch=gfx950 -O3 tools/occ_probe.hip -o tools/_abl/occ_probe && tools/_abl/occ_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <string>
#include <vector>

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int B = 1024;

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int K, int M, bool NT>
__global__ void __launch_bounds__(64) k_occ(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t G) {
    extern __shared__ uint32_t pad[];
    const uint64_t g = blockIdx.x;
    if (g >= G) return;
    const int lane = threadIdx.x;
    const u32x4* s = reinterpret_cast<const u32x4*>(src + g * (uint64_t)(K * B)) + lane;
    u32x4* d = reinterpret_cast<u32x4*>(dst + g * (uint64_t)(M * B)) + lane;
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = ld<NT>(s + i * (B / 16));
    u32x4 a = x[0];
#pragma unroll
    for (int i = 1; i < K; ++i) a ^= x[i];
#pragma unroll
    for (int r = 0; r < M; ++r) st<NT>(d + r * (B / 16), (r < K ? x[r] : a) ^ a);
    if (G == 0) pad[lane] = a.x;  // never true: keeps the allocation referenced
}

template <int K, int M, bool NT>
static int run(uint8_t* src, uint8_t* dst, double bytes) {
    const uint64_t G = (uint64_t)(bytes / ((K + M) * B));
    const int ldsk[] = {0, 10, 14, 20, 27, 40};
    for (int l : ldsk) {
        const size_t lds = (size_t)l * 1024;
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_occ<K, M, NT>), dim3((unsigned)G), dim3(64), lds, 0, src, dst, G);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        std::vector<float> t;
        for (int rep = 0; rep < 5; ++rep) {
            CHECK(hipEventRecord(e0, 0));
            for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((k_occ<K, M, NT>), dim3((unsigned)G), dim3(64), lds, 0, src, dst, G);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms / 10);
        }
        std::sort(t.begin(), t.end());
        const double ms = t[2];
        printf("%2d:%-2d %s lds %2d KiB (%s waves/CU)  %.1f us  %.0f GB/s\n", K, M, NT ? "nt   " : "plain", l,
               l ? std::to_string(160 / l).c_str() : "max", ms * 1e3, (double)G * (K + M) * B / ms / 1e6);
        fflush(stdout);
        CHECK(hipEventDestroy(e0));
        CHECK(hipEventDestroy(e1));
    }
    return 0;
}

int main() {
    const double bytes = 1.3e9;
    uint8_t *src, *dst;
    CHECK(hipMalloc(&src, (size_t)bytes));
    CHECK(hipMalloc(&dst, (size_t)bytes));
    CHECK(hipMemset(src, 0x5A, (size_t)bytes));
    CHECK(hipMemset(dst, 0, (size_t)bytes));
    if (run<10, 3, true>(src, dst, bytes)) return 1;
    if (run<10, 3, false>(src, dst, bytes)) return 1;
    if (run<10, 10, true>(src, dst, bytes)) return 1;
    if (run<1, 1, true>(src, dst, bytes)) return 1;
    if (run<1, 1, false>(src, dst, bytes)) return 1;
    CHECK(hipFree(src));
    CHECK(hipFree(dst));
    return 0;
}
