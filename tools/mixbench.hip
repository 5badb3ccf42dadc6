// mixbench.hip -- the encode kernel's HBM traffic shape (per group: 10 rows of 1 KiB read,
// 3 rows of 1 KiB written, XOR instead of GF so that VALU is no factor) under different
// wave -> group schedules, to find what the shape itself can reach on MI355X.
//   hipcc --offload-arch=gfx950 -O3 tools/mixbench.hip -o tools/_abl/mixbench && tools/_abl/mixbench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int K = 10, M = 3, B = 1024;

template <bool NTL>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if constexpr (NTL) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NTS>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
    if constexpr (NTS) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <bool NTL, bool NTS>
__device__ __forceinline__ void group(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t g, int lane) {
    const u32x4* s = reinterpret_cast<const u32x4*>(src + g * (K * B)) + lane;
    u32x4* d = reinterpret_cast<u32x4*>(dst + g * (M * B)) + lane;
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = ld<NTL>(s + i * (B / 16));
#pragma unroll
    for (int r = 0; r < M; ++r) {
        u32x4 a = x[r];
#pragma unroll
        for (int i = 0; i < K; ++i) a ^= (i == r ? u32x4{0, 0, 0, 0} : x[i]) + (uint32_t)r;
        st<NTS>(d + r * (B / 16), a);
    }
}

// MODE 0: wave w -> group w (the encode kernel's schedule)
// MODE 1: XCD-contiguous: workgroup b runs on XCD b % 8; remap so each XCD walks one
//         contiguous eighth of the groups
// MODE 2: two groups per wave, all 20 loads before any store
template <int MODE, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_mix(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t G) {
    const int lane = threadIdx.x & 63;
    uint32_t b = blockIdx.x;
    if (MODE == 1) {
        const uint32_t nb = gridDim.x, per = (nb + 7) / 8, x = b % 8, i = b / 8;
        b = x * per + i;  // logical block: XCD x covers [x * per, (x + 1) * per)
        if (b >= nb) return;
    }
    const uint64_t w = (uint64_t)b * 4 + (threadIdx.x >> 6);
    if (MODE == 2) {
        const uint64_t g0 = 2 * w;
        if (g0 >= G) return;
        if (g0 + 1 < G) {
            const u32x4* s0 = reinterpret_cast<const u32x4*>(src + g0 * (K * B)) + lane;
            u32x4 x[2 * K];
#pragma unroll
            for (int i = 0; i < 2 * K; ++i) x[i] = ld<NTL>(s0 + i * (B / 16));
            u32x4* d0 = reinterpret_cast<u32x4*>(dst + g0 * (M * B)) + lane;
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int r = 0; r < M; ++r) {
                    u32x4 a = x[h * K + r];
#pragma unroll
                    for (int i = 0; i < K; ++i) a ^= (i == r ? u32x4{0, 0, 0, 0} : x[h * K + i]) + (uint32_t)r;
                    st<NTS>(d0 + (h * M + r) * (B / 16), a);
                }
        } else {
            group<NTL, NTS>(src, dst, g0, lane);
        }
        return;
    }
    if (w >= G) return;
    group<NTL, NTS>(src, dst, w, lane);
}

template <int MODE, bool NTL, bool NTS>
int run(const char* name, const uint8_t* src, uint8_t* dst, uint64_t G, hipEvent_t a, hipEvent_t b) {
    const uint64_t waves = MODE == 2 ? (G + 1) / 2 : G;
    const unsigned grid = (unsigned)((waves + 3) / 4);
    for (int w = 0; w < 5; ++w) k_mix<MODE, NTL, NTS><<<grid, 256>>>(src, dst, G);
    float best = 1e9, sum = 0;
    for (int r = 0; r < 20; ++r) {
        CHECK(hipEventRecord(a, 0));
        k_mix<MODE, NTL, NTS><<<grid, 256>>>(src, dst, G);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
        sum += ms;
    }
    const double bytes = (double)G * (K + M) * B;
    printf("%-44s avg %7.1f us %7.1f GB/s   best %7.1f us %7.1f GB/s\n", name, sum / 20 * 1e3,
           bytes / (sum / 20 * 1e-3) / 1e9, best * 1e3, bytes / (best * 1e-3) / 1e9);
    return 0;
}

int main() {
    const uint64_t G = 100000;
    uint8_t *src, *dst;
    CHECK(hipMalloc(&src, G * K * B));
    CHECK(hipMalloc(&dst, G * M * B));
    CHECK(hipMemset(src, 3, G * K * B));
    CHECK(hipMemset(dst, 0, G * M * B));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int round = 0; round < 2; ++round) {
        printf("-- round %d: RS(10,3)-shaped XOR, 100000 groups x 13 KiB\n", round);
        run<0, true, true>("wave per group, nt loads, nt stores", src, dst, G, a, b);
        run<0, false, true>("wave per group, plain loads, nt stores", src, dst, G, a, b);
        run<0, true, false>("wave per group, nt loads, plain stores", src, dst, G, a, b);
        run<0, false, false>("wave per group, plain loads, plain stores", src, dst, G, a, b);
        run<1, true, true>("XCD-contiguous, nt / nt", src, dst, G, a, b);
        run<2, true, true>("two groups per wave, nt / nt", src, dst, G, a, b);
    }
    return 0;
}
