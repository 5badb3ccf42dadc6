// membench.hip -- HBM streaming calibration for the RS encode traffic shape on MI355X.
//
// Measures what the memory system delivers for "read k rows of a group, write m rows"
// (RS(10,3), 1 KiB rows, 100 000 groups = 1.33 GB algorithmic) under several access
// forms, plus plain copy / read-only / write-only streams.  Informs the kernel design in
// quicknet_amd/csrc/qfec_kernels.hip; not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/build/membench tools/membench.hip && tools/build/membench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int NT_LD, int NT_ST>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if (NT_LD) return __builtin_nontemporal_load(p);
    return *p;
}
template <int NT_ST>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
    if (NT_ST) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// one lane per 16-B column; K rows in, M rows out, XOR only
template <int K, int M, int NT_LD, int NT_ST, int COLS_PER_LANE>
__global__ void __launch_bounds__(256) k_shape(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                               uint64_t groups, uint32_t cols, uint64_t pitch) {
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t lanes_per_group = cols / COLS_PER_LANE;
    const uint64_t g = t / lanes_per_group;
    if (g >= groups) return;
    const uint32_t l = (uint32_t)(t - g * lanes_per_group);
#pragma unroll
    for (int q = 0; q < COLS_PER_LANE; ++q) {
        const uint32_t col = l + q * (uint32_t)lanes_per_group;
        const u32x4* src = (const u32x4*)(data + g * K * pitch + col * 16u);
        u32x4* dst = (u32x4*)(par + g * M * pitch + col * 16u);
        u32x4 x[K];
#pragma unroll
        for (int c = 0; c < K; ++c) x[c] = ld<NT_LD, NT_ST>(src + c * (pitch / 16));
        u32x4 acc = x[0];
#pragma unroll
        for (int c = 1; c < K; ++c) acc ^= x[c];
#pragma unroll
        for (int r = 0; r < M; ++r) {
            st<NT_ST>(dst + r * (pitch / 16), acc);
            acc.x += 1;
        }
    }
}

// grid-stride persistent version
template <int K, int M, int NT_LD>
__global__ void __launch_bounds__(256) k_shape_gs(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                                  uint64_t groups, uint32_t cols, uint64_t pitch) {
    const uint64_t total = groups * cols;
    for (uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x; t < total; t += (uint64_t)gridDim.x * 256u) {
        const uint64_t g = t / cols;
        const uint32_t col = (uint32_t)(t - g * cols);
        const u32x4* src = (const u32x4*)(data + g * K * pitch + col * 16u);
        u32x4* dst = (u32x4*)(par + g * M * pitch + col * 16u);
        u32x4 x[K];
#pragma unroll
        for (int c = 0; c < K; ++c) x[c] = ld<NT_LD, 0>(src + c * (pitch / 16));
        u32x4 acc = x[0];
#pragma unroll
        for (int c = 1; c < K; ++c) acc ^= x[c];
#pragma unroll
        for (int r = 0; r < M; ++r) {
            dst[r * (pitch / 16)] = acc;
            acc.x += 1;
        }
    }
}

__global__ void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) b[i] = a[i];
}
__global__ void k_copy1(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i < n) b[i] = a[i];
}
__global__ void k_read(const u32x4* __restrict__ a, uint64_t n, unsigned* out) {
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u)
        acc ^= __builtin_nontemporal_load(a + i);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}
__global__ void k_write(u32x4* __restrict__ b, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u)
        b[i] = (u32x4){(unsigned)i, 1, 2, 3};
}
__global__ void k_write_nt(u32x4* __restrict__ b, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u)
        __builtin_nontemporal_store((u32x4){(unsigned)i, 1, 2, 3}, b + i);
}
__global__ void k_copy_nt(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
}

template <typename F>
static double time_ms(F f, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) f();
    CHECK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) f();
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const uint64_t G = 100000, K = 10, M = 3, B = 1024;
    const uint64_t dbytes = G * K * B, pbytes = G * M * B, alg = dbytes + pbytes;
    uint8_t *d, *p;
    unsigned* flag;
    CHECK(hipMalloc(&d, dbytes));
    CHECK(hipMalloc(&p, pbytes * 4));
    CHECK(hipMalloc(&flag, 4));
    CHECK(hipMemset(d, 1, dbytes));
    const uint32_t cols = B / 16;
    const unsigned grid1 = (unsigned)((G * cols + 255) / 256);
    auto rep = [&](const char* name, double ms, double bytes) {
        printf("%-44s %8.1f us  %7.1f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    };
    const int R = 20;
    rep("shape nt-ld plain-st 1col/lane", time_ms([&] { k_shape<10, 3, 1, 0, 1><<<grid1, 256>>>(d, p, G, cols, B); }, R), alg);
    rep("shape plain-ld plain-st", time_ms([&] { k_shape<10, 3, 0, 0, 1><<<grid1, 256>>>(d, p, G, cols, B); }, R), alg);
    rep("shape nt-ld nt-st", time_ms([&] { k_shape<10, 3, 1, 1, 1><<<grid1, 256>>>(d, p, G, cols, B); }, R), alg);
    rep("shape plain-ld nt-st", time_ms([&] { k_shape<10, 3, 0, 1, 1><<<grid1, 256>>>(d, p, G, cols, B); }, R), alg);
    rep("shape nt-ld 2col/lane", time_ms([&] { k_shape<10, 3, 1, 0, 2><<<grid1 / 2, 256>>>(d, p, G, cols, B); }, R), alg);
    rep("shape nt-ld 4col/lane", time_ms([&] { k_shape<10, 3, 1, 0, 4><<<grid1 / 4, 256>>>(d, p, G, cols, B); }, R), alg);
    for (unsigned gs : {1024u, 2048u, 4096u, 8192u})
    {
        char nm[64];
        snprintf(nm, sizeof nm, "shape grid-stride nt-ld grid=%u", gs);
        rep(nm, time_ms([&] { k_shape_gs<10, 3, 1><<<gs, 256>>>(d, p, G, cols, B); }, R), alg);
    }
    const uint64_t n16 = dbytes / 16 / 2;  // copy half of data region into parity x4 space
    rep("copy 512MB grid-stride 4096", time_ms([&] { k_copy<<<4096, 256>>>((const u32x4*)d, (u32x4*)p, n16 / 1); }, R), 2.0 * n16 * 16);
    rep("copy 512MB 1 elem/thread", time_ms([&] { k_copy1<<<(unsigned)((n16 + 255) / 256), 256>>>((const u32x4*)d, (u32x4*)p, n16); }, R), 2.0 * n16 * 16);
    rep("read-only 1GB nt grid 4096", time_ms([&] { k_read<<<4096, 256>>>((const u32x4*)d, dbytes / 16, flag); }, R), (double)dbytes);
    rep("read-only 1GB nt grid 16384", time_ms([&] { k_read<<<16384, 256>>>((const u32x4*)d, dbytes / 16, flag); }, R), (double)dbytes);
    rep("write-only nt 1.2GB grid 4096", time_ms([&] { k_write_nt<<<4096, 256>>>((u32x4*)p, pbytes * 4 / 16); }, R), (double)pbytes * 4);
    rep("copy nt 512MB 1 elem/thread", time_ms([&] { k_copy_nt<<<(unsigned)((n16 + 255) / 256), 256>>>((const u32x4*)d, (u32x4*)p, n16); }, R), 2.0 * n16 * 16);
    rep("shape nt-ld nt-st 256 thr (again)", time_ms([&] { k_shape<10, 3, 1, 1, 1><<<grid1, 256>>>(d, p, G, cols, B); }, R), alg);
    rep("write-only 1.2GB grid 4096", time_ms([&] { k_write<<<4096, 256>>>((u32x4*)p, pbytes * 4 / 16); }, R), (double)pbytes * 4);
    return 0;
}
