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

// store cache-policy variants through buffer stores (aux: 1 sc0, 2 nt, 16 sc1)
template <int AUX>
__global__ void __launch_bounds__(256) k_shape_aux(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                                   uint64_t groups, uint32_t cols, uint64_t pitch) {
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t g = t / cols;
    if (g >= groups) return;
    const uint32_t col = (uint32_t)(t - g * cols);
    const u32x4* src = (const u32x4*)(data + g * 10 * pitch + col * 16u);
    u32x4 x[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) x[c] = __builtin_nontemporal_load(src + c * (pitch / 16));
    u32x4 acc = x[0];
#pragma unroll
    for (int c = 1; c < 10; ++c) acc ^= x[c];
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(par + g * 3 * pitch, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        __builtin_amdgcn_raw_buffer_store_b128(acc, rs, (int)(r * pitch + col * 16u), 0, AUX);
        acc.x += 1;
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
    // what the NEXT kernel pays after each store flavour (bench.py runs reconstruct right after encode)
    {
        hipEvent_t e0, e1, e2;
        CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1)); CHECK(hipEventCreate(&e2));
        auto pair = [&](const char* nm, auto kfn) {
            double tw = 0, tr = 0;
            for (int i = 0; i < 12; ++i) {
                CHECK(hipEventRecord(e0, 0));
                kfn();
                CHECK(hipEventRecord(e1, 0));
                k_read<<<4096, 256>>>((const u32x4*)d, dbytes / 16, flag);
                CHECK(hipEventRecord(e2, 0));
                CHECK(hipEventSynchronize(e2));
                float a = 0, b = 0;
                CHECK(hipEventElapsedTime(&a, e0, e1));
                CHECK(hipEventElapsedTime(&b, e1, e2));
                if (i >= 2) { tw += a; tr += b; }
            }
            printf("%-40s shape %7.1f us (%6.1f GB/s) | next read-only 1GB %7.1f us (%6.1f GB/s)\n", nm, tw / 10 * 1e3,
                   alg / (tw / 10 * 1e-3) / 1e9, tr / 10 * 1e3, dbytes / (tr / 10 * 1e-3) / 1e9);
        };
        pair("store plain (aux 0)", [&] { k_shape_aux<0><<<grid1, 256>>>(d, p, G, cols, B); });
        pair("store nt (aux 2)", [&] { k_shape_aux<2><<<grid1, 256>>>(d, p, G, cols, B); });
        pair("store sc1 (aux 16)", [&] { k_shape_aux<16><<<grid1, 256>>>(d, p, G, cols, B); });
        pair("store nt sc1 (aux 18)", [&] { k_shape_aux<18><<<grid1, 256>>>(d, p, G, cols, B); });
        pair("store sc0 sc1 (aux 17)", [&] { k_shape_aux<17><<<grid1, 256>>>(d, p, G, cols, B); });
        pair("store nt sc0 sc1 (aux 19)", [&] { k_shape_aux<19><<<grid1, 256>>>(d, p, G, cols, B); });
        pair("read-only itself (baseline)", [&] { k_read<<<4096, 256>>>((const u32x4*)d, dbytes / 16, flag); });
        // does reading the lines the previous kernel just wrote cost more?
        double tw = 0, tr = 0, tr2 = 0;
        for (int i = 0; i < 12; ++i) {
            CHECK(hipEventRecord(e0, 0));
            k_shape_aux<2><<<grid1, 256>>>(d, p, G, cols, B);
            CHECK(hipEventRecord(e1, 0));
            k_read<<<4096, 256>>>((const u32x4*)p, pbytes / 16, flag);
            CHECK(hipEventRecord(e2, 0));
            CHECK(hipEventSynchronize(e2));
            float a = 0, b = 0;
            CHECK(hipEventElapsedTime(&b, e1, e2));
            k_read<<<4096, 256>>>((const u32x4*)(d + dbytes - pbytes), pbytes / 16, flag);
            CHECK(hipEventRecord(e1, 0));
            k_read<<<4096, 256>>>((const u32x4*)(p + pbytes), pbytes / 16, flag);
            CHECK(hipEventRecord(e2, 0));
            CHECK(hipEventSynchronize(e2));
            CHECK(hipEventElapsedTime(&a, e1, e2));
            if (i >= 2) { tr += b; tr2 += a; }
        }
        printf("after nt-store shape: read of the 307MB just written %7.1f us; read of 307MB not written %7.1f us\n",
               tr / 10 * 1e3, tr2 / 10 * 1e3);
    }
    rep("write-only 1.2GB grid 4096", time_ms([&] { k_write<<<4096, 256>>>((u32x4*)p, pbytes * 4 / 16); }, R), (double)pbytes * 4);
    return 0;
}
