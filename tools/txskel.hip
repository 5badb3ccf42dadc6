// txskel.hip -- memory skeleton of the fused datagram send (k_pack_body's mapping) on MI355X:
// the same loads and stores with XOR in place of the GF arithmetic, checksums and headers, to
// separate what the mapping costs from what the arithmetic costs.  Measurement only.
//   lanes flat over (group, datagram chunk t = T0 .. T0 + lpg - 1); lane loads the K payload
//   windows at payload offset 16 t - SHIFT (unaligned unless SHIFT % 16 == 0), stores N wire
//   chunks at wire + (g N + r) wpitch + 16 t
//   hipcc --offload-arch=gfx950 -O3 -o tools/txskel tools/txskel.hip && tools/txskel
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int K, int N, int MODE>  // MODE 0 load+store, 1 load only (one store per lane), 2 store only
__global__ void __launch_bounds__(256) k_tx(const uint8_t* __restrict__ pay, uint8_t* __restrict__ wire, uint32_t lanes,
                                            uint32_t lpg, int t0, int shift, uint32_t S, uint32_t wpitch) {
    const uint32_t flat = blockIdx.x * 256u + threadIdx.x;
    if (flat >= lanes) return;
    const uint32_t g = flat / lpg;
    const int t = t0 + (int)(flat - g * lpg);
    const int p = min(max(16 * t - shift, 0), (int)S);
    u32x4 x[K];
    if (MODE != 2) {
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const uint8_t* a = pay + ((uint64_t)g * K + i) * S + p;
            if (shift & 15) {
                const uint32_t* w = reinterpret_cast<const uint32_t*>(a);  // unaligned dwordx4
                x[i] = u32x4{w[0], w[1], w[2], w[3]};
            } else {
                x[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a));
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = u32x4{(uint32_t)t, (uint32_t)i, g, 0u};
    }
    u32x4 acc = x[0];
#pragma unroll
    for (int i = 1; i < K; ++i) acc ^= x[i];
    uint8_t* out = wire + (uint64_t)g * N * wpitch + 16 * t;
    if (MODE == 1) {
        if (acc.x == 0x12345678u) __builtin_nontemporal_store(acc, reinterpret_cast<u32x4*>(out));
        return;
    }
#pragma unroll
    for (int r = 0; r < N; ++r) {
        const u32x4 v = r < K ? x[r] : acc + u32x4{(uint32_t)r, 0u, 0u, 0u};
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + (uint64_t)r * wpitch));
    }
}

int main() {
    constexpr int K = 10, N = 13;
    const uint32_t G = 100000, S = 1024;
    uint8_t *pay, *wire;
    CHECK(hipMalloc(&pay, (size_t)G * K * S + 64));
    CHECK(hipMalloc(&wire, (size_t)G * N * 1152));
    CHECK(hipMemset(pay, 1, (size_t)G * K * S + 64));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    struct V { const char* name; int mode, t0, lpg, shift; uint32_t wp; };
    const V vs[] = {
        {"pack body mapping (t 1..65, unaligned, wire 1056)", 0, 1, 65, 17, 1056},
        {"same, aligned payload windows", 0, 1, 65, 16, 1056},
        {"t 0..65 (66 lanes/group), unaligned", 0, 0, 66, 17, 1056},
        {"t 0..63 (64 lanes/group = one wave), unaligned", 0, 0, 64, 17, 1056},
        {"t 1..65, unaligned, wire 1088", 0, 1, 65, 17, 1088},
        {"loads only (t 1..65, unaligned)", 1, 1, 65, 17, 1056},
        {"stores only (t 1..65, wire 1056)", 2, 1, 65, 17, 1056},
    };
    for (int rep = 0; rep < 2; ++rep)
        for (const V& v : vs) {
            const uint32_t lanes = G * (uint32_t)v.lpg;
            auto go = [&]() {
                if (v.mode == 0) hipLaunchKernelGGL((k_tx<K, N, 0>), dim3((lanes + 255) / 256), dim3(256), 0, 0, pay, wire, lanes, v.lpg, v.t0, v.shift, S, v.wp);
                if (v.mode == 1) hipLaunchKernelGGL((k_tx<K, N, 1>), dim3((lanes + 255) / 256), dim3(256), 0, 0, pay, wire, lanes, v.lpg, v.t0, v.shift, S, v.wp);
                if (v.mode == 2) hipLaunchKernelGGL((k_tx<K, N, 2>), dim3((lanes + 255) / 256), dim3(256), 0, 0, pay, wire, lanes, v.lpg, v.t0, v.shift, S, v.wp);
            };
            for (int i = 0; i < 5; ++i) go();
            CHECK(hipEventRecord(e0, 0));
            for (int i = 0; i < 20; ++i) go();
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1000.0 / 20;
            const double rd = v.mode == 2 ? 0 : (double)G * K * S, wr = v.mode == 1 ? 0 : (double)G * N * 16 * v.lpg;
            printf("%-52s %7.1f us  %6.0f GB/s moved (rd %.2f + wr %.2f GB)\n", v.name, us, (rd + wr) / us / 1e3, rd / 1e9, wr / 1e9);
        }
    return 0;
}
