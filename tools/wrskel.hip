// wrskel.hip -- store-pattern study for the fused datagram send (measurement only): 16-B
// stores, lanes flat over (group, chunk t = t0 .. t0 + lpg - 1), each lane storing `rows`
// chunks at base + g gs + r pitch + 16 t.  Compares the send's pattern with contiguous ones.
//   hipcc --offload-arch=gfx950 -O3 -o tools/wrskel tools/wrskel.hip && tools/wrskel
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int NT>
__global__ void __launch_bounds__(256) k_w(uint8_t* __restrict__ base, uint32_t lanes, uint32_t lpg, int t0, uint32_t rows,
                                           uint32_t pitch, uint64_t gs) {
    const uint32_t flat = blockIdx.x * 256u + threadIdx.x;
    if (flat >= lanes) return;
    const uint32_t g = flat / lpg;
    const int t = t0 + (int)(flat - g * lpg);
    uint8_t* out = base + (uint64_t)g * gs + 16 * t;
    for (uint32_t r = 0; r < rows; ++r) {
        const u32x4 v = u32x4{(uint32_t)t, r, g, 7u};
        if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + (uint64_t)r * pitch));
        else *reinterpret_cast<u32x4*>(out + (uint64_t)r * pitch) = v;
    }
}

int main() {
    uint8_t* buf;
    const size_t cap = (size_t)100000 * 13 * 1152;
    CHECK(hipMalloc(&buf, cap));
    CHECK(hipMemset(buf, 0, cap));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    struct V { const char* name; uint32_t G, lpg; int t0; uint32_t rows, pitch; uint64_t gs; };
    const V vs[] = {
        {"contiguous, 1 store/lane", 1300000, 64, 0, 1, 0, 1024},
        {"contiguous 13 KB per wave, 13 stores/lane", 100000, 64, 0, 13, 1024, 13312},
        {"send: t 1..65, pitch 1056 (k_pack_body)", 100000, 65, 1, 13, 1056, 13728},
        {"send: t 0..65, pitch 1056", 100000, 66, 0, 13, 1056, 13728},
        {"t 0..63, pitch 1088 (64-B rows, gap lines)", 100000, 64, 0, 13, 1088, 14144},
        {"t 0..67, pitch 1088 (whole 64-B rows)", 100000, 68, 0, 13, 1088, 14144},
        {"t 0..65, pitch 1056, 2 waves' worth per group padded to 128 lanes", 100000, 128, 0, 13, 1056, 13728},
    };
    for (int rep = 0; rep < 2; ++rep)
        for (int nt = 1; nt >= 0; --nt)
            for (const V& v : vs) {
                uint32_t lanes = v.G * v.lpg;
                uint32_t lpg = v.lpg;
                int chunks = v.lpg;
                if (v.lpg == 128) chunks = 66;
                auto go = [&]() {
                    if (v.lpg == 128) {  // lanes >= 66 of each group idle
                        if (nt) hipLaunchKernelGGL(k_w<1>, dim3((lanes + 255) / 256), dim3(256), 0, 0, buf, lanes, lpg, -1000000, v.rows, v.pitch, v.gs);
                    }
                    if (nt) hipLaunchKernelGGL(k_w<1>, dim3((lanes + 255) / 256), dim3(256), 0, 0, buf, lanes, lpg, v.t0, v.rows, v.pitch, v.gs);
                    else hipLaunchKernelGGL(k_w<0>, dim3((lanes + 255) / 256), dim3(256), 0, 0, buf, lanes, lpg, v.t0, v.rows, v.pitch, v.gs);
                };
                if (v.lpg == 128) continue;  // (placeholder variant, not run)
                for (int i = 0; i < 5; ++i) go();
                CHECK(hipEventRecord(e0, 0));
                for (int i = 0; i < 20; ++i) go();
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1000.0 / 20;
                const double wr = (double)v.G * v.rows * 16 * chunks;
                printf("%s %-48s %7.1f us  %6.0f GB/s stored (%.2f GB)\n", nt ? "nt   " : "plain", v.name, us, wr / us / 1e3, wr / 1e9);
            }
    return 0;
}
