// partial_write.hip -- what a write that covers only part of a memory sector costs on MI355X.
// The datagram kernels (qfec_wire.hip) leave a few partly written 16-B pieces per datagram
// (chunk 0 / byte 16 from the send head, the last partial chunk of each row).  This writes a
// 1 GiB region in 16-B pieces with stride S (S = 16: every byte; 32: half of every 32-B
// sector; 64: a quarter of every 64-B line; 128: an eighth of every 128-B line) and reports
// the time and the rate in bytes actually stored and in bytes spanned.
//   hipcc --offload-arch=gfx950 -O3 tools/partial_write.hip -o tools/_abl/partial_write && tools/_abl/partial_write
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

// one 16-B store per lane at byte i * stride
__global__ void __launch_bounds__(256) k_store_strided(uint8_t* __restrict__ dst, uint64_t n, int stride, int nt) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
    u32x4* p = reinterpret_cast<u32x4*>(dst + i * (uint64_t)stride);
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}

int main() {
    const uint64_t span = 1ull << 30;
    uint8_t* dst;
    CHECK(hipMalloc(&dst, span));
    CHECK(hipMemset(dst, 0, span));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int round = 0; round < 2; ++round) {
        for (int nt = 0; nt < 2; ++nt) {
            for (int stride : {16, 32, 64, 128}) {
                const uint64_t n = span / stride;
                const unsigned grid = (unsigned)((n + 255) / 256);
                for (int w = 0; w < 3; ++w) k_store_strided<<<grid, 256>>>(dst, n, stride, nt);
                CHECK(hipEventRecord(a, 0));
                for (int r = 0; r < 10; ++r) k_store_strided<<<grid, 256>>>(dst, n, stride, nt);
                CHECK(hipEventRecord(b, 0));
                CHECK(hipEventSynchronize(b));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, a, b));
                ms /= 10;
                if (round == 1)
                    printf("%s stores, 16 B every %3d B: %8.1f us  %7.1f GB/s stored  %7.1f GB/s spanned\n",
                           nt ? "nt   " : "plain", stride, ms * 1e3, 16.0 * n / (ms * 1e-3) / 1e9,
                           (double)span / (ms * 1e-3) / 1e9);
            }
        }
    }
    return 0;
}
