// unaligned.hip -- what a byte-misaligned 16-B-per-lane load stream costs on MI355X.
// The fused datagram send (qfec_wire.hip k_pack_body) reads payload windows at any byte
// offset; this copies 512 MiB from src + OFF (OFF = 0, 1, 4, 8, 13) into an aligned buffer
// with one global_load_dwordx4 per lane, and reports GB/s (read + write bytes) per offset.
//   hipcc --offload-arch=gfx950 -O3 tools/unaligned.hip -o tools/unaligned && tools/unaligned
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

__global__ void __launch_bounds__(256) k_copy_off(const uint8_t* __restrict__ src, u32x4* __restrict__ dst,
                                                  uint64_t n, int off) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    u32x4 v;
    __builtin_memcpy(&v, src + off + 16 * i, 16);
    __builtin_nontemporal_store(v, dst + i);
}

int main() {
    const uint64_t bytes = 512ull << 20, n = bytes / 16;
    uint8_t* src;
    u32x4* dst;
    CHECK(hipMalloc(&src, bytes + 64));
    CHECK(hipMalloc(&dst, bytes));
    CHECK(hipMemset(src, 7, bytes + 64));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const unsigned grid = (unsigned)((n + 255) / 256);
    for (int round = 0; round < 2; ++round) {
        for (int off : {0, 1, 4, 8, 13}) {
            for (int w = 0; w < 3; ++w) k_copy_off<<<grid, 256>>>(src, dst, n, off);
            CHECK(hipEventRecord(a, 0));
            for (int r = 0; r < 20; ++r) k_copy_off<<<grid, 256>>>(src, dst, n, off);
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            ms /= 20;
            if (round == 1) printf("src offset %2d: %8.1f us  %7.1f GB/s (read + write)\n", off, ms * 1e3,
                                   2.0 * bytes / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
