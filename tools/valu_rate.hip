// Issue rate of v_perm_b32 / v_bitop3_b32 streams per SIMD at 1..8 waves per SIMD:
// cycles per wave64 instruction on one SIMD, from s_memtime around an unrolled loop.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_rate tools/valu_rate.hip && /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int OP>
__global__ void __launch_bounds__(64) k_rate(uint32_t* out, unsigned long long* t, uint32_t seed, int iters) {
    uint32_t a[8];
    const uint32_t s = seed ^ threadIdx.x;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = s * (i + 3);
    const uint32_t x = s * 0x9E3779B9u, y = s ^ 0x5bd1e995u, z = s + 77u;
    __builtin_amdgcn_s_barrier();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (OP == 0) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(x), "v"(y));
                else if (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(x), "v"(y));
                else asm volatile("v_lshrrev_b32 %0, 3, %0\n\tv_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(z));
            }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * 64 + threadIdx.x] = r;
    if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 2000;
    uint32_t* out; unsigned long long* t;
    hipMalloc(&out, 64 * 4 * 8 * cus * 4 * 2);
    hipMalloc(&t, 8 * 4 * 8 * cus * 2);
    for (int op = 0; op < 3; ++op)
        for (int w : {1, 2, 4, 8}) {
            const int blocks = cus * 4 * w;  // one-wave blocks: w per SIMD
            for (int rep = 0; rep < 2; ++rep) {
                if (op == 0) hipLaunchKernelGGL(k_rate<0>, dim3(blocks), dim3(64), 0, 0, out, t, 1u, iters);
                if (op == 1) hipLaunchKernelGGL(k_rate<1>, dim3(blocks), dim3(64), 0, 0, out, t, 1u, iters);
                if (op == 2) hipLaunchKernelGGL(k_rate<2>, dim3(blocks), dim3(64), 0, 0, out, t, 1u, iters);
            }
            hipDeviceSynchronize();
            std::vector<unsigned long long> h(blocks);
            hipMemcpy(h.data(), t, 8 * blocks, hipMemcpyDeviceToHost);
            std::sort(h.begin(), h.end());
            const double med = (double)h[blocks / 2];
            const double insts = (op == 2 ? 2.0 : 1.0) * iters * 64;  // per wave (op 2: shift + and)
            printf("op %s waves/SIMD %d: %.0f cycles per wave-loop, %.2f cycles per instruction per wave, "
                   "%.2f per instruction per SIMD\n", op == 0 ? "v_perm " : op == 1 ? "xor3   " : "shr+and",
                   w, med, med / insts, med / insts / w);
        }
    return 0;
}
