// qfec_percall.hip -- see qfec_percall.hpp.  One lane per 16-B column of the packets; each
// lane reads its column of the k input packets straight from pinned host memory and writes e
// output columns back, so a call is CPU staging memcpy + one launch + a spin on the completion word (or a
// stream synchronise).
#include "qfec_device.hpp"
#include "qfec_percall.hpp"

namespace qfec {

__global__ void __launch_bounds__(256) k_percall(PcArgs a) {
    const uint32_t col = blockIdx.x * 256u + threadIdx.x;
    if (col < a.chunks) {
        const uint64_t off = (uint64_t)col * 16u;
        uint4 acc[4];  // up to 4 outputs per sweep over the inputs
        constexpr int KB = 16;  // input rows loaded before any of them is used: the reads cross
                                // PCIe, so one round trip per batch instead of one per row
        for (uint32_t j0 = 0; j0 < a.e; j0 += 4) {
            const uint32_t ej = min(4u, a.e - j0);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = make_uint4(0, 0, 0, 0);
            for (uint32_t c0 = 0; c0 < a.k; c0 += KB) {
                uint4 x[KB];
#pragma unroll
                for (int i = 0; i < KB; ++i) {  // rows past k re-read row k - 1 (no branch, no use)
                    const uint32_t c = min(c0 + i, a.k - 1);
                    x[i] = *reinterpret_cast<const uint4*>(a.in + (uint64_t)c * a.pitch + off);
                }
#pragma unroll
                for (int i = 0; i < KB; ++i) {
                    if (c0 + i >= a.k) continue;
                    Sel s[4];
                    sel16(s, x[i]);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if ((uint32_t)j < ej) gf_mac16(acc[j], s, a.tab + ((j0 + j) * a.k + c0 + i) * 5);
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((uint32_t)j < ej) *reinterpret_cast<uint4*>(a.out + (uint64_t)(j0 + j) * a.pitch + off) = acc[j];
        }
    }
    if (a.done) {  // one-block grids only (the host checks): every wave's stores reach the
        __threadfence_system();  // host before the barrier, then one lane publishes `seq`
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(a.done, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t launch_percall(const PcArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_percall, dim3((a.chunks + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace qfec
