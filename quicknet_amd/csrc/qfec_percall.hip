// qfec_percall.hip -- see qfec_percall.hpp.  One lane per 16-B column of the packets; each
// lane reads its column of the k input packets straight from pinned host memory and writes e
// output columns back, so a call is CPU staging memcpy + one launch + one synchronise.
#include "qfec_device.hpp"
#include "qfec_percall.hpp"

namespace qfec {

__global__ void __launch_bounds__(256) k_percall(PcArgs a) {
    const uint32_t col = blockIdx.x * 256u + threadIdx.x;
    if (col >= a.chunks) return;
    const uint64_t off = (uint64_t)col * 16u;
    uint4 acc[4];  // up to 4 outputs per sweep over the inputs
    for (uint32_t j0 = 0; j0 < a.e; j0 += 4) {
        const uint32_t ej = min(4u, a.e - j0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = make_uint4(0, 0, 0, 0);
        for (uint32_t c = 0; c < a.k; ++c) {
            const uint4 x = *reinterpret_cast<const uint4*>(a.in + (uint64_t)c * a.pitch + off);
            Sel s[4];
            sel16(s, x);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((uint32_t)j < ej) gf_mac16(acc[j], s, a.tab + ((j0 + j) * a.k + c) * 5);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((uint32_t)j < ej) *reinterpret_cast<uint4*>(a.out + (uint64_t)(j0 + j) * a.pitch + off) = acc[j];
    }
}

hipError_t launch_percall(const PcArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_percall, dim3((a.chunks + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace qfec
