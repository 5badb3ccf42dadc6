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

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {  // polls: past the caches, no invalidation
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_rel_sys(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// e output columns from k input rows (x: the first min(k, KB) rows, loaded by the caller) with
// the [e][k] tables in LDS
template <int KB>
__device__ __forceinline__ void pc_serve_cols(const uint8_t* in, uint8_t* out, const uint32_t* s_tab, uint32_t k,
                                              uint32_t e, uint32_t pitch, uint64_t off, const uint4 (&x0)[KB]) {
    for (uint32_t j0 = 0; j0 < e; j0 += 4) {
        const uint32_t ej = min(4u, e - j0);
        uint4 acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = make_uint4(0, 0, 0, 0);
        for (uint32_t c0 = 0; c0 < k; c0 += KB) {
            uint4 x[KB];
#pragma unroll
            for (int i = 0; i < KB; ++i) {
                if (c0 == 0) {
                    x[i] = x0[i];
                } else {
                    const uint32_t c = min(c0 + i, k - 1);
                    x[i] = *reinterpret_cast<const uint4*>(in + (uint64_t)c * pitch + off);
                }
            }
#pragma unroll
            for (int i = 0; i < KB; ++i) {
                if (c0 + i >= k) continue;
                Sel s[4];
                sel16(s, x[i]);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if ((uint32_t)j < ej) gf_mac16(acc[j], s, s_tab + ((j0 + j) * k + c0 + i) * 5);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((uint32_t)j < ej) *reinterpret_cast<uint4*>(out + (uint64_t)(j0 + j) * pitch + off) = acc[j];
    }
}

// One block of 256 lanes, lane = one 16-B column of the packets.  Lane 0 polls the 8-byte request
// word (system-scope loads that bypass the caches), which carries the call's shape; a
// system-scope acquire fence once a request is seen invalidates the caches, so the block then
// reads what the CPU wrote.  Each lane issues its first 16 input rows' loads before the table
// loads into LDS, so the two round trips overlap.  Every iteration ends in the same place for
// every lane, and the loop exits on idle or stop, so the grid always drains.
__global__ void __launch_bounds__(256) k_percall_server(PcBell* bell, const uint8_t* in, uint8_t* out, PcStatus* st,
                                                        uint32_t served, uint32_t gen) {
    constexpr int KB = 16;
    __shared__ uint32_t s_tab[kPcMaxCoef * 5];
    __shared__ uint64_t s_bell;
    __shared__ uint32_t s_quit;
    const uint32_t t = threadIdx.x;
    if (t == 0) st_rel_sys(&st->state, (gen << 1) | 1u);
    uint64_t t0 = wall_clock64();
    for (;;) {
        if (t == 0) {
            uint64_t b = 0;
            uint32_t quit = 0;
            for (;;) {
                b = ld_sys64(&bell->bell);
                if ((uint32_t)b != served) break;
                if (ld_sys(&bell->stop) || wall_clock64() - t0 > kPcIdleTicks) {
                    quit = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!quit) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: what the CPU wrote first
            s_bell = b;
            s_quit = quit;
        }
        __syncthreads();
        if (s_quit) break;
        const uint64_t b = s_bell;
        const uint32_t r = (uint32_t)b, k = (uint32_t)(b >> 32) & 0xFFu, e = (uint32_t)(b >> 40) & 0xFFu,
                       chunks = (uint32_t)(b >> 48) + 1u, pitch = chunks * 16u;
        const uint64_t off = (uint64_t)t * 16u;
        const bool col = t < chunks;
        uint4 x0[KB];
#pragma unroll
        for (int i = 0; i < KB; ++i) {
            x0[i] = make_uint4(0, 0, 0, 0);
            if (col && (uint32_t)i < k) x0[i] = *reinterpret_cast<const uint4*>(in + (uint64_t)i * pitch + off);
        }
        for (uint32_t i = t; i < k * e * 5; i += 256) s_tab[i] = bell->tab[i];
        __syncthreads();
        if (col) pc_serve_cols<KB>(in, out, s_tab, k, e, pitch, off, x0);
        __threadfence_system();  // every lane's outputs reach the host before the completion word
        __syncthreads();         // (and no lane still reads s_tab when the next request refills it)
        if (t == 0) st_rel_sys(&st->done, r);
        served = r;
        t0 = wall_clock64();
    }
    if (t == 0) st_rel_sys(&st->state, gen << 1);  // this generation has exited
}

hipError_t launch_percall_server(PcBell* bell, const uint8_t* in, uint8_t* out, PcStatus* st, uint32_t served,
                                 uint32_t gen, hipStream_t s) {
    hipLaunchKernelGGL(k_percall_server, dim3(1), dim3(256), 0, s, bell, in, out, st, served, gen);
    return hipGetLastError();
}

hipError_t launch_percall(const PcArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_percall, dim3((a.chunks + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace qfec
