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
// 16 bytes past the caches (two system-scope 8-byte loads, global_load_dwordx2 sc0 sc1): what
// the CPU wrote into device or host memory, with no cache invalidation before it
__device__ __forceinline__ uint4 ld_sys16(const void* p) {
    const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
    const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}
__device__ __forceinline__ void st_rel_sys(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- the resident server (qfec_percall.hpp)
// Serves calls with k <= 16 and k * e <= 64 (kPcSrvMaxCoef; others take k_percall): lane c holds
// coefficient c's perm table (5 dwords; v_readlane with the wave-uniform coefficient index
// gives it to the MAC as scalars, no LDS round trip per coefficient), and every input byte the
// call needs is in registers before the first multiply.  The inputs and tables are read past the
// caches (system-scope loads), so no cache invalidation is needed; they live in fine-grained
// memory whose reads each go to memory, so only what the call needs is read -- KB >= k rows
// (KB - k < 6 rows re-read row k - 1), only lanes inside the packet -- and all of it is issued
// before any of it is used (one enclosing branch per group of loads: a branch per load makes the
// compiler wait for each load before it issues the next).
template <int NQ, int KB>
__device__ __forceinline__ void pc_wave_serve(const PcBell* bell, const uint8_t* in, uint8_t* out, uint32_t k,
                                              uint32_t e, uint32_t chunks, uint32_t col0, uint32_t lane) {
    const uint32_t pitch = chunks * 16u;
    uint4 x[NQ][KB];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const uint32_t col = col0 + lane + 64u * q;
#pragma unroll
        for (int i = 0; i < KB; ++i) x[q][i] = make_uint4(0, 0, 0, 0);
        if (col < chunks) {
#pragma unroll
            for (int i = 0; i < KB; ++i) x[q][i] = ld_sys16(in + (uint64_t)min((uint32_t)i, k - 1) * pitch + (uint64_t)col * 16u);
        }
    }
    uint4 ta = make_uint4(0, 0, 0, 0), tb = make_uint4(0, 0, 0, 0);  // coefficient `lane`: dwords 0-3, 4
    if (lane < k * e) {
        ta = ld_sys16(bell->tab + 8u * lane);
        tb = ld_sys16(bell->tab + 8u * lane + 4u);
    }
    for (uint32_t j0 = 0; j0 < e; j0 += 4) {
        const uint32_t ej = min(4u, e - j0);
        uint4 acc[NQ][4];
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[q][j] = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < KB; ++i) {
            if ((uint32_t)i >= k) continue;
            Sel sl[NQ][4];
#pragma unroll
            for (int q = 0; q < NQ; ++q) sel16(sl[q], x[q][i]);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if ((uint32_t)j >= ej) continue;
                const int c = (int)((j0 + j) * k + i);  // wave-uniform
                const uint32_t t[5] = {(uint32_t)__builtin_amdgcn_readlane((int)ta.x, c),
                                       (uint32_t)__builtin_amdgcn_readlane((int)ta.y, c),
                                       (uint32_t)__builtin_amdgcn_readlane((int)ta.z, c),
                                       (uint32_t)__builtin_amdgcn_readlane((int)ta.w, c),
                                       (uint32_t)__builtin_amdgcn_readlane((int)tb.x, c)};
#pragma unroll
                for (int q = 0; q < NQ; ++q) gf_mac16(acc[q][j], sl[q], t);
            }
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const uint32_t col = col0 + lane + 64u * q;
            if (col < chunks) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if ((uint32_t)j < ej)
                        *reinterpret_cast<uint4*>(out + (uint64_t)(j0 + j) * pitch + (uint64_t)col * 16u) = acc[q][j];
            }
        }
    }
}

template <int NQ>
__device__ __forceinline__ void pc_wave_serve_k(const PcBell* bell, const uint8_t* in, uint8_t* out, uint32_t k,
                                                uint32_t e, uint32_t chunks, uint32_t col0, uint32_t lane) {
    if (k <= 4) pc_wave_serve<NQ, 4>(bell, in, out, k, e, chunks, col0, lane);
    else if (k <= 10) pc_wave_serve<NQ, 10>(bell, in, out, k, e, chunks, col0, lane);
    else pc_wave_serve<NQ, 16>(bell, in, out, k, e, chunks, col0, lane);
}

// One wave, lane = 16-B columns lane, lane + 64, ... of the packets.  The wave polls the 8-byte
// request word (system-scope loads that bypass the caches), which carries the call's shape.
// One wave, not a block of four: one system fence per call and no workgroup barriers.  Every
// iteration ends in the same place for every lane, and the loop exits on idle or stop, so the
// grid always drains.
__global__ void __launch_bounds__(64) k_percall_server(PcBell* bell, const uint8_t* in, uint8_t* out, PcStatus* st,
                                                       uint32_t served, uint32_t gen, uint32_t trace) {
    const uint32_t lane = threadIdx.x;
    if (lane == 0) st_rel_sys(&st->state, (gen << 1) | 1u);
    uint64_t t0 = wall_clock64();
    for (;;) {
        uint64_t b = 0;
        bool quit = false;
        for (uint32_t it = 1;; ++it) {  // one load per poll; `stop` and the idle clock every 16th
            const uint64_t v = ld_sys64(&bell->bell);  // every lane loads the same word: make it uniform
            b = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
                ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
            if ((uint32_t)b != served) break;
            if ((it & 15u) == 0 && (ld_sys(&bell->stop) || wall_clock64() - t0 > kPcIdleTicks)) {
                quit = true;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (quit) break;
        const uint64_t ts0 = trace ? wall_clock64() : 0;
        const uint32_t r = (uint32_t)b, k = (uint32_t)(b >> 32) & 0xFFu, e = (uint32_t)(b >> 40) & 0xFFu,
                       chunks = (uint32_t)(b >> 48) + 1u;
        if (chunks <= 64) {
            pc_wave_serve_k<1>(bell, in, out, k, e, chunks, 0, lane);
        } else {  // 128 columns at a time (2 KiB packets in one round trip)
            for (uint32_t c0 = 0; c0 < chunks; c0 += 128) pc_wave_serve_k<2>(bell, in, out, k, e, chunks, c0, lane);
        }
        const uint64_t ts2 = trace ? wall_clock64() : 0;
        __threadfence_system();  // every lane's outputs reach the host before the completion word
        if (trace && lane == 0) {
            st->ts[0] = ts0;
            st->ts[1] = ts0;
            st->ts[2] = ts2;
            st->ts[3] = wall_clock64();
            __threadfence_system();
        }
        if (lane == 0) st_rel_sys(&st->done, r);
        served = r;
        t0 = wall_clock64();
    }
    if (lane == 0) st_rel_sys(&st->state, gen << 1);  // this generation has exited
}

hipError_t launch_percall_server(PcBell* bell, const uint8_t* in, uint8_t* out, PcStatus* st, uint32_t served,
                                 uint32_t gen, uint32_t trace, hipStream_t s) {
    hipLaunchKernelGGL(k_percall_server, dim3(1), dim3(64), 0, s, bell, in, out, st, served, gen, trace);
    return hipGetLastError();
}

hipError_t launch_percall(const PcArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_percall, dim3((a.chunks + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace qfec
