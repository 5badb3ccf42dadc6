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
// Serves calls with k <= 16 and k * e <= 64 (kPcSrvMaxCoef; others take k_percall).  One block of
// four waves, lane = one 8-byte column of the packets (a 1 028-B packet is 129 columns): the
// multiply is VALU work that one wave would do alone (measured: 3.8 us of a call with 16-B lanes
// in one wave, the 65th column costing a whole second pass), so it is spread over the four SIMDs.
// Lane c of every wave holds coefficient c's perm table (5 dwords; v_readlane with the
// wave-uniform coefficient index gives it to the MAC as scalars, no LDS round trip per
// coefficient).  Every input byte the call needs is in registers before the first multiply: KB >=
// k rows (KB - k < 6 rows re-read row k - 1), only lanes inside the packet, all loads issued
// before any is used (one enclosing branch per group of loads: a branch per load makes the
// compiler wait for each load before it issues the next).
// rows j0 .. j0 + E - 1 of the request over the KB (k when KX) inputs in registers
template <int NQ, int KB, int E, bool KX>
__device__ __forceinline__ void pc_mac(const uint2 (&x)[NQ][KB], const uint4& ta, uint32_t tb, uint32_t k, uint32_t j0,
                                       uint2 (&acc)[NQ][4], uint32_t ej = E) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[q][j] = make_uint2(0, 0);
#pragma unroll
    for (int i = 0; i < KB; ++i) {
        if (!KX && (uint32_t)i >= k) continue;  // wave-uniform
        Sel sl[NQ][2];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            sl[q][0] = gf_sel(x[q][i].x);
            sl[q][1] = gf_sel(x[q][i].y);
        }
#pragma unroll
        for (int j = 0; j < E; ++j) {
            if ((uint32_t)j >= ej) continue;  // the generic body only (ej == E otherwise)
            const int c = (int)((j0 + j) * (KX ? (uint32_t)KB : k) + i);  // wave-uniform
            const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)ta.x, c),
                           t1 = (uint32_t)__builtin_amdgcn_readlane((int)ta.y, c),
                           t2 = (uint32_t)__builtin_amdgcn_readlane((int)ta.z, c),
                           t3 = (uint32_t)__builtin_amdgcn_readlane((int)ta.w, c),
                           t4 = (uint32_t)__builtin_amdgcn_readlane((int)tb, c);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                acc[q][j].x = xor3(acc[q][j].x, pp0(sl[q][0], t0, t1), pp1(sl[q][0], t2, t3)) ^ pp2(sl[q][0], t4);
                acc[q][j].y = xor3(acc[q][j].y, pp0(sl[q][1], t0, t1), pp1(sl[q][1], t2, t3)) ^ pp2(sl[q][1], t4);
            }
        }
    }
}

template <int NQ, int KB>
__device__ __forceinline__ void pc_block_serve(const PcBell* bell, const uint8_t* in, uint8_t* out, uint32_t k,
                                               uint32_t e, uint32_t cols, uint32_t pitch, uint32_t t,
                                               uint64_t& ts_loaded) {
    const uint32_t lane = t & 63u;
    uint2 x[NQ][KB];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const uint32_t col = t + 256u * q;
#pragma unroll
        for (int i = 0; i < KB; ++i) x[q][i] = make_uint2(0, 0);
        if (col < cols) {
#pragma unroll
            for (int i = 0; i < KB; ++i)
                x[q][i] = *reinterpret_cast<const uint2*>(in + (uint64_t)min((uint32_t)i, k - 1) * pitch + (uint64_t)col * 8u);
        }
    }
    uint4 ta = make_uint4(0, 0, 0, 0);  // coefficient `lane`: table dwords 0-3, then 4
    uint32_t tb = 0;
    if (lane < k * e) {
        ta = *reinterpret_cast<const uint4*>(bell->tab + 8u * lane);
        tb = bell->tab[8u * lane + 4u];
    }
    if (ts_loaded) {  // QFEC_PERCALL_TRACE: when every load has landed
        __builtin_amdgcn_s_waitcnt(0);
        ts_loaded = __builtin_amdgcn_s_memtime();
    }
    if ((t & ~63u) >= cols) return;  // a wave with no column (wave-uniform)
    const bool kx = k == (uint32_t)KB;
    for (uint32_t j0 = 0; j0 < e; j0 += 4) {
        const uint32_t ej = min(4u, e - j0);
        uint2 acc[NQ][4];
        // straight-line bodies for the chunk's exact row count (and k == KB): no branch between
        // coefficients, so the table reads of the next coefficient overlap this one's multiply
        if constexpr (NQ != 1) {  // rows over 2 KiB: one generic body
            pc_mac<NQ, KB, 4, false>(x, ta, tb, k, j0, acc, ej);
        } else switch (ej * 2u + (kx ? 1u : 0u)) {
            case 2: pc_mac<NQ, KB, 1, false>(x, ta, tb, k, j0, acc); break;
            case 3: pc_mac<NQ, KB, 1, true>(x, ta, tb, k, j0, acc); break;
            case 4: pc_mac<NQ, KB, 2, false>(x, ta, tb, k, j0, acc); break;
            case 5: pc_mac<NQ, KB, 2, true>(x, ta, tb, k, j0, acc); break;
            case 6: pc_mac<NQ, KB, 3, false>(x, ta, tb, k, j0, acc); break;
            case 7: pc_mac<NQ, KB, 3, true>(x, ta, tb, k, j0, acc); break;
            case 8: pc_mac<NQ, KB, 4, false>(x, ta, tb, k, j0, acc); break;
            default: pc_mac<NQ, KB, 4, true>(x, ta, tb, k, j0, acc); break;
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const uint32_t col = t + 256u * q;
            if (col < cols) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if ((uint32_t)j < ej)
                        *reinterpret_cast<uint2*>(out + (uint64_t)(j0 + j) * pitch + (uint64_t)col * 8u) = acc[q][j];
            }
        }
    }
}

template <int NQ>
__device__ __forceinline__ void pc_block_serve_k(const PcBell* bell, const uint8_t* in, uint8_t* out, uint32_t k,
                                                 uint32_t e, uint32_t cols, uint32_t pitch, uint32_t t, uint64_t& ts) {
    if (k <= 4) pc_block_serve<NQ, 4>(bell, in, out, k, e, cols, pitch, t, ts);
    else if (k <= 10) pc_block_serve<NQ, 10>(bell, in, out, k, e, cols, pitch, t, ts);
    else pc_block_serve<NQ, 16>(bell, in, out, k, e, cols, pitch, t, ts);
}

// Lane 0 polls the 8-byte request word (system-scope loads that bypass the caches), which carries
// the call's shape, and after it a system-scope acquire fence invalidates the caches, so the block
// then reads what the CPU wrote before the word.  Every iteration ends in the same place for
// every lane, and the loop exits on idle or stop, so the grid always drains.
__global__ void __launch_bounds__(256)
k_percall_server(PcBell* bell, const uint8_t* in, uint8_t* out, PcStatus* st, uint32_t served, uint32_t gen,
                 uint32_t flags, uint64_t idle_ticks) {
    const uint32_t trace = flags & 1u;
    __shared__ uint64_t s_bell;
    __shared__ uint32_t s_quit;
    const uint32_t t = threadIdx.x;
    if (t == 0) st_rel_sys(&st->state, (gen << 1) | 1u);
    uint64_t t0 = wall_clock64();
    for (;;) {
        if (t == 0) {
            uint64_t b = 0;
            uint32_t quit = 0;
            for (uint32_t it = 1;; ++it) {  // one load per poll; `stop` and the idle clock every 16th
                b = ld_sys64(&bell->bell);
                if ((uint32_t)b != served) break;
                if ((it & 15u) == 0 && (ld_sys(&bell->stop) || wall_clock64() - t0 > idle_ticks)) {
                    quit = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!quit) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
            s_bell = b;
            s_quit = quit;
        }
        __syncthreads();
        if (s_quit) break;
        // QFEC_PERCALL_TRACE stage stamps in shader clocks (s_memtime, read in the CU): a
        // s_memrealtime read takes a round trip of its own that would land in the stage it
        // brackets; two wall-clock reads at the ends calibrate the clock
        const uint64_t rt0 = trace ? wall_clock64() : 0;
        const uint64_t ts0 = trace ? __builtin_amdgcn_s_memtime() : 0;
        const uint64_t b = s_bell;
        const uint32_t r = (uint32_t)b, k = (uint32_t)(b >> 32) & 0xFFu, e = (uint32_t)(b >> 40) & 0xFFu,
                       chunks = (uint32_t)(b >> 48) + 1u, pitch = chunks * 16u, cols = chunks * 2u;
        uint64_t ts1 = trace;
        if (cols <= 256) pc_block_serve_k<1>(bell, in, out, k, e, cols, pitch, t, ts1);
        else pc_block_serve_k<2>(bell, in, out, k, e, cols, pitch, t, ts1);
        const uint64_t ts2 = trace ? __builtin_amdgcn_s_memtime() : 0;
        __threadfence_system();  // every lane's outputs reach the host before the completion word
        __syncthreads();         // (and s_bell is not rewritten before every lane has read it)
        if (trace && t == 0) {
            st->ts[0] = ts0;
            st->ts[1] = ts1;
            st->ts[2] = ts2;
            st->ts[3] = __builtin_amdgcn_s_memtime();
            st->rt = wall_clock64() - rt0;
            __threadfence_system();
        }
        if (t == 0) st_rel_sys(&st->done, r);
        served = r;
        t0 = wall_clock64();
    }
    if (t == 0) st_rel_sys(&st->state, gen << 1);  // this generation has exited
}

hipError_t launch_percall_server(PcBell* bell, const uint8_t* in, uint8_t* out, PcStatus* st, uint32_t served,
                                 uint32_t gen, uint32_t flags, uint64_t idle_ticks, hipStream_t s) {
    hipLaunchKernelGGL(k_percall_server, dim3(1), dim3(256), 0, s, bell, in, out, st, served, gen, flags, idle_ticks);
    return hipGetLastError();
}

hipError_t launch_percall(const PcArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_percall, dim3((a.chunks + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace qfec
