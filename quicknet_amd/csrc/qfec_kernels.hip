// qfec_kernels.hip -- GF(2^8) Reed-Solomon kernels for MI355X (gfx950 / CDNA4).
//
// What is computed (bit-exact with the reference, skywind3000/QuickNet):
//   encode       parity[g][r][b] = XOR_c P[r][c] * data[g][c][b]
//                  module/rs.c:364-378 (code_some_shards), module/fec.c:714-733 (fec_encode)
//   reconstruct  data[g][lost_r][b] = XOR_s D_pat[r][s] * survivor[g][s][b]
//                  module/rs.c:500-643, module/fec.c:821-862
// GF(2^8) over x^8+x^4+x^3+x^2+1 (0x11D).  No floating point, no MFMA: this is byte-wise
// Galois arithmetic, HBM-bound.
//
// GF multiply by a constant, four bytes per VALU op.  Multiplication by a fixed c is
// linear over GF(2), so c*x = c*(x & 7) ^ c*(x & 0x38) ^ c*(x & 0xC0).  Each of the three
// partial products is a lookup in an 8-entry (or 4-entry) byte table, which is exactly
// what v_perm_b32 does for four byte lanes at once (selector bytes 0..7 pick a byte of
// the 64-bit {src0:src1} pair).  Per coefficient that is 5 dwords of table ("perm
// table", built on the host by gf256.cpp) and 3 v_perm_b32 + 2 XOR per 4 bytes; the
// three selector words of an input dword are shared by every output row.  The tables are
// wave-uniform (scalar loads, SGPRs); no LDS traffic and no bank conflicts on the hot path.
//
// A second variant stages the classic log/exp tables in LDS (the north-star sketch) for
// A/B comparison (QFEC_VARIANT_LDSLOG).
//
// Memory mapping: one lane per 16-byte column of a shard row (global_load_dwordx4 /
// global_store_dwordx4, 1 KiB per wave-instruction).  Encode flattens (group, column)
// over the grid, so a wave reads 64 consecutive 16-B columns of each of the k shard rows:
// fully coalesced.  Reconstruct runs one wave per group so the erasure pattern, and with
// it the decode coefficients, are wave-uniform.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "qfec_internal.hpp"

namespace qfec {

}  // namespace qfec
#include "qfec_device.hpp"
namespace qfec {

// ------------------------------------------------------------------ encode (perm tables)
// tab layout: [rows][k][QFEC_TAB_STRIDE] dwords; dword 5 of (r, 0) = 1 if row r starts
// from the destination's previous bytes (rs.c column-0 zero-coefficient quirk).

template <int K, int M, int BS = 256>
__global__ void __launch_bounds__(256) k_encode_perm(EncodeArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * (uint64_t)BS + threadIdx.x;
    if (t >= a.work) return;
    const uint64_t g = fast_div(t, a.cols_div);
    const uint32_t col = (uint32_t)(t - g * (uint64_t)a.cols);
    const uint8_t* src = a.data + g * a.dgs + (uint64_t)col * 16u;
    uint8_t* dst = a.parity + g * a.pgs + (uint64_t)col * 16u;
    const uint32_t* __restrict__ tab = a.tab;

    uint4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = ld16(src + (uint64_t)c * a.pitch);

    uint4 acc[M];
#pragma unroll
    for (int r = 0; r < M; ++r) {
        acc[r] = make_uint4(0, 0, 0, 0);
        if (tab[(r * K) * QFEC_TAB_STRIDE + 5]) acc[r] = *reinterpret_cast<const uint4*>(dst + (uint64_t)r * a.pitch);
    }
#pragma unroll
    for (int c = 0; c + 1 < K; c += 2) {
        Sel sa[4], sb[4];
        sel16(sa, x[c]);
        sel16(sb, x[c + 1]);
#pragma unroll
        for (int r = 0; r < M; ++r)
            gf_mac16x2(acc[r], sa, sb, tab + (r * K + c) * QFEC_TAB_STRIDE, tab + (r * K + c + 1) * QFEC_TAB_STRIDE);
    }
    if (K & 1) {
        Sel s[4];
        sel16(s, x[K - 1]);
#pragma unroll
        for (int r = 0; r < M; ++r) gf_mac16(acc[r], s, tab + (r * K + K - 1) * QFEC_TAB_STRIDE);
    }
#pragma unroll
    for (int r = 0; r < M; ++r) st16(dst + (uint64_t)r * a.pitch, acc[r]);
}

// Variant (tuning "encode_impl" = 2): the K inputs in two halves, the second half's loads issued
// only after the first half has been multiplied in -- half the input registers live at a time
// (RS(16,4): 69 instead of 116 VGPRs, 7 waves per SIMD instead of 4; RS(10,3): 60 instead of 102),
// so more waves share the memory latency; each wave has one round trip more.  Same VALU as impl 0.
template <int K, int M, int BS = 256>
__global__ void __launch_bounds__(256) k_encode_perm_halves(EncodeArgs a) {
    constexpr int H = (K + 1) / 2;
    const uint64_t t = (uint64_t)blockIdx.x * (uint64_t)BS + threadIdx.x;
    if (t >= a.work) return;
    const uint64_t g = fast_div(t, a.cols_div);
    const uint32_t col = (uint32_t)(t - g * (uint64_t)a.cols);
    const uint8_t* src = a.data + g * a.dgs + (uint64_t)col * 16u;
    uint8_t* dst = a.parity + g * a.pgs + (uint64_t)col * 16u;
    const uint32_t* __restrict__ tab = a.tab;
    uint4 acc[M];
#pragma unroll
    for (int r = 0; r < M; ++r) {
        acc[r] = make_uint4(0, 0, 0, 0);
        if (tab[(r * K) * QFEC_TAB_STRIDE + 5]) acc[r] = *reinterpret_cast<const uint4*>(dst + (uint64_t)r * a.pitch);
    }
#pragma unroll
    for (int c0 = 0; c0 < K; c0 += H) {
        // a scheduling fence, not a memory one: the next half's loads are not hoisted above this
        // half's multiply (and the table loads stay scalar -- an asm pin would make them vector)
        __builtin_amdgcn_sched_barrier(0);
        constexpr int HH = H;
        const int n = min(HH, K - c0);
        uint4 x[H];
#pragma unroll
        for (int i = 0; i < H; ++i)
            if (i < n) x[i] = ld16(src + (uint64_t)(c0 + i) * a.pitch);
#pragma unroll
        for (int i = 0; i + 1 < H; i += 2) {
            if (i + 1 >= n) continue;
            Sel sa[4], sb[4];
            sel16(sa, x[i]);
            sel16(sb, x[i + 1]);
#pragma unroll
            for (int r = 0; r < M; ++r)
                gf_mac16x2(acc[r], sa, sb, tab + (r * K + c0 + i) * QFEC_TAB_STRIDE,
                           tab + (r * K + c0 + i + 1) * QFEC_TAB_STRIDE);
        }
        if (n & 1) {
            Sel sl[4];
            sel16(sl, x[n - 1]);
#pragma unroll
            for (int r = 0; r < M; ++r) gf_mac16(acc[r], sl, tab + (r * K + c0 + n - 1) * QFEC_TAB_STRIDE);
        }
    }
#pragma unroll
    for (int r = 0; r < M; ++r) st16(dst + (uint64_t)r * a.pitch, acc[r]);
}

// runtime k, m: output rows in chunks of RCH; the k input rows are re-read per chunk
// (L1/L2 hits).  Used for uncommon shapes and for the single-row fec_encode calls.
constexpr int RCH = 4;

__global__ void __launch_bounds__(256) k_encode_perm_any(EncodeArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (t >= a.work) return;
    const uint64_t g = fast_div(t, a.cols_div);
    const uint32_t col = (uint32_t)(t - g * (uint64_t)a.cols);
    const int k = a.k, m = a.m;
    const uint8_t* src = a.data + g * a.dgs + (uint64_t)col * 16u;
    uint8_t* dst = a.parity + g * a.pgs + (uint64_t)col * 16u;
    for (int r0 = 0; r0 < m; r0 += RCH) {
        uint4 acc[RCH];
#pragma unroll
        for (int j = 0; j < RCH; ++j) {
            acc[j] = make_uint4(0, 0, 0, 0);
            if (r0 + j < m && a.tab[((r0 + j) * k) * QFEC_TAB_STRIDE + 5])
                acc[j] = *reinterpret_cast<const uint4*>(dst + (uint64_t)(r0 + j) * a.pitch);
        }
        for (int c = 0; c < k; ++c) {
            const uint4 v = ld16(src + (uint64_t)c * a.pitch);
            Sel s[4];
            sel16(s, v);
#pragma unroll
            for (int j = 0; j < RCH; ++j)
                if (r0 + j < m) gf_mac16(acc[j], s, a.tab + ((r0 + j) * k + c) * QFEC_TAB_STRIDE);
        }
#pragma unroll
        for (int j = 0; j < RCH; ++j)
            if (r0 + j < m) st16(dst + (uint64_t)(r0 + j) * a.pitch, acc[j]);
    }
}

// byte-granular fallback for pitches / pointers that are not 16-B aligned
__global__ void __launch_bounds__(256) k_encode_bytes(EncodeArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (t >= a.work) return;
    const uint64_t g = fast_div(t, a.cols_div);
    const uint32_t b = (uint32_t)(t - g * (uint64_t)a.cols);
    const int k = a.k, m = a.m;
    const uint8_t* src = a.data + g * a.dgs + b;
    uint8_t* dst = a.parity + g * a.pgs + b;
    for (int r = 0; r < m; ++r) {
        const uint32_t* tr = a.tab + (r * k) * QFEC_TAB_STRIDE;
        uint32_t acc = tr[5] ? (uint32_t)dst[(uint64_t)r * a.pitch] : 0u;
        for (int c = 0; c < k; ++c) {
            const uint32_t* tc = tr + c * QFEC_TAB_STRIDE;
            const Sel s = gf_sel((uint32_t)src[(uint64_t)c * a.pitch]);
            acc ^= gf_mul4(s, tc[0], tc[1], tc[2], tc[3], tc[4]);
        }
        dst[(uint64_t)r * a.pitch] = (uint8_t)acc;
    }
}

// ------------------------------------------------------------------ encode (LDS log/exp)
// The textbook form: log[x] looked up once per input byte and shared by the m rows, one
// exp lookup per multiply-accumulate, zero handled by a select.  Tables staged in LDS per
// workgroup.  Kept as the A/B baseline for the perm-table kernel.

__global__ void __launch_bounds__(256) k_encode_ldslog(EncodeArgs a) {
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    for (int i = threadIdx.x; i < 512; i += 256) s_exp[i] = a.gf_exp[i];
    s_log[threadIdx.x] = a.gf_log[threadIdx.x];
    __syncthreads();
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (t >= a.work) return;
    const uint64_t g = fast_div(t, a.cols_div);
    const uint32_t col = (uint32_t)(t - g * (uint64_t)a.cols);
    const int k = a.k, m = a.m;
    const uint8_t* src = a.data + g * a.dgs + (uint64_t)col * 16u;
    uint8_t* dst = a.parity + g * a.pgs + (uint64_t)col * 16u;
    for (int r0 = 0; r0 < m; r0 += RCH) {
        uint32_t acc[RCH][4];
#pragma unroll
        for (int j = 0; j < RCH; ++j) {
            uint4 init = make_uint4(0, 0, 0, 0);
            if (r0 + j < m && a.tab[((r0 + j) * k) * QFEC_TAB_STRIDE + 5])
                init = *reinterpret_cast<const uint4*>(dst + (uint64_t)(r0 + j) * a.pitch);
            acc[j][0] = init.x; acc[j][1] = init.y; acc[j][2] = init.z; acc[j][3] = init.w;
        }
        for (int c = 0; c < k; ++c) {
            const uint4 v = ld16(src + (uint64_t)c * a.pitch);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int byte = 0; byte < 4; ++byte) {
                    const uint32_t x = (w[q] >> (8 * byte)) & 0xFFu;
                    const uint32_t lx = s_log[x];
#pragma unroll
                    for (int j = 0; j < RCH; ++j) {
                        if (r0 + j >= m) continue;
                        const uint32_t lc = a.tab[((r0 + j) * k + c) * QFEC_TAB_STRIDE + 6];  // log of coefficient
                        if (lc == 0xFFu) continue;                                        // zero coefficient
                        const uint32_t p = x ? (uint32_t)s_exp[lx + lc] : 0u;
                        acc[j][q] ^= p << (8 * byte);
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < RCH; ++j)
            if (r0 + j < m) st16(dst + (uint64_t)(r0 + j) * a.pitch, make_uint4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]));
    }
}

// ------------------------------------------------------------------ reconstruct
// One wave per group.  The group's erasure pattern (ballot over its n marks) indexes a
// host-built LUT to a decode record: e, stale mask, survivor shard ids, erased data ids,
// then e x k perm tables (gf256.cpp: build_decode_record).  In explicit mode the host
// supplies the record offset per group instead (n > 24 or host-side marks).
// Record (RecordLayout, qfec_internal.hpp): [0] e, [surv_off + c] survivor shard id (0..n-1),
// [lost_off + j] erased data index, [coff + j*k + c] byte offset of the coefficient's table in
// the 256-entry table (bit 0 on column 0 = stale flag), [hdr + (j*k + c)*QFEC_TAB_STRIDE] perm
// table; dword 5 of (j, 0) = stale flag.

__device__ __forceinline__ const uint8_t* shard_ptr(const ReconArgs& a, uint64_t g, uint32_t s) {
    return s < (uint32_t)a.k ? a.data + g * a.dgs + (uint64_t)s * a.pitch
                             : a.parity + g * a.pgs + (uint64_t)(s - a.k) * a.pitch;
}

__device__ __forceinline__ int group_record(const ReconArgs& a, uint64_t g, int lane) {
    int rec;
    if (a.group_rec) {
        rec = a.group_rec[g];
    } else {
        const int n = a.k + a.m;
        uint32_t mk = 0;
        if (lane < a.k) mk = a.marks[g * (uint64_t)a.k + lane];
        else if (lane < n) mk = a.marks[(uint64_t)a.groups * a.k + g * (uint64_t)a.m + (lane - a.k)];
        const uint64_t bal = __ballot(mk != 0);
        const uint32_t mask = (uint32_t)(bal & ((1ull << n) - 1ull));
        rec = a.lut[mask];
    }
    return __builtin_amdgcn_readfirstlane(rec);
}

// Exactly E rows (E = the group's erased-data count, wave-uniform): all E rows at once,
// selectors formed once per input and shared by the rows, no work on the M - E rows a group
// does not need.  3 random erasures of 13 give e = 1, 2, 3
// with probability 0.10, 0.47, 0.42, so RS(10,3) does 77 % of the all-rows VALU work.
// D = dwords per lane (4: 16-B columns, 2: 8-B columns for rows whose 16-B column count
// leaves a wave mostly idle, e.g. B = 1400: 88 16-B columns on 2 waves, 175 8-B on 3).
template <int D>
__device__ __forceinline__ void ldv(uint32_t (&v)[D], const uint8_t* p) {
    if constexpr (D == 4) {
        const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else if constexpr (D == 3) {  // merged into one global_load_dwordx3 ... nt
        const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
        v[0] = __builtin_nontemporal_load(q);
        v[1] = __builtin_nontemporal_load(q + 1);
        v[2] = __builtin_nontemporal_load(q + 2);
    } else {
        static_assert(D == 2, "4, 3 or 2 dwords per lane");
        const u32x2 t = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
        v[0] = t.x; v[1] = t.y;
    }
}
template <int D>
__device__ __forceinline__ void stv(uint8_t* p, const uint32_t (&v)[D]) {
    if constexpr (D == 4) {
        const u32x4 t = {v[0], v[1], v[2], v[3]};
        __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(p));
    } else if constexpr (D == 3) {
        uint32_t* q = reinterpret_cast<uint32_t*>(p);
        __builtin_nontemporal_store(v[0], q);
        __builtin_nontemporal_store(v[1], q + 1);
        __builtin_nontemporal_store(v[2], q + 2);
    } else {
        const u32x2 t = {v[0], v[1]};
        __builtin_nontemporal_store(t, reinterpret_cast<u32x2*>(p));
    }
}
template <int D>
__device__ __forceinline__ void ldv_plain(uint32_t (&v)[D], const uint8_t* p) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = reinterpret_cast<const uint32_t*>(p)[d];
}

// where a decode record's coefficient tables are: in the 256-entry table of every coefficient
// value, at the byte offsets the record's header lists (RecordLayout::coff).  Reading only the
// record's header keeps the records of all patterns cache-resident (RS(16,4): 4 844 records of
// 2.4 KB would not fit the 4 MB L2; their headers do).  The tables are read through the
// constant address space: loads from it are scalar (SMEM) whatever stores the kernel makes.
typedef const __attribute__((address_space(4))) uint32_t* cptr32;
typedef const __attribute__((address_space(4))) uint8_t* cptr8;
struct RTab {
    cptr32 rec;  // the record: [1] quirk flags, [coff + j*K + c] table byte offsets
    cptr32 offs;
    cptr32 t256;
    __device__ RTab(const uint32_t* r, int coff, const uint32_t* t)
        : rec((cptr32)r), offs((cptr32)r + coff), t256((cptr32)t) {}
    __device__ __forceinline__ cptr32 at(int j, int c, int K) const {
        return (cptr32)((cptr8)t256 + offs[j * K + c]);
    }
    __device__ __forceinline__ bool quirk(int j, int K) const { return (rec[1] >> j) & 1u; }
    __device__ __forceinline__ void load5(int j, int c, int K, uint32_t (&t5)[5]) const {
#pragma unroll
        for (int i = 0; i < 5; ++i) t5[i] = at(j, c, K)[i];
    }
};
// acc[j] ^= sum_c coef(j, c) * x[c] over one column, exact E rows, survivors already in registers
template <int K, int E, int D>
__device__ __forceinline__ void recon_mac_core(const uint32_t (&x)[K][D], uint32_t (&acc)[E][D], const RTab& T) {
#pragma unroll
    for (int c = 0; c + 1 < K; c += 2) {
        Sel sa[D], sb[D];
#pragma unroll
        for (int d = 0; d < D; ++d) { sa[d] = gf_sel(x[c][d]); sb[d] = gf_sel(x[c + 1][d]); }
#pragma unroll
        for (int j = 0; j < E; ++j) {
            uint32_t a5[5], b5[5];
            T.load5(j, c, K, a5);
            T.load5(j, c + 1, K, b5);
#pragma unroll
            for (int d = 0; d < D; ++d) acc[j][d] = mac2(acc[j][d], sa[d], sb[d], a5, b5);
        }
    }
    if (K & 1) {
        Sel sl[D];
#pragma unroll
        for (int d = 0; d < D; ++d) sl[d] = gf_sel(x[K - 1][d]);
#pragma unroll
        for (int j = 0; j < E; ++j) {
            uint32_t t[5];
            T.load5(j, K - 1, K, t);
#pragma unroll
            for (int d = 0; d < D; ++d)
                acc[j][d] = xor3(acc[j][d], pp0(sl[d], t[0], t[1]), pp1(sl[d], t[2], t[3])) ^ pp2(sl[d], t[4]);
        }
    }
}

template <int K, int E, int D>
__device__ __forceinline__ void recon_column_e(const uint8_t* const (&src)[K], uint8_t* __restrict__ data_g,
                                               uint64_t lost_bits, const RTab& T, uint64_t pitch, uint64_t off) {
    uint32_t x[K][D];
#pragma unroll
    for (int c = 0; c < K; ++c) ldv<D>(x[c], src[c] + off);
    uint8_t* dst[E];
    uint32_t acc[E][D];
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const uint32_t l = (uint32_t)__builtin_ctzll(lost_bits);
        lost_bits &= lost_bits - 1;
        dst[j] = data_g + (uint64_t)l * pitch + off;
#pragma unroll
        for (int d = 0; d < D; ++d) acc[j][d] = 0;
        if (T.quirk(j, K)) ldv_plain<D>(acc[j], dst[j]);  // rs.c column-0 quirk
    }
    recon_mac_core<K, E, D>(x, acc, T);
#pragma unroll
    for (int j = 0; j < E; ++j) stv<D>(dst[j], acc[j]);
}

// wave-uniform dispatch on e to the exact-row-count body
template <int K, int M, int D, int E = M>
__device__ __forceinline__ void recon_column_by_e(const uint8_t* const (&src)[K], uint8_t* __restrict__ data_g,
                                                  uint64_t lost_bits, const RTab& T, int e, uint64_t pitch, uint64_t off) {
    if constexpr (E > 1) {
        if (e < E) {
            recon_column_by_e<K, M, D, E - 1>(src, data_g, lost_bits, T, e, pitch, off);
            return;
        }
    }
    recon_column_e<K, E, D>(src, data_g, lost_bits, T, pitch, off);
}

// LUT mode, compile-time K, M.  The survivor set follows from the erasure mask alone --
// it is the lowest K non-erased shard ids (all surviving data, then the first e surviving
// parity rows: module/rs.c:620-629) -- so the shard loads issue right after the ballot,
// while the decode record (coefficients only) is still in flight.
// One wave per 64 columns of a group: a group of `cols` columns gets wpg = ceil(cols / 64)
// waves, all in flight together, no column loop.  IMPL: 2 exact-e rows on 16-B lanes, 3 on
// 8-B lanes, 4 on 12-B lanes; 8 = 3 launched with one group per block (blocks of wpg8 waves),
// so a group's slab waves share a CU and its scalar data (marks, LUT entry, record header,
// tables)
template <int K, int M, int IMPL>
__device__ __forceinline__ void recon_item(const ReconArgs& a, uint8_t* __restrict__ data,
                                           const uint8_t* __restrict__ parity, const uint8_t* __restrict__ marks,
                                           const int32_t* __restrict__ lut, const uint32_t* __restrict__ records,
                                           uint32_t wid, int lane) {
    constexpr int N = K + M;
    const uint32_t wpg = IMPL == 3 ? a.wpg8 : IMPL == 4 ? a.wpg12 : a.wpg;
    const uint64_t g = wid / wpg;
    const uint32_t part = wid - (uint32_t)g * wpg;
    if (g >= a.groups) return;
    uint32_t mk = 0;
    if (lane < K) mk = marks[g * K + lane];
    else if (lane < N) mk = marks[a.groups * K + g * M + (lane - K)];
    const uint64_t mask = __ballot(mk != 0) & ((1ull << N) - 1ull);
    const uint64_t lost_bits = mask & ((1ull << K) - 1ull);
    const int e = __builtin_popcountll(lost_bits);
    if (e == 0) return;
    uint64_t avail = ~mask & ((1ull << N) - 1ull);
    if (__builtin_popcountll(avail) < K) {
        if (part == 0 && lane == 0 && a.failed) atomicAdd(a.failed, 1u);
        return;
    }
    const int rec = ((const __attribute__((address_space(4))) int32_t*)lut)[mask];
    const RTab T{records + rec, a.coff, a.t256};
    const uint64_t pitch = a.pitch;
    uint8_t* data_g = data + g * a.dgs;
    const uint8_t* par_g = parity + g * a.pgs;
    const uint8_t* src[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const uint32_t s = (uint32_t)__builtin_ctzll(avail);
        avail &= avail - 1;
        src[c] = s < (uint32_t)K ? data_g + (uint64_t)s * pitch : par_g + (uint64_t)(s - K) * pitch;
    }
    const uint32_t col = part * 64u + lane;
    if (col < (IMPL == 3 ? a.cols8 : IMPL == 4 ? a.cols12 : a.cols)) {
        if (IMPL == 2) recon_column_by_e<K, M, 4>(src, data_g, lost_bits, T, e, pitch, (uint64_t)col * 16u);
        else if (IMPL == 3) recon_column_by_e<K, M, 2>(src, data_g, lost_bits, T, e, pitch, (uint64_t)col * 8u);
        else recon_column_by_e<K, M, 3>(src, data_g, lost_bits, T, e, pitch, (uint64_t)col * 12u);
    }
}

template <int K, int M, int IMPL_>
__global__ void __launch_bounds__(256) k_reconstruct_perm(ReconArgs a, uint8_t* __restrict__ data,
                                                          const uint8_t* __restrict__ parity,
                                                          const uint8_t* __restrict__ marks,
                                                          const int32_t* __restrict__ lut,
                                                          const uint32_t* __restrict__ records) {
    // __restrict__ parameters: the LUT and records are provably not written by this
    // launch, so their loads stay scalar (SGPR) even across the row loop's stores.
    constexpr int IMPL = IMPL_ == 8 ? 3 : IMPL_;
    const int lane = threadIdx.x & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * (IMPL_ == 8 ? a.wpg8 : 4u) + (threadIdx.x >> 6));
    recon_item<K, M, IMPL>(a, data, parity, marks, lut, records, wid, lane);
}

// runtime k, e; any vector width via the byte path when the layout is not 16-B aligned
template <bool VEC16>
__global__ void __launch_bounds__(256) k_reconstruct_any(ReconArgs a) {
    const int lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (g >= a.groups) return;
    const int rec = group_record(a, g, lane);
    if (rec < 0) {
        if (rec == QFEC_REC_FAIL && lane == 0 && a.failed) atomicAdd(a.failed, 1u);
        return;
    }
    const uint32_t* __restrict__ r = a.records + rec;
    const int e = (int)r[0];
    const int k = a.k;
    const uint32_t* surv = r + a.surv_off;
    const uint32_t* lost = r + a.lost_off;
    const uint32_t* tab = r + a.hdr;

    for (uint32_t col = lane; col < (uint32_t)a.cols; col += 64) {
        for (int j0 = 0; j0 < e; j0 += RCH) {
            if (VEC16) {
                const uint64_t off = (uint64_t)col * 16u;
                uint4 acc[RCH];
#pragma unroll
                for (int j = 0; j < RCH; ++j) {
                    acc[j] = make_uint4(0, 0, 0, 0);
                    const int jj = j0 + j;
                    if (jj < e && tab[(jj * k) * QFEC_TAB_STRIDE + 5])
                        acc[j] = *reinterpret_cast<const uint4*>(a.data + g * a.dgs + (uint64_t)lost[jj] * a.pitch + off);
                }
                for (int c = 0; c < k; ++c) {
                    const uint4 v = ld16(shard_ptr(a, g, surv[c]) + off);
                    Sel s[4];
                    sel16(s, v);
#pragma unroll
                    for (int j = 0; j < RCH; ++j)
                        if (j0 + j < e) gf_mac16(acc[j], s, tab + ((j0 + j) * k + c) * QFEC_TAB_STRIDE);
                }
#pragma unroll
                for (int j = 0; j < RCH; ++j)
                    if (j0 + j < e) st16(a.data + g * a.dgs + (uint64_t)lost[j0 + j] * a.pitch + off, acc[j]);
            } else {
                const uint64_t off = col;
                uint32_t acc[RCH];
#pragma unroll
                for (int j = 0; j < RCH; ++j) {
                    acc[j] = 0;
                    const int jj = j0 + j;
                    if (jj < e && tab[(jj * k) * QFEC_TAB_STRIDE + 5])
                        acc[j] = a.data[g * a.dgs + (uint64_t)lost[jj] * a.pitch + off];
                }
                for (int c = 0; c < k; ++c) {
                    const Sel s = gf_sel((uint32_t)shard_ptr(a, g, surv[c])[off]);
#pragma unroll
                    for (int j = 0; j < RCH; ++j)
                        if (j0 + j < e) {
                            const uint32_t* tc = tab + ((j0 + j) * k + c) * QFEC_TAB_STRIDE;
                            acc[j] ^= gf_mul4(s, tc[0], tc[1], tc[2], tc[3], tc[4]);
                        }
                }
#pragma unroll
                for (int j = 0; j < RCH; ++j)
                    if (j0 + j < e) a.data[g * a.dgs + (uint64_t)lost[j0 + j] * a.pitch + off] = (uint8_t)acc[j];
            }
        }
    }
}

// ------------------------------------------------------------------ utilities

__global__ void __launch_bounds__(256) k_synth_fill(uint8_t* p, uint64_t nbytes, uint64_t seed) {
    const uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t nwords = (nbytes + 7) / 8;
    if (j >= nwords) return;
    uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    const uint64_t base = j * 8;
    if (base + 8 <= nbytes && ((reinterpret_cast<uintptr_t>(p) & 7u) == 0)) {
        *reinterpret_cast<uint64_t*>(p + base) = z;
    } else {
        for (int i = 0; i < 8 && base + i < nbytes; ++i) p[base + i] = (uint8_t)(z >> (8 * i));
    }
}

// streaming probe with the encode's traffic shape (k rows in, m rows out, XOR only):
// the memory-side ceiling the GF arithmetic is measured against.
template <int BS = 256>
__global__ void __launch_bounds__(256) k_probe_xor(EncodeArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * (uint64_t)BS + threadIdx.x;
    if (t >= a.work) return;
    const uint64_t g = fast_div(t, a.cols_div);
    const uint32_t col = (uint32_t)(t - g * (uint64_t)a.cols);
    const uint8_t* src = a.data + g * a.dgs + (uint64_t)col * 16u;
    uint8_t* dst = a.parity + g * a.pgs + (uint64_t)col * 16u;
    uint4 acc = make_uint4(0, 0, 0, 0);
    // up to 16 rows in flight per lane, as the encode has them (a load-then-XOR loop would keep one)
    for (int c0 = 0; c0 < a.k; c0 += 16) {
        uint4 v[16];
#pragma unroll
        for (int c = 0; c < 16; ++c)
            if (c0 + c < a.k) v[c] = ld16(src + (uint64_t)(c0 + c) * a.pitch);
#pragma unroll
        for (int c = 0; c < 16; ++c)
            if (c0 + c < a.k) { acc.x ^= v[c].x; acc.y ^= v[c].y; acc.z ^= v[c].z; acc.w ^= v[c].w; }
    }
    for (int r = 0; r < a.m; ++r) {
        st16(dst + (uint64_t)r * a.pitch, acc);
        acc.x += 1u;
    }
}

// the reconstruct's memory skeleton (calibration, not a codec): the auto body's mapping (8-B lanes,
// one group per block of wpg8 waves) and accesses -- the marks, the K lowest surviving rows
// (data and parity regions), the e erased data rows written -- with XOR in place of the decode
template <int K, int M>
__global__ void __launch_bounds__(256) k_probe_recon(ReconArgs a) {
    constexpr int N = K + M;
    const int lane = threadIdx.x & 63;
    const uint64_t g = blockIdx.x;
    const uint32_t part = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t mk = 0;
    if (lane < K) mk = a.marks[g * K + lane];
    else if (lane < N) mk = a.marks[a.groups * K + g * M + (lane - K)];
    const uint64_t mask = __ballot(mk != 0) & ((1ull << N) - 1ull);
    uint64_t lost = mask & ((1ull << K) - 1ull);
    if (!lost) return;
    uint64_t avail = ~mask & ((1ull << N) - 1ull);
    if (__builtin_popcountll(avail) < K) return;
    const uint32_t col = part * 64u + lane;
    if (col >= a.cols8) return;
    const uint64_t off = (uint64_t)col * 8u;
    uint8_t* data_g = a.data + g * a.dgs;
    const uint8_t* par_g = a.parity + g * a.pgs;
    uint32_t x[K][2];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const uint32_t s = (uint32_t)__builtin_ctzll(avail);
        avail &= avail - 1;
        ldv<2>(x[c], (s < (uint32_t)K ? data_g + (uint64_t)s * a.pitch : par_g + (uint64_t)(s - K) * a.pitch) + off);
    }
    uint32_t acc[2] = {0, 0};
#pragma unroll
    for (int c = 0; c < K; ++c) { acc[0] ^= x[c][0]; acc[1] ^= x[c][1]; }
    while (lost) {
        const uint32_t l = (uint32_t)__builtin_ctzll(lost);
        lost &= lost - 1;
        stv<2>(data_g + (uint64_t)l * a.pitch + off, acc);
        acc[0] += 1u;
    }
}

hipError_t launch_probe_recon(const ReconArgs& a, hipStream_t stream) {
    if (a.groups == 0) return hipSuccess;
    if (a.wpg8 < 1 || a.wpg8 > 4 || a.groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
#define QFEC_PROBE_REC(KK, MM)                                                                                    \
    if (a.k == KK && a.m == MM) {                                                                                 \
        hipLaunchKernelGGL((k_probe_recon<KK, MM>), dim3((unsigned)a.groups), dim3(64 * a.wpg8),               \
                           (size_t)std::max(a.rlds, 0), stream, a);                                               \
        return hipGetLastError();                                                                                 \
    }
    QFEC_PROBE_REC(10, 3)
    QFEC_PROBE_REC(16, 4)
#undef QFEC_PROBE_REC
    return hipErrorInvalidValue;
}

// ------------------------------------------------------------------ launchers

static inline unsigned grid_for(uint64_t work, unsigned block) {
    return (unsigned)((work + block - 1) / block);
}

// auto (encode_impl -1): inputs in halves for k >= 16, where all k inputs in registers cap the
// kernel at 4 waves per SIMD (RS(16,4) B=1400: 1 202 against 1 244 us, 0.98 of the XOR probe;
// RS(10,3) equal within 1 %, profiles/r04c/)
//
// Resident waves (tuning "encode_lds" -1, auto): a dynamic LDS allocation per 256-thread block,
// out of the CU's 160 KiB, holds the blocks per CU below what the registers allow.  Fewer
// concurrent row streams per CU move more bytes per second through HBM (tools/occ_probe.hip: an
// XOR stream of the 10:3 shape at 16 -> 5 waves per CU, 6.03 -> 6.36 TB/s); interleaved A/B of
// the encode on four boxes (profiles/r05ak, r05al, r05am, r05an2):
//   all k inputs in registers (impl 0), k = 10, rows >= 512 B, >= 16 384 blocks: 2 blocks = 8 waves
//                                                 per CU  RS(10,3) B=512/1024/1400 +2-5 % at 100 000
//                                                 groups, +0.7 % at 50 000, -4 % / -7 % at 25 000 /
//                                                 17 000 (the last round of blocks runs half empty)
//   inputs in halves (impl 2), rows <= 1 KiB:   6 blocks = 24 waves per CU  RS(16,4), RS(20,4) B=1024 +1-4 %
//   otherwise, k >= 3:                          4 blocks = 16 waves per CU  RS(3,2), (4,2), (5,3), (6,2),
//                                                 (8,4), (12,4), RS(16,4) B=1400 +1-5 %, RS(10,3) B=64 equal
//   k <= 2: none (RS(2,1) 2 % slower capped)
// Launches under 8 192 blocks keep every slot (RS(16,4) B=1400 at 31 250 groups, config 4's share
// of 8 ranks, 10 742 blocks: +4 %, profiles/r05ap).  The reconstruct and the
// datagram kernels lose with any cap (profiles/r05ak, r05al) and have none.
// One-wave blocks (tuning "encode_block" -1 auto, 64, 256; round 6): the all-rows body of k = 10
// on rows of at least 1 KiB (64 16-B columns) in launches of >= 2^21 lanes runs 64-thread blocks
// held at 10 per CU (16 KiB of LDS each): RS(10,3) B=1024 100 000 groups 200.1 / 201.4 against
// 209.2 / 210.4 us, B=1400 276.6 against 292.0, 50 000 groups 102.1 against 109.5; equal at 25 000
// and 17 000 groups; B=512 not better (108-111 against 108), so left out (interleaved,
// profiles/r06_enc/).  Blocks of one wave leave a CU's slots one wave at a time and can hold 10
// waves, which 4-wave blocks cannot (8 or 12).  RS(16,4) (the two-half body), RS(4,2), RS(16,4)
// B=1024 and every reconstruct body measured no gain from them (r06z_*): 256-thread blocks there.
// Over the other templated shapes (r06ak): RS(8,2) 172.5 -> 156.2 us and RS(6,2) 132.6 -> 124.6 at
// 10 per CU; RS(8,4), RS(12,4) and RS(5,3) within 1.3 %: the rule takes 6 <= k <= 10 with m <= 3.
// Only where every wave starts on a 128-B line (pitch, group strides and bases multiples of 128 B):
// one-wave blocks are dealt round-robin over the XCDs, and a line two waves share is then fetched
// and written from two L2s -- RS(10,3) B=1500 (1 504-B pitch) ran 253.8 against 227.3 us on them,
// while B=1400 (1 408 = 11 x 128) and B=2048 / 4096 gain 5.4 / 2.4 / 3.4 % (r06av).
static inline unsigned enc_block(const EncodeArgs& a, int K, int im) {
    if (a.block == 64 || a.block == 256) return (unsigned)a.block;
    const bool lines = (a.pitch % 128 == 0) && (a.dgs % 128 == 0) && (a.pgs % 128 == 0) &&
                       ((reinterpret_cast<uintptr_t>(a.data) | reinterpret_cast<uintptr_t>(a.parity)) % 128 == 0);
    return im == 0 && K >= 6 && K <= 10 && a.m <= 3 && a.cols >= 64 && lines && a.work >= (8192ull << 8) ? 64u : 256u;
}

static inline size_t enc_lds(const EncodeArgs& a, int K, int im, unsigned grid, unsigned bs = 256) {
    if (a.lds >= 0) return (size_t)a.lds;
    if (bs == 64) return 16384;
    if (grid < 8192 || K <= 2) return 0;
    if (im == 0 && K == 10) return a.cols >= 32 && grid >= 16384 ? 65536 : 40960;
    if (im == 2 && a.cols <= 64) return 27000;
    return 40960;
}

#define QFEC_ENC_CASE(KK, MM)                                                                 \
    if (a.k == KK && a.m == MM) {                                                             \
        const int im = a.impl < 0 ? (KK >= 16 ? 2 : 0) : a.impl;                              \
        const unsigned bs = enc_block(a, KK, im);                                             \
        const size_t lds = enc_lds(a, KK, im, grid, bs);                                      \
        if (im == 2 && bs == 64)                                                              \
            hipLaunchKernelGGL((k_encode_perm_halves<KK, MM, 64>), dim3(grid_for(a.work, 64)), dim3(64), lds, stream, a); \
        else if (im == 2)                                                                     \
            hipLaunchKernelGGL((k_encode_perm_halves<KK, MM>), dim3(grid), dim3(256), lds, stream, a); \
        else if (bs == 64)                                                                    \
            hipLaunchKernelGGL((k_encode_perm<KK, MM, 64>), dim3(grid_for(a.work, 64)), dim3(64), lds, stream, a); \
        else                                                                                  \
            hipLaunchKernelGGL((k_encode_perm<KK, MM>), dim3(grid), dim3(256), lds, stream, a);  \
        return hipGetLastError();                                                             \
    }

hipError_t launch_encode(const EncodeArgs& a, int variant, hipStream_t stream) {
    if (a.work == 0) return hipSuccess;
    const unsigned grid = grid_for(a.work, 256);
    if (!a.vec16) {
        hipLaunchKernelGGL(k_encode_bytes, dim3(grid), dim3(256), 0, stream, a);
        return hipGetLastError();
    }
    if (variant == QFEC_VARIANT_LDSLOG_I) {
        hipLaunchKernelGGL(k_encode_ldslog, dim3(grid), dim3(256), 0, stream, a);
        return hipGetLastError();
    }
    QFEC_ENC_CASE(10, 3)
    QFEC_ENC_CASE(16, 4)
    QFEC_ENC_CASE(4, 2)
    QFEC_ENC_CASE(2, 1)
    QFEC_ENC_CASE(2, 2)
    QFEC_ENC_CASE(3, 1)
    QFEC_ENC_CASE(3, 2)
    QFEC_ENC_CASE(4, 1)
    QFEC_ENC_CASE(5, 1)
    QFEC_ENC_CASE(5, 3)
    QFEC_ENC_CASE(6, 2)
    QFEC_ENC_CASE(7, 1)
    QFEC_ENC_CASE(8, 2)
    QFEC_ENC_CASE(8, 4)
    QFEC_ENC_CASE(12, 4)
    QFEC_ENC_CASE(20, 4)
    hipLaunchKernelGGL(k_encode_perm_any, dim3(grid), dim3(256), 0, stream, a);
    return hipGetLastError();
}

#define QFEC_REC_LAUNCH(KK, MM, AR)                                                                        \
    do {                                                                                                   \
        const dim3 blk(AR == 8 ? 64u * a.wpg8 : 256u), grd(AR == 8 ? (unsigned)a.groups : pgrid);          \
        hipLaunchKernelGGL((k_reconstruct_perm<KK, MM, AR>), grd, blk, 0, stream, a, a.data, a.parity, a.marks, \
                           a.lut, a.records);                                                              \
    } while (0)

#define QFEC_REC_CASE(KK, MM)                                                      \
    if (a.k == KK && a.m == MM) {                                                  \
        /* auto: exact-e rows on 12-B lanes for k*m <= 30 where they fill the waves */ \
        /* best, on 8-B lanes where those fill better than 16-B lanes or for k >= 10 */ \
        /* (one group per block where a group is at most 4 waves), else 16-B lanes   */ \
        const bool wide8 = KK >= 10 && fill8 >= fill16 - 0.01;                     \
        int im = a.impl < 0 ? (KK * MM <= 30 && lanes12 ? 4 : (lanes8 || wide8) ? 3 : 2) : a.impl; \
        if (im == 4 && !lanes12_ok) im = 2;                                        \
        const unsigned pgrid = im == 3 ? pgrid8 : im == 4 ? pgrid12 : pgrid16;     \
        /* 8-B lanes run one group per block where a group is at most 4 waves: its slab */ \
        /* waves share a CU (RS(16,4) B=1400: 1 218 against 1 224 us, r03blk)            */ \
        if (im == 3 && a.impl < 0) im = 8;                                         \
        if (im == 8 && (a.wpg8 < 1 || a.wpg8 > 4)) im = 3;                         \
        if (im == 8) QFEC_REC_LAUNCH(KK, MM, 8);                                   \
        else if (im == 4) QFEC_REC_LAUNCH(KK, MM, 4);                              \
        else if (im == 3) QFEC_REC_LAUNCH(KK, MM, 3);                              \
        else QFEC_REC_LAUNCH(KK, MM, 2);                                           \
        return hipGetLastError();                                                  \
    }

hipError_t launch_reconstruct(const ReconArgs& a, hipStream_t stream) {
    if (a.groups == 0) return hipSuccess;
    const unsigned grid = grid_for(a.groups, 4);
    if (!a.vec16) {
        hipLaunchKernelGGL((k_reconstruct_any<false>), dim3(grid), dim3(256), 0, stream, a);
        return hipGetLastError();
    }
    if (a.group_rec) {  // explicit (host-record) mode: survivors come from the record
        hipLaunchKernelGGL((k_reconstruct_any<true>), dim3(grid), dim3(256), 0, stream, a);
        return hipGetLastError();
    }
    const uint64_t waves = a.groups * (uint64_t)std::max(std::max(a.wpg, a.wpg8), a.wpg12);
    if (waves > 0xFFFFFFFFull) return hipErrorInvalidValue;  // caller chunks batches
    const unsigned pgrid16 = grid_for(a.groups * (uint64_t)a.wpg, 4);
    const unsigned pgrid8 = grid_for(a.groups * (uint64_t)a.wpg8, 4);
    const unsigned pgrid12 = grid_for(a.groups * (uint64_t)a.wpg12, 4);
    // 12-B lanes write no further than the 16-B columns do (B = 1400: 117 x 12 = 1404 <= 1408)
    const bool lanes12_ok = a.cols12 * 12u <= a.cols * 16u;
    // 12-B lanes where they fill as well as 8-B lanes with 2/3 of the waves; for small k*m
    // only (profiles/r01ak_recon_lanes.txt: RS(10,3) B=1400 12-B 5 918 vs 8-B 5 734 GB/s,
    // RS(16,4) B=1400 4 964 vs 5 108 -- at 90 VGPRs the 12-B body drops to 5 waves/SIMD)
    const double fill16 = (double)a.cols / (64.0 * a.wpg), fill8 = (double)a.cols8 / (64.0 * a.wpg8),
                 fill12 = (double)a.cols12 / (64.0 * a.wpg12);
    const bool lanes12 = lanes12_ok && fill12 > fill16 + 0.1 && fill12 >= fill8 - 0.01;
    // 8-B lanes when they fill the group's waves clearly better than 16-B lanes
    const bool lanes8 = fill8 > fill16 + 0.1;
    // and for k >= 10 even when 16-B lanes fill their waves: the 8-B body's lower register
    // count (RS(10,3) 69 vs 103 VGPRs: 7 vs 4 waves/SIMD) wins when reconstruct runs right
    // after an encode, as in the bench step (profiles/r01aq_pairs.txt: RS(10,3) B=1024
    // +2.5 %, RS(16,4) B=1024 +6.2 %; RS(4,2) B=1024 loses 6.7 % and stays on 16-B lanes)
    QFEC_REC_CASE(10, 3)
    QFEC_REC_CASE(16, 4)
    QFEC_REC_CASE(4, 2)
    QFEC_REC_CASE(2, 1)
    QFEC_REC_CASE(3, 2)
    QFEC_REC_CASE(8, 4)
    QFEC_REC_CASE(12, 4)
    QFEC_REC_CASE(5, 3)
    QFEC_REC_CASE(6, 2)
    QFEC_REC_CASE(7, 1)
    QFEC_REC_CASE(8, 2)
    QFEC_REC_CASE(20, 4)
    hipLaunchKernelGGL((k_reconstruct_any<true>), dim3(grid), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_synth_fill(uint8_t* p, uint64_t nbytes, uint64_t seed, hipStream_t stream) {
    const uint64_t nwords = (nbytes + 7) / 8;
    if (!nwords) return hipSuccess;
    hipLaunchKernelGGL(k_synth_fill, dim3(grid_for(nwords, 256)), dim3(256), 0, stream, p, nbytes, seed);
    return hipGetLastError();
}

hipError_t launch_probe_xor(const EncodeArgs& a, hipStream_t stream) {
    if (a.work == 0) return hipSuccess;
    // the ceiling of the shape: the encode's block rule for that k; on one-wave blocks the stream
    // runs best at 6 per CU (27 000 B of LDS: 199.8 us against 218.5 at the encode's 10, 211.5 at
    // 4-wave blocks x 2, RS(10,3) B=1024, profiles/r06_enc/r06ab_g100.log)
    const unsigned grid = grid_for(a.work, 256);
    const unsigned bs = enc_block(a, a.k, 0);
    const size_t lds = bs == 64 && a.lds < 0 ? 27000 : enc_lds(a, a.k, 0, grid, bs);
    if (bs == 64)
        hipLaunchKernelGGL(k_probe_xor<64>, dim3(grid_for(a.work, 64)), dim3(64), lds, stream, a);
    else
        hipLaunchKernelGGL(k_probe_xor<>, dim3(grid), dim3(256), lds, stream, a);
    return hipGetLastError();
}

}  // namespace qfec
