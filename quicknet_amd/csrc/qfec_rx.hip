// qfec_rx.hip -- the fused FEC datagram receive on the device (round 5): qfec_unpack_datagrams
// and qfec_unpack_frames for the templated (k, m) shapes, one wave per group.
//
// What a group's wave does is the reference's receive side for a whole group at once
// (skywind3000/QuickNet network/FecCodecBuf.cpp, network/NetFecCodec.cpp,
// network/ProtocolBasic.cpp):
//   * unpack_fec_head (FecCodecBuf.cpp:334-411) on each of the n received rows: tag, header
//     length, (n, k, ik), shard size; frames first pass RecvPacket's length / cmd tests
//     (ProtocolBasic.cpp:155-199);
//   * the decode of the missing data shards from the first k valid rows in group order
//     (NetFecCodec.cpp:504-528, add_packet_fec_buf; == module/rs.c:620-629), with the shard
//     checksum of every row it uses verified (a row that fails is dropped and the group decoded
//     again without it), and the rows it does not use checksummed too;
//   * dec_src_pkt_info (FecCodecBuf.cpp:109-133) on every data row: payload size, payload
//     checksum, status.
// Outputs are those of the staged path (k_parse_wire -> reconstruct -> k_check_payloads) and of
// the receive kernel of rounds 2-4 (retired in round 5), byte for byte.
//
// The design is set by what bounds the receive: issue, not bytes (profiles/r05a: the
// round-4 kernel issued 1 775 VALU + 1 137 SALU per group and its waves waited on memory half of
// their lifetime, while the same memory skeleton runs at 0.68 of 8 TB/s).  So, per group:
//   * every survivor row is loaded once as 16-B (or 8-B) lanes over [0, 1024) (or [0, 512));
//     the last 16 bytes of a 1 040-B (528-B) shard pitch are not a fifth (third) dword of every
//     lane -- which costs a whole wave instruction per survivor and per decoded row for 4 busy
//     lanes -- but ONE lane-mapped tail: lane 4c + d holds dword d of survivor c's tail, and the
//     decoded tail dwords come from per-lane perm tables (vector loads of the record) and an XOR
//     reduction over the survivor lanes;
//   * the MAC is compiled per exact erased-row count e (no per-row branch inside it);
//   * row checksums are reduced four values at a time (v_permlane32_swap, v_permlane16_swap,
//     four DPP steps, one readlane each) instead of six DPP steps per value;
//   * survivor bookkeeping is scalar (SGPR arrays over the compile-time K), no lane-shuffled
//     plan vectors;
//   * the K data rows are staged in LDS and stored as one flat byte range (LDSW), so a row
//     that ends mid-line does not leave a 64-B line written in two parts.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "qfec_device.hpp"
#include "qfec_internal.hpp"

// QFEC_RX_ABLATE (measurement builds only, tools/rx_stage_ablate.sh; results are wrong in such
// a build): bit 0 drops the decode MAC, bit 1 the row checksums (byte sums and their totals),
// bit 2 the row stores, bit 3 the unaligned row loads (rows read at a 16-B-aligned offset).
// The SQ counters of each build against the full one give the per-stage instruction counts.
#ifndef QFEC_RX_ABLATE
#define QFEC_RX_ABLATE 0
#endif
namespace qfec {

namespace {

__device__ __forceinline__ uint32_t rlane(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }

__device__ __forceinline__ uint32_t get_byte4(const uint4& v, int pos) {
    const uint32_t w = (pos >> 2) == 0 ? v.x : (pos >> 2) == 1 ? v.y : (pos >> 2) == 2 ? v.z : v.w;
    return (w >> (8 * (pos & 3))) & 0xFFu;
}

// the low nb bytes of x (nb clamped to 0..4)
__device__ __forceinline__ uint32_t keep_dw(uint32_t x, int nb) {
    const int c = min(max(nb, 0), 4);
    return c >= 4 ? x : x & ((1u << (8 * c)) - 1u);
}

// bytes [s, s + 16) of the 32-byte window (a | b), s in {0, 4, 8, 12} wave-uniform (frame prefixes)
__device__ __forceinline__ uint4 window32(const uint4& a, const uint4& b, int s) {
    switch (s >> 2) {
        case 0: return a;
        case 1: return make_uint4(a.y, a.z, a.w, b.x);
        case 2: return make_uint4(a.z, a.w, b.x, b.y);
        default: return make_uint4(a.w, b.x, b.y, b.z);
    }
}

__device__ __forceinline__ uint32_t sad(uint32_t x, uint32_t acc) { return __builtin_amdgcn_sad_u8(x, 0u, acc); }

// sum of the 16 lanes of each row, in every lane of the row
__device__ __forceinline__ uint32_t row_total(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    return v;
}

// 64-lane totals of T values at once: pairs of registers trade halves (v_permlane32_swap: rows 2-3
// of the first with rows 0-1 of the second), pairs of those trade rows (v_permlane16_swap: odd rows
// of the first with even rows of the second), each 16-lane row is summed by DPP, and one readlane
// per value takes the total.  3.5 VALU per value against 7 for a DPP reduction of each.
template <int T>
__device__ __forceinline__ void totals(const uint32_t (&v)[T], uint32_t (&out)[T]) {
    constexpr int Q = (T + 3) / 4;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint32_t x = v[4 * q], y = 4 * q + 1 < T ? v[4 * q + 1] : 0u;
        const uint32_t z = 4 * q + 2 < T ? v[4 * q + 2] : 0u, w = 4 * q + 3 < T ? v[4 * q + 3] : 0u;
        const auto s0 = __builtin_amdgcn_permlane32_swap(x, y, false, false);  // [x_lo, y_lo], [x_hi, y_hi]
        const auto s1 = __builtin_amdgcn_permlane32_swap(z, w, false, false);
        const uint32_t a = s0[0] + s0[1];                                      // x: lanes 0-31, y: 32-63
        const uint32_t b = s1[0] + s1[1];                                      // z, w
        const auto s2 = __builtin_amdgcn_permlane16_swap(a, b, false, false);  // [a_r0, b_r0, a_r2, b_r2], [a_r1, b_r1, a_r3, b_r3]
        const uint32_t r = row_total(s2[0] + s2[1]);                            // rows: x, z, y, w
        out[4 * q] = rlane(r, 0);
        if (4 * q + 1 < T) out[4 * q + 1] = rlane(r, 32);
        if (4 * q + 2 < T) out[4 * q + 2] = rlane(r, 16);
        if (4 * q + 3 < T) out[4 * q + 3] = rlane(r, 48);
    }
}

// lanes of one wave hand data to each other through LDS: make the order explicit
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_total(uint32_t v) {
    v = row_total(v);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return rlane(v, 63);
}

__device__ __forceinline__ uint32_t head_bytes_sum(uint32_t w0, int head) {
    return __builtin_amdgcn_sad_u8(head == 4 ? w0 : (w0 & 0xFFFFu), 0u, 0u);
}

// XOR over the lanes {l, l + 4, l + 8, ...} of the first 4 * CR lanes: every lane with the same
// l & 3 gets the XOR (the tail's dword d of a decoded row over the survivor lanes)
template <int CR>
__device__ __forceinline__ uint32_t xor_over_c(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    if constexpr (CR > 4) v ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);  // lane ^ 16
    if constexpr (CR > 8) v ^= (uint32_t)__builtin_amdgcn_ds_bpermute((int)((threadIdx.x ^ 32u) * 4u), (int)v);
    return v;
}

extern __shared__ uint4 rx_stage[];

// one row chunk of NV dwords
template <int NV>
struct Chunk {
    uint32_t d[NV];
};

template <int NV>
__device__ __forceinline__ void load_chunk(Chunk<NV>& x, const uint8_t* p) {
    if constexpr (NV == 4) {
        uint4 w;
        __builtin_memcpy(&w, p, 16);
        x.d[0] = w.x; x.d[1] = w.y; x.d[2] = w.z; x.d[3] = w.w;
    } else {
        uint2 w;
        __builtin_memcpy(&w, p, 8);
        x.d[0] = w.x; x.d[1] = w.y;
    }
}

// store a row chunk into the LDS stage (16- or 8-B aligned) or into HBM (non-temporal)
template <int NV, bool LDSW>
__device__ __forceinline__ void store_chunk(uint8_t* p, const Chunk<NV>& x) {
    if constexpr (LDSW) {
        if constexpr (NV == 4) *reinterpret_cast<uint4*>(p) = make_uint4(x.d[0], x.d[1], x.d[2], x.d[3]);
        else *reinterpret_cast<uint2*>(p) = make_uint2(x.d[0], x.d[1]);
    } else {
        if constexpr (NV == 4) {
            const u32x4 w = {x.d[0], x.d[1], x.d[2], x.d[3]};
            __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
        } else {
            const u32x2 w = {x.d[0], x.d[1]};
            __builtin_nontemporal_store(w, reinterpret_cast<u32x2*>(p));
        }
    }
}

template <bool LDSW>
__device__ __forceinline__ void store_dw(uint8_t* p, uint32_t x) {
    if constexpr (LDSW) *reinterpret_cast<uint32_t*>(p) = x;
    else __builtin_nontemporal_store(x, reinterpret_cast<uint32_t*>(p));
}

// v with lane l replaced by the wave-uniform x: one v_writelane_b32 (l a constant after unrolling)
__device__ __forceinline__ uint32_t wlanei(uint32_t v, int l, uint32_t x) {
    const uint32_t xs = (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
    asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(xs), "i"(l));
    return v;
}

// OR of v over the wave (every lane)
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    v |= (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);                       // lane ^ 16
    return rlane(v, 0) | rlane(v, 32);
}

// where a row chunk goes: LDSW stages the K data rows in LDS (row r byte b at stage offset
// r * P + b - X) and stores them flat afterwards, except bytes [0, X) of row 0, which go to HBM
// directly -- X ends on a 64-B line of HBM, so the split costs no partial line, and the stage is
// 976 B or more smaller than K * P: RS(10,13) with 1 KiB payloads then fits 16 groups per CU (LDS)
// instead of 15.  Without LDSW every row goes straight to HBM.
template <bool LDSW>
struct RowOut {
    uint8_t* hbm;  // the group's first data row
    int P, X;
    template <int NV>
    __device__ __forceinline__ void chunk(uint32_t r, int pos, const Chunk<NV>& x) const {
        if constexpr (LDSW) {
            if (r == 0 && pos < X) store_chunk<NV, false>(hbm + pos, x);
            else store_chunk<NV, true>(reinterpret_cast<uint8_t*>(rx_stage) + ((int)r * P + pos - X), x);
        } else {
            store_chunk<NV, false>(hbm + r * P + pos, x);
        }
    }
    __device__ __forceinline__ void dw(uint32_t r, int pos, uint32_t x) const {  // pos >= X
        if constexpr (LDSW) store_dw<true>(reinterpret_cast<uint8_t*>(rx_stage) + ((int)r * P + pos - X), x);
        else store_dw<false>(hbm + r * P + pos, x);
    }
};

// the round's plan: wave-uniform scalars, and per survivor c the values lane c of three VGPRs holds
template <int K, int M>
struct Plan {
    uint32_t v_soff;   // lane c: survivor c's shard offset in the group's rows (row * wp + fp + hdr)
    uint32_t v_srow;   // lane c: survivor c's row | size << 16
    uint32_t v_smm;    // lane c: survivor c's frame XOR word
    int ns, e;
    bool dec;
    uint32_t lostw;    // decoded row j: bits 4j..4j+3
    uint32_t zero_rows;
    int min_size;
    const uint32_t* tab;  // the record's perm tables [j][c][8]
};

// one pass over row bytes [base, base + 64 * 4 * NV) (lanes at pos >= P idle): survivor chunks
// loaded, frames un-XORed, masked past each survivor's size where the pass reaches it, summed;
// the E decoded rows' chunks by the MAC; data survivors and decoded chunks stored; decoded sums.
// On the first pass, dword 0 of every survivor (lane c of v_w0) and decoded row (dw0[j]).
template <int K, int M, int NV, bool FR, bool LDSW, int E>
__device__ __forceinline__ void rx_pass(const Plan<K, M>& pl, const uint8_t* __restrict__ wire_g, const RowOut<LDSW>& out,
                                        int P, int base, bool first, int head, uint32_t (&dsum)[K],
                                        uint32_t (&psl)[M], uint32_t& v_w0, uint32_t (&dw0)[M], int lane) {
    const int pos = base + 4 * NV * lane;
    const bool act = pos < P;
    const int pend = min(P, base + 256 * NV);
    Chunk<NV> x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
#pragma unroll
        for (int d = 0; d < NV; ++d) x[c].d[d] = 0;
        if (c < pl.ns && act)
            load_chunk<NV>(x[c], wire_g + ((QFEC_RX_ABLATE & 8) ? rlane(pl.v_soff, c) & ~15u : rlane(pl.v_soff, c)) + pos);
    }
    if constexpr (FR) {
#pragma unroll
        for (int c = 0; c < K; ++c)
            if (c < pl.ns) {
                const uint32_t mm = act ? rlane(pl.v_smm, c) : 0u;
#pragma unroll
                for (int d = 0; d < NV; ++d) x[c].d[d] ^= mm;
            }
    }
    if (pend > pl.min_size) {  // some survivor's shard ends inside this pass: keep [0, size)
#pragma unroll
        for (int c = 0; c < K; ++c)
            if (c < pl.ns) {
                const int sz = (int)(rlane(pl.v_srow, c) >> 16);
                if (pend > sz) {
#pragma unroll
                    for (int d = 0; d < NV; ++d) x[c].d[d] = keep_dw(x[c].d[d], sz - pos - 4 * d);
                }
            }
    }
    if constexpr (!(QFEC_RX_ABLATE & 2)) {
#pragma unroll
        for (int c = 0; c < K; ++c) {
            uint32_t s = dsum[c];
#pragma unroll
            for (int d = 0; d < NV; ++d) s = sad(x[c].d[d], s);
            dsum[c] = s;
        }
    }
    Chunk<NV> acc[E > 0 ? E : 1];
#pragma unroll
    for (int j = 0; j < (E > 0 ? E : 1); ++j)
#pragma unroll
        for (int d = 0; d < NV; ++d) acc[j].d[d] = 0;
    if constexpr (E > 0 && !(QFEC_RX_ABLATE & 1)) {
#pragma unroll
        for (int c = 0; c < K; ++c) {
            Sel sc[NV];
#pragma unroll
            for (int d = 0; d < NV; ++d) sc[d] = gf_sel(x[c].d[d]);
            uint32_t toff = (uint32_t)(c * QFEC_TAB_STRIDE);
            asm volatile("" : "+s"(toff));  // this column's tables fetched here, not all E * K up front
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const uint32_t* t = pl.tab + toff + j * K * QFEC_TAB_STRIDE;
                const uint32_t t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3], t4 = t[4];
#pragma unroll
                for (int d = 0; d < NV; ++d)
                    acc[j].d[d] = xor3(acc[j].d[d], pp0(sc[d], t0, t1), pp1(sc[d], t2, t3)) ^ pp2(sc[d], t4);
            }
        }
#pragma unroll
        for (int j = 0; j < E; ++j)
#pragma unroll
            for (int d = 0; d < NV; ++d) asm volatile("" : "+v"(acc[j].d[d]));
    }
    if (first) {  // lane 0, dword 0 of the first pass: bytes 0-3 of every row, [size][cksum]
        uint32_t w = 0;
#pragma unroll
        for (int c = 0; c < K; ++c) w = wlanei(w, c, rlane(x[c].d[0], 0));
        v_w0 = w;
#pragma unroll
        for (int j = 0; j < E; ++j) dw0[j] = rlane(acc[j].d[0], 0);
    }
    if (act && !(QFEC_RX_ABLATE & 4)) {
#pragma unroll
        for (int c = 0; c < K; ++c) {
            const uint32_t r = rlane(pl.v_srow, c) & 0xFFFFu;
            if (c < pl.ns && r < (uint32_t)K) out.chunk(r, pos, x[c]);
        }
#pragma unroll
        for (int j = 0; j < E; ++j) out.chunk((pl.lostw >> (4 * j)) & 0xFu, pos, acc[j]);
        if (pl.zero_rows) {
            Chunk<NV> z;
#pragma unroll
            for (int d = 0; d < NV; ++d) z.d[d] = 0;
            for (uint32_t zr = pl.zero_rows; zr; zr &= zr - 1) out.chunk(__builtin_ctz(zr), pos, z);
        }
    }
#pragma unroll
    for (int j = 0; j < ((QFEC_RX_ABLATE & 2) ? 0 : E); ++j) {
        const int hi = head + (int)(dw0[j] & 0xFFFFu);  // payload end of decoded row j
        uint32_t s = psl[j];
        if (pend > hi) {
#pragma unroll
            for (int d = 0; d < NV; ++d) s = sad(act ? keep_dw(acc[j].d[d], hi - pos - 4 * d) : 0u, s);
        } else {
#pragma unroll
            for (int d = 0; d < NV; ++d) s = sad(acc[j].d[d], s);
        }
        psl[j] = s;
    }
}

// the lane-mapped 16-B tail of every row (P = F * 64 * 4 * NV + 16): lane 4c + d holds dword d of
// survivor c's tail; decoded tail dwords from per-lane perm tables (vector loads of the record,
// L2-resident) and an XOR over the survivor lanes.  Returns the survivors' tail sums in tsum
// (lanes 4c..4c+3) and the decoded rows' in tpsl (lanes 4j..4j+3)
template <int K, int M, int NV, bool FR, bool LDSW, int E>
__device__ __forceinline__ void rx_tail(const Plan<K, M>& pl, const uint8_t* __restrict__ wire_g, const RowOut<LDSW>& out, int P,
                                        int tb, int head, const uint32_t (&dw0)[M], uint32_t& tsum, uint32_t& tpsl,
                                        int lane) {
    const int tc = lane >> 2, td = lane & 3;
    // survivor tc's offset, row | size << 16 and XOR word, from lane tc
    const uint32_t off = (uint32_t)__builtin_amdgcn_ds_bpermute(tc * 4, (int)pl.v_soff);
    const uint32_t srw = (uint32_t)__builtin_amdgcn_ds_bpermute(tc * 4, (int)pl.v_srow);
    const bool tact = tc < pl.ns;
    const int pos = tb + 4 * td;
    uint32_t x = 0;
    if (tact) __builtin_memcpy(&x, wire_g + off + pos, 4);
    if constexpr (FR) {
        const uint32_t mm = (uint32_t)__builtin_amdgcn_ds_bpermute(tc * 4, (int)pl.v_smm);
        x ^= tact ? mm : 0u;
    }
    x = keep_dw(x, (int)(srw >> 16) - pos);
    tsum = sad(x, 0u);
    if (tact && (srw & 0xFFFFu) < (uint32_t)K) out.dw(srw & 0xFFFFu, pos, x);
    tpsl = 0;
    if constexpr (E > 0) {
        uint32_t res = 0, hi_lane = 0;
        const Sel s = gf_sel(x);
#pragma unroll
        for (int j = 0; j < E; ++j) {
            const uint32_t* t = pl.tab + (j * K + min(tc, K - 1)) * QFEC_TAB_STRIDE;
            uint4 t03;
            __builtin_memcpy(&t03, t, 16);
            const uint32_t t4 = t[4];
            uint32_t r = gf_mul4(s, t03.x, t03.y, t03.z, t03.w, t4);
            r = xor_over_c<K>(tact ? r : 0u);
            res = tc == j ? r : res;
            hi_lane = tc == j ? (uint32_t)(head + (int)(dw0[j] & 0xFFFFu)) : hi_lane;
        }
        if (tc < E) {
            out.dw((pl.lostw >> (4 * tc)) & 0xFu, pos, res);
            tpsl = sad(keep_dw(res, (int)hi_lane - pos), 0u);
        }
    }
    if (pl.zero_rows && lane < 4)
        for (uint32_t zr = pl.zero_rows; zr; zr &= zr - 1) out.dw(__builtin_ctz(zr), pos, 0u);
}

}  // namespace

// K data + M check rows per group, NV dwords per lane (4: 16-B lanes, 2: 8-B), FR: the rows are
// ProtocolUdp frames with an fp-byte prefix (4, or 12 with the Session's conv/hid), LDSW: the K
// data rows staged in LDS (K * pitch bytes of dynamic LDS) and stored as one flat range
template <int K, int M, int NV, bool FR, bool LDSW>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NV == 4 ? 4 : 5))) k_rx(WireArgs a, const uint8_t* __restrict__ wire, const int32_t* __restrict__ wire_len,
                                           const int32_t* __restrict__ lut, const uint32_t* __restrict__ records,
                                           uint32_t rec_hdr, uint8_t* __restrict__ shards, FrameRecv fr, int fp) {
    static_assert(M >= 1 && K + M <= 15 && K + M <= 32, "datagram groups: n <= 15");
    constexpr int N = K + M;
    constexpr int A = 256 * NV;  // row bytes per full pass
    const int lane = threadIdx.x;
    const uint64_t g = blockIdx.x;
    const int P = (int)a.pitch;
    const uint32_t wp = (uint32_t)a.wire_pitch;
    const uint8_t* wire_g = wire + g * (uint64_t)N * wp;
    uint8_t* const out_hbm = shards + g * a.group_stride;
    // bytes [0, X) of row 0 straight to HBM, up to a 64-B line of HBM (16-B lanes, rows >= 1 KiB)
    const int X = (LDSW && NV == 4 && P >= 1024) ? 1024 - (int)(((uintptr_t)out_hbm + 1024) & 63) : 0;
    const RowOut<LDSW> out{out_hbm, P, X};
    if (!FR) fp = 0;
    // ---- headers (unpack_fec_head's checks, FecCodecBuf.cpp:334-411), one row per lane
    int len = 0, hdr = 11, size = 0;
    uint32_t stated = 0;
    bool okh = false;
    // frames, lane r, packed so little stays live through the passes: bits 0-12 the prefix and
    // header byte sum, 13-15 RecvPacket's verdict before the checksum, 16-23 the XOR byte, 24-31 the
    // stated frame check byte
    uint32_t v_fs = 0, v_fx = 0;
    int fst = 0;                  // frames, lane r: RecvPacket's verdict before the checksum
    if (lane < N) {
        len = wire_len[g * N + lane];
        int dlen = len;
        uint4 h = make_uint4(0u, 0u, 0u, 0u);
        const bool rd = len > 0;  // a row not received is not read
        if constexpr (FR) {
            const uint8_t* frow = wire_g + (uint64_t)lane * wp;
            uint4 f0 = make_uint4(0u, 0u, 0u, 0u), f1 = f0;
            if (rd) {
                f0 = *reinterpret_cast<const uint4*>(frow);
                f1 = *reinterpret_cast<const uint4*>(frow + 16);
            }
            v_fx = (get_byte4(f0, 0) ^ fr.gmask ^ 0x5Au) & 0xFFu;
            const uint32_t mmx = v_fx * 0x01010101u;
            const uint4 u0 = make_uint4(f0.x ^ mmx, f0.y ^ mmx, f0.z ^ mmx, f0.w ^ mmx);
            const uint4 u1 = make_uint4(f1.x ^ mmx, f1.y ^ mmx, f1.z ^ mmx, f1.w ^ mmx);
            h = window32(u0, u1, fp);
            dlen = len - fp;
            const uint32_t cmd = get_byte4(u0, 2);
            fst = len < fp ? 1 : len > (int)wp ? 4 : (cmd & 0xE0u) != 0xA0u ? 3 : 0;
            uint32_t pre = cmd + get_byte4(u0, 3);  // frame bytes 2 .. fp - 1
            if (fp == 12) {
                pre = __builtin_amdgcn_sad_u8(u0.y, 0u, __builtin_amdgcn_sad_u8(u0.z, 0u, pre));
                if (fr.conv_hid && fst == 0) {
                    fr.conv_hid[2 * (g * N + lane)] = u0.y;
                    fr.conv_hid[2 * (g * N + lane) + 1] = u0.z;
                }
            }
            v_fs = pre | ((uint32_t)fst << 13) | (v_fx << 16) | (get_byte4(u0, 1) << 24);
        } else {
            if (rd) h = *reinterpret_cast<const uint4*>(wire_g + (uint64_t)lane * wp);
        }
        const uint32_t tag = get_byte4(h, 0);
        hdr = tag == 0xED ? 13 : 11;
        const uint32_t ikn = get_byte4(h, 9) | (get_byte4(h, 10) << 8);
        okh = fst == 0 && dlen >= 11 && dlen <= (int)wp && (tag == 0xEC || tag == 0xED) && dlen >= hdr &&
              (int)(ikn & 0xF) == N && (int)((ikn >> 4) & 0xF) == K && (int)((ikn >> 8) & 0xF) == lane && dlen - hdr <= P;
        size = okh ? dlen - hdr : 0;
        stated = get_byte4(h, 11) | (get_byte4(h, 12) << 8);
        if constexpr (FR) {  // the datagram header's bytes join the frame checksum
            uint32_t hs = 0;
            const uint32_t hw[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
            for (int d = 0; d < 4; ++d) hs = sad(keep_dw(hw[d], hdr - 4 * d), hs);
            v_fs += hs;
        }
    }
    const uint32_t rowmask = (1u << N) - 1u, kmask = (1u << K) - 1u;
    const uint32_t good = (uint32_t)__ballot(okh) & rowmask;
    const uint32_t summed = (uint32_t)__ballot(okh && hdr == 13) & rowmask;
    // frames: rows the FEC header rejected whose RecvPacket checksum still decides their verdict
    const uint32_t chk_rows = FR ? (uint32_t)__ballot(lane < N && (fst == 0 || fst == 3) && !okh) & rowmask : 0u;
    const uint32_t v_ss = (uint32_t)size | (stated << 16);  // lane r: row r's size | stated checksum
    // the first round's record, requested before the loads (used unless a survivor fails)
    const bool rec0_needed = __builtin_popcount(good) >= K && (~good & kmask);
    const int rec0 = rec0_needed ? __builtin_amdgcn_readfirstlane(lut[~good & rowmask]) : 0;
    const int head = a.checksum ? 4 : 2;
    const int F = P / A, R = P - F * A;  // full passes, remainder (a multiple of 16)
    const bool tail = F > 0 && R == 16 && K <= 16;
    const int passes = F + ((R > 0 && !tail) ? 1 : 0);
    uint32_t bad = 0, verified = 0, fbad = 0;
    Plan<K, M> pl;
    uint32_t v_w0 = 0, v_dt = 0;  // lane c: survivor c's dword 0, shard byte total; lane K + j: decoded row j's
    uint32_t dw0[M];
    for (int round = 0;; ++round) {
        // the lane id and the group's row base made opaque per round: nothing lane- or
        // address-derived is hoisted out of this (nearly always single-trip) loop to stay live in
        // registers across it
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const uint8_t* wg = wire_g;
        asm volatile("" : "+s"(wg));
        // ---- plan: survivors = the lowest K good rows (or the good data rows if too few)
        const uint32_t avail = good & ~bad;
        const uint32_t lost_data = ~avail & kmask;
        const bool recoverable = __builtin_popcount(avail) >= K;
        pl.zero_rows = recoverable ? 0u : lost_data;
        uint32_t take = recoverable ? avail : (avail & kmask);
        pl.ns = min(__builtin_popcount(take), K);
        // ln c < ns: the c-th set bit of take (its rank among the set bits below it)
        const uint32_t myrow_bits = ln < N ? (take & ((1u << ln) - 1u)) : 0u;
        const int rank = __builtin_popcount(myrow_bits);
        const bool mine = ln < N && ((take >> ln) & 1u) && rank < K;
        // push row r's (offset, row | size, XOR word) to ln rank (ds_permute: ln rank receives)
        const uint32_t my_off = (uint32_t)ln * wp + (uint32_t)fp + (((summed >> ln) & 1u) ? 13u : 11u);
        const uint32_t my_srow = (uint32_t)ln | ((uint32_t)size << 16);
        const int dst = mine ? rank * 4 : 63 * 4;  // lanes not sending write ln 63 (never a survivor)
        pl.v_soff = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(mine ? my_off : 0u));
        pl.v_srow = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(mine ? my_srow : 0u));
        pl.v_smm = FR ? (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(mine ? ((v_fs >> 16) & 0xFFu) * 0x01010101u : 0u)) : 0u;
        const uint32_t sv = (uint32_t)__ballot(mine);  // the survivors' rows
        {  // smallest survivor size (lanes c < ns of v_srow)
            uint32_t msz = ln < pl.ns ? (pl.v_srow >> 16) : (uint32_t)P;
            msz = min(msz, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)msz, 0xB1, 0xF, 0xF, false));
            msz = min(msz, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)msz, 0x4E, 0xF, 0xF, false));
            msz = min(msz, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)msz, 0x124, 0xF, 0xF, false));
            msz = min(msz, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)msz, 0x128, 0xF, 0xF, false));
            msz = min(msz, (uint32_t)__builtin_amdgcn_ds_swizzle((int)msz, 0x401F));
            pl.min_size = (int)min(rlane(msz, 0), rlane(msz, 32));
        }
        pl.dec = recoverable && lost_data;
        pl.e = 0;
        pl.lostw = 0;
        pl.tab = records;
        if (pl.dec) {
            const int rec = round == 0 ? rec0 : __builtin_amdgcn_readfirstlane(lut[~avail & rowmask]);
            pl.tab = records + rec + rec_hdr;
            pl.e = (int)records[rec];
#pragma unroll
            for (int j = 0; j < M; ++j)
                if (j < pl.e) pl.lostw |= (records[rec + 4 + K + j] & 0xFu) << (4 * j);
        }
        // ---- the byte passes, the MAC compiled for the exact erased-row count
        uint32_t dsum[K], psl[M], tsum = 0, tpsl = 0;
#pragma unroll
        for (int c = 0; c < K; ++c) dsum[c] = 0;
#pragma unroll
        for (int j = 0; j < M; ++j) psl[j] = 0, dw0[j] = 0;
        auto run = [&](auto ec) {
            constexpr int E = decltype(ec)::value;
            for (int q = 0; q < passes; ++q)
                rx_pass<K, M, NV, FR, LDSW, E>(pl, wg, out, P, A * q, q == 0, head, dsum, psl, v_w0, dw0, ln);
            if (tail) rx_tail<K, M, NV, FR, LDSW, E>(pl, wg, out, P, A * F, head, dw0, tsum, tpsl, ln);
        };
        switch (pl.e) {
            case 0: run(std::integral_constant<int, 0>{}); break;
            case 1: run(std::integral_constant<int, 1>{}); break;
            case 2: if constexpr (M >= 2) run(std::integral_constant<int, 2>{}); break;
            case 3: if constexpr (M >= 3) run(std::integral_constant<int, 3>{}); break;
            default: if constexpr (M >= 4) run(std::integral_constant<int, M>{}); break;
        }
        // ---- totals: survivors' shard sums (ln c of v_dt), decoded rows' payload-prefix sums
        // (ln K + j)
        {
            uint32_t v[K + M], o[K + M];
#pragma unroll
            for (int c = 0; c < K; ++c) v[c] = dsum[c];
#pragma unroll
            for (int j = 0; j < M; ++j) v[K + j] = psl[j];
            if constexpr (QFEC_RX_ABLATE & 2) {
#pragma unroll
                for (int i = 0; i < K + M; ++i) o[i] = v[i];
            } else {
                totals<K + M>(v, o);
            }
            uint32_t t = 0;
#pragma unroll
            for (int i = 0; i < K + M; ++i) t = wlanei(t, i, o[i]);
            if (tail) {  // plus the ln-mapped tails: ln 4c (4j) holds survivor c's (decoded j's) quad
                tsum += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)tsum, 0xB1, 0xF, 0xF, false);
                tsum += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)tsum, 0x4E, 0xF, 0xF, false);
                tpsl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)tpsl, 0xB1, 0xF, 0xF, false);
                tpsl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)tpsl, 0x4E, 0xF, 0xF, false);
                const uint32_t ts = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (4 * ln), (int)tsum);
                const uint32_t tp = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (4 * (ln - K)), (int)tpsl);
                t += ln < K ? ts : (ln < K + M ? tp : 0u);
            }
            v_dt = t;
        }
        // ---- verdicts on the survivors (a survivor whose header or shard checksum fails is dropped and
        // the group decoded from the next valid row, NetFecCodec.cpp:504-528), ln c for survivor c
        uint32_t nb = 0, vr = 0, fb = 0;  // ln c: row bit if bad / verified / frame-checksum bad
        {
            const uint32_t r = pl.v_srow & 0xFu, rb_bit = 1u << r;
            // row r's stated checksum and frame sum, to ln c (every ln takes part in the permutes)
            const uint32_t sr = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * r), (int)v_ss);
            const uint32_t fs = FR ? (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * r), (int)v_fs) : 0u;
            if (ln < pl.ns) {
                bool rb = false, rv = false;
                if ((summed >> r) & 1u) {
                    // (ablation builds whose sums are wrong by construction take every row as good)
                    if (!(QFEC_RX_ABLATE & 10) && (v_dt & 0xFFFFu) != (sr >> 16)) rb = true;
                    else rv = true;
                }
                if constexpr (FR) {  // ProtocolUdp::CheckSum over frame bytes 2.. (ProtocolBasic.cpp:80-87)
                    const uint32_t s = (fs & 0x1FFFu) + v_dt;
                    if ((~((s >> 16) + (s & 0xFFFFu)) & 0xFFu) != (fs >> 24)) {
                        rb = true;
                        fb = rb_bit;
                    } else {
                        rv = true;
                    }
                }
                nb = rb ? rb_bit : 0u;
                vr = !rb && rv ? rb_bit : 0u;
            }
        }
        const uint32_t newbad = wave_or(nb);
        verified |= wave_or(vr);
        if constexpr (FR) fbad |= wave_or(fb);
        if (!(newbad & sv)) {
            // rows only checksummed (frames: every good row, for its frame checksum): rare -- they
            // exist only where more than k rows arrived; one row at a time over the wave
            uint32_t extra = good & (FR ? rowmask : summed) & ~sv & ~verified & ~bad;
            while (extra) {
                const int r = __builtin_ctz(extra);
                extra &= extra - 1;
                const int xs = (int)(rlane(v_ss, r) & 0xFFFFu);
                const uint32_t mm = FR ? ((rlane(v_fs, r) >> 16) & 0xFFu) * 0x01010101u : 0u;
                const uint8_t* row = wg + (uint64_t)r * wp + fp + (((summed >> r) & 1u) ? 13u : 11u);
                uint32_t s = 0;
                for (int p0 = 0; p0 < P; p0 += 1024) {
                    const int pos = p0 + 16 * ln;
                    if (pos < P) {
                        uint4 w;
                        __builtin_memcpy(&w, row + pos, 16);
                        s = sad(keep_dw(w.x ^ mm, xs - pos), s);
                        s = sad(keep_dw(w.y ^ mm, xs - pos - 4), s);
                        s = sad(keep_dw(w.z ^ mm, xs - pos - 8), s);
                        s = sad(keep_dw(w.w ^ mm, xs - pos - 12), s);
                    }
                }
                const uint32_t t = wave_total(s);
                bool rb = ((summed >> r) & 1u) && (t & 0xFFFFu) != (rlane(v_ss, r) >> 16);
                if constexpr (FR) {
                    const uint32_t fs = rlane(v_fs, r), s2 = (fs & 0x1FFFu) + t;
                    if ((~((s2 >> 16) + (s2 & 0xFFFFu)) & 0xFFu) != (fs >> 24)) {
                        rb = true;
                        fbad |= 1u << r;
                    }
                }
                if (rb) bad |= 1u << r;
                else verified |= 1u << r;
            }
            break;
        }
        bad |= newbad;
    }
    if constexpr (LDSW) {  // the K data rows, staged whole, as one flat range
        wave_lds_sync();
        const int total = K * P;
        for (int o = X + 16 * lane; o < total; o += 1024) st16(out_hbm + o, rx_stage[(o - X) >> 4]);
    }
    // ---- per-row results
    const uint32_t okrows = good & ~bad;
    if (lane < N) {
        const bool ok = (okrows >> lane) & 1u;
        if (lane < K) a.marks[g * K + lane] = ok ? 0 : 1;
        else a.marks[a.groups * K + g * M + (lane - K)] = ok ? 0 : 1;
        if (a.rx_size) a.rx_size[g * N + lane] = ok ? (int)(v_ss & 0xFFFFu) : -1;
    }
    // dec_src_pkt_info (FecCodecBuf.cpp:109-133): lane c < ns for survivor c (when a data row),
    // lane K + j for decoded row j; each writes its own row's status
    int orow = -1;
    uint32_t w0 = v_w0, ps = 0;
    if (lane < pl.ns) {
        orow = (int)(pl.v_srow & 0xFFFFu);
        if (orow >= K) orow = -1;
        ps = v_dt - head_bytes_sum(w0, head);
    } else if (lane >= K && lane < K + pl.e) {
        orow = (int)((pl.lostw >> (4 * (lane - K))) & 0xFu);
        ps = v_dt;
    }
    {  // decoded rows' dword 0 into lanes K + j
        uint32_t wd = w0;
#pragma unroll
        for (int j = 0; j < M; ++j) wd = wlanei(wd, K + j, dw0[j]);
        if (lane >= K && lane < K + pl.e) {
            w0 = wd;
            ps = v_dt - head_bytes_sum(w0, head);
        }
    }
    // a received payload shorter than its shard (bytes after the payload inside the datagram): the
    // payload checksum over [head, head + p) exactly, one such row at a time (rare)
    if (a.checksum) {
        const int sz = (int)(pl.v_srow >> 16), p = (int)(w0 & 0xFFFFu);
        uint32_t need = (uint32_t)__ballot(lane < pl.ns && orow >= 0 && head + p < sz);
        while (need) {
            const int c = __builtin_ctz(need);
            need &= need - 1;
            const int csz = (int)(rlane(pl.v_srow, c) >> 16), cp = (int)(rlane(w0, c) & 0xFFFFu);
            const uint8_t* row = wire_g + rlane(pl.v_soff, c);
            const uint32_t mm = FR ? rlane(pl.v_smm, c) : 0u;
            uint32_t s = 0;
            for (int p0 = 0; p0 < csz; p0 += 1024) {
                const int pos = p0 + 16 * lane;
                if (pos < csz) {
                    uint4 w;
                    __builtin_memcpy(&w, row + pos, 16);
                    const uint32_t wd[4] = {w.x ^ mm, w.y ^ mm, w.z ^ mm, w.w ^ mm};
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        const int b = pos + 4 * d;  // keep bytes in [head, min(sz, head + p))
                        s = sad(keep_dw(wd[d], min(csz, head + cp) - b) ^ keep_dw(wd[d], head - b), s);
                    }
                }
            }
            s = wave_total(s);
            ps = lane == c ? s : ps;
        }
    }
    if (orow >= 0) {
        const int psz = (int)(w0 & 0xFFFFu);
        const int st = psz >= a.dec_pkt_size || head + psz > P ? -1
                       : a.checksum && (ps & 0xFFFFu) != (w0 >> 16) ? -1 : head;
        a.status[g * K + orow] = st;
        a.psize[g * K + orow] = psz;
    }
    if constexpr (FR) {
        // frames the FEC header rejected were not read by the passes: their RecvPacket checksum,
        // one row at a time over the wave (only malformed rows come here).  A bad cmd is judged
        // after the checksum, as RecvPacket does (ProtocolBasic.cpp:167-196), so those rows too.
        uint32_t chk = chk_rows;
        while (chk) {
            const int r = __builtin_ctz(chk);
            chk &= chk - 1;
            const int flen = wire_len[g * N + r];
            const uint32_t mmr = ((rlane(v_fs, r) >> 16) & 0xFFu) * 0x01010101u;
            const uint8_t* row = wire_g + (uint64_t)r * wp;
            uint32_t s = 0;
            for (int pos = 16 * lane; pos < flen; pos += 1024) {
                const uint4 w = *reinterpret_cast<const uint4*>(row + pos);
                const uint32_t wd[4] = {w.x ^ mmr, w.y ^ mmr, w.z ^ mmr, w.w ^ mmr};
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const int b = pos + 4 * d;  // bytes [2, flen)
                    s = sad(keep_dw(wd[d], flen - b) ^ keep_dw(wd[d], 2 - b), s);
                }
            }
            s = wave_total(s);
            if ((~((s >> 16) + (s & 0xFFFFu)) & 0xFFu) != (rlane(v_fs, r) >> 24)) fbad |= 1u << r;
        }
        if (fr.status && lane < N)
        {
            const int fs0 = (int)((v_fs >> 13) & 7u);
            fr.status[g * N + lane] = fs0 == 1 || fs0 == 4 ? fs0 : ((fbad >> lane) & 1u) ? 2 : fs0;
        }
    }
    // data rows no survivor or decoded row wrote: 0, or -2 where lost and not recoverable
    const uint32_t written = wave_or(orow >= 0 ? 1u << orow : 0u);
    if (lane < K && !((written >> lane) & 1u)) {
        a.status[g * K + lane] = ((pl.zero_rows >> lane) & 1u) ? -2 : 0;
        a.psize[g * K + lane] = 0;
    }
}

// ------------------------------------------------------------------ launch
namespace {

template <int K, int M, bool FR>
hipError_t rx_launch(const WireArgs& a, const int32_t* lut, const uint32_t* records, uint32_t rec_hdr, hipStream_t s,
                     const FrameRecv& fr, int fp) {
    // lanes: 16 B where one pass covers most of the row (768 < pitch <= 1280), else 8 B.  The K
    // data rows are staged in LDS where that leaves at least 3/4 of the waves per CU the registers
    // allow (16 on 16-B lanes, 24 on 8-B lanes; 160 KiB of LDS per CU): RS(10,13) 1 KiB payloads
    // yes, 1 400-B payloads (14 KB per group) no.  Tuning "wire_rx" 2..5 forces a lane width and
    // staging (tests hold every form to the same outputs)
    const int rx = tuning().wire_rx;
    const size_t stage = (size_t)K * a.pitch;
    bool lanes16 = a.pitch > 768 && a.pitch <= 1280;
    const size_t lds_waves = (size_t)(160 * 1024) / stage, reg_waves = lanes16 ? 16 : 24;
    bool ldsw = stage <= 16384 && 4 * lds_waves >= 3 * reg_waves;
    if (rx >= 2) {
        lanes16 = rx <= 3;
        ldsw = (rx == 2 || rx == 4) && stage <= 65536;
    }
    const dim3 grid((unsigned)a.groups), block(64);
    // (the first 976..1024 bytes of row 0 bypass the stage on 16-B lanes, rows >= 1 KiB)
    const size_t sh = ldsw ? stage - (lanes16 && a.pitch >= 1024 ? 976 : 0) : 0;
    if (lanes16) {
        if (ldsw) hipLaunchKernelGGL((k_rx<K, M, 4, FR, true>), grid, block, sh, s, a, a.wire, (const int32_t*)a.wire_len, lut, records, rec_hdr, a.shards, fr, fp);
        else hipLaunchKernelGGL((k_rx<K, M, 4, FR, false>), grid, block, sh, s, a, a.wire, (const int32_t*)a.wire_len, lut, records, rec_hdr, a.shards, fr, fp);
    } else {
        if (ldsw) hipLaunchKernelGGL((k_rx<K, M, 2, FR, true>), grid, block, sh, s, a, a.wire, (const int32_t*)a.wire_len, lut, records, rec_hdr, a.shards, fr, fp);
        else hipLaunchKernelGGL((k_rx<K, M, 2, FR, false>), grid, block, sh, s, a, a.wire, (const int32_t*)a.wire_len, lut, records, rec_hdr, a.shards, fr, fp);
    }
    return hipGetLastError();
}

template <bool FR>
hipError_t rx_dispatch(const WireArgs& a, const int32_t* lut, const uint32_t* records, uint32_t rec_hdr, hipStream_t s,
                       bool* launched, const FrameRecv& fr, int fp) {
    *launched = false;
    if (!a.groups) return hipSuccess;
    if (a.groups > 0x7FFFFFFFull || a.pitch >= 32768 || (uint64_t)(a.k + a.m) * a.wire_pitch >= 65536) return hipSuccess;
#define QFEC_RX_CASE(KK, MM)                                                  \
    if (a.k == KK && a.m == MM) {                                             \
        *launched = true;                                                     \
        return rx_launch<KK, MM, FR>(a, lut, records, rec_hdr, s, fr, fp);    \
    }
    QFEC_RX_CASE(10, 3)
#ifndef QFEC_RX_ONLY_10_3
    QFEC_RX_CASE(4, 1)
    QFEC_RX_CASE(4, 2)
    QFEC_RX_CASE(2, 2)
    QFEC_RX_CASE(3, 1)
    QFEC_RX_CASE(3, 2)
    QFEC_RX_CASE(5, 1)
    QFEC_RX_CASE(5, 3)
    QFEC_RX_CASE(7, 1)
    QFEC_RX_CASE(8, 4)
#endif
#undef QFEC_RX_CASE
    return hipSuccess;
}

}  // namespace

hipError_t launch_rx(const WireArgs& a, const int32_t* lut, const uint32_t* records, uint32_t rec_hdr, hipStream_t s,
                     bool* launched) {
    return rx_dispatch<false>(a, lut, records, rec_hdr, s, launched, FrameRecv{}, 0);
}

hipError_t launch_unpack_frames(const WireArgs& a, const FrameRecv& fr, int fp, const int32_t* lut,
                                const uint32_t* records, uint32_t rec_hdr, hipStream_t s, bool* launched) {
    return rx_dispatch<true>(a, lut, records, rec_hdr, s, launched, fr, fp);
}

}  // namespace qfec
