// qfec_wire.hip -- FEC datagram batches on the device.
//
// The network layer wraps every packet in a shard and every shard in a datagram
// (skywind3000/QuickNet network/FecCodecBuf.cpp):
//   shard    = [size u16][cksum16(payload) u16, if checksum][payload], zero-filled
//              (set_fec_enc_buf, :66-103); check shards are fec_encode(.., groupMax)
//              over the k shards (get_fec_encoded_pkt, :137-156)
//   datagram = [0xEC | 0xED][sent u32][src u32][n | k<<4 | ik<<8 : u16]
//              [cksum16(shard bytes) u16, if 0xED][shard bytes]   (pack_fec_head, :274-328)
// with sequence numbers as zfec_pack_input assigns them (network/NetFecCodec.cpp:96-172).
// The receive side reverses it: unpack_fec_head (:334-411, the shard checksum drops a
// corrupted datagram), decode of the missing data shards, dec_src_pkt_info (:109-133).
//
// These kernels do that for whole batches of groups in HBM, around the GF kernels of
// qfec_kernels.hip.  Layout: shards[G][n][pitch] (data rows then check rows per group),
// wire[G][n][wire_pitch].  Every kernel is a byte stream (HBM-bound, integer work): one
// wave per row, one lane per 16-byte chunk, byte sums by v_sad_u8 and a wave reduction.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "qfec_device.hpp"
#include "qfec_internal.hpp"

namespace qfec {

namespace {

// unaligned 16-byte load (gfx950 global loads accept byte-aligned addresses)
__device__ __forceinline__ uint4 ldu16(const uint8_t* p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

__device__ __forceinline__ void st16a(uint8_t* p, const uint4& v) { *reinterpret_cast<uint4*>(p) = v; }

// 0xFF in every byte position b of dword t (bytes 4t..4t+3 of a chunk) with lo <= b < hi
__device__ __forceinline__ uint32_t byte_mask(int lo, int hi, int t) {
    const int a = min(max(lo - 4 * t, 0), 4), b = min(max(hi - 4 * t, 0), 4);
    if (b <= a) return 0u;
    const uint64_t mb = (1ull << (8 * b)) - 1ull, ma = (1ull << (8 * a)) - 1ull;
    return (uint32_t)(mb & ~ma);
}

__device__ __forceinline__ uint4 mask16(uint4 v, int lo, int hi) {
    v.x &= byte_mask(lo, hi, 0);
    v.y &= byte_mask(lo, hi, 1);
    v.z &= byte_mask(lo, hi, 2);
    v.w &= byte_mask(lo, hi, 3);
    return v;
}

__device__ __forceinline__ uint32_t sum16(const uint4& v, uint32_t acc) {
    acc = __builtin_amdgcn_sad_u8(v.x, 0u, acc);
    acc = __builtin_amdgcn_sad_u8(v.y, 0u, acc);
    acc = __builtin_amdgcn_sad_u8(v.z, 0u, acc);
    return __builtin_amdgcn_sad_u8(v.w, 0u, acc);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// put byte value b at byte position pos (0..15) of chunk v
__device__ __forceinline__ void put_byte(uint4& v, int pos, uint32_t b) {
    const uint32_t sh = 8u * (pos & 3), m = ~(0xFFu << sh), x = (b & 0xFFu) << sh;
    switch (pos >> 2) {
        case 0: v.x = (v.x & m) | x; break;
        case 1: v.y = (v.y & m) | x; break;
        case 2: v.z = (v.z & m) | x; break;
        default: v.w = (v.w & m) | x; break;
    }
}

__device__ __forceinline__ uint32_t get_byte(const uint4& v, int pos) {
    const uint32_t w = (pos >> 2) == 0 ? v.x : (pos >> 2) == 1 ? v.y : (pos >> 2) == 2 ? v.z : v.w;
    return (w >> (8 * (pos & 3))) & 0xFFu;
}

// datagram store: non-temporal or write-back (tuning "wire_store_nt"), wave-uniform flag
__device__ __forceinline__ void stw(uint8_t* p, const uint4& v, int nt) {
    if (nt) st16(p, v);
    else st16a(p, v);
}

// c ? a : b per dword (a ?: on the struct is lowered through scratch memory)
__device__ __forceinline__ uint4 pick16(bool c, const uint4& a, const uint4& b) {
    return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

// bytes [s, s + 16) of the 32-byte window (a | b), s in [0, 16)
__device__ __forceinline__ uint4 window(const uint4& a, const uint4& b, int s) {
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t r = (uint32_t)(s & 3);
    uint4 o;
    switch (s >> 2) {  // wave-uniform
        case 0:
            o = make_uint4(__builtin_amdgcn_alignbyte(w[1], w[0], r), __builtin_amdgcn_alignbyte(w[2], w[1], r),
                           __builtin_amdgcn_alignbyte(w[3], w[2], r), __builtin_amdgcn_alignbyte(w[4], w[3], r));
            break;
        case 1:
            o = make_uint4(__builtin_amdgcn_alignbyte(w[2], w[1], r), __builtin_amdgcn_alignbyte(w[3], w[2], r),
                           __builtin_amdgcn_alignbyte(w[4], w[3], r), __builtin_amdgcn_alignbyte(w[5], w[4], r));
            break;
        case 2:
            o = make_uint4(__builtin_amdgcn_alignbyte(w[3], w[2], r), __builtin_amdgcn_alignbyte(w[4], w[3], r),
                           __builtin_amdgcn_alignbyte(w[5], w[4], r), __builtin_amdgcn_alignbyte(w[6], w[5], r));
            break;
        default:
            o = make_uint4(__builtin_amdgcn_alignbyte(w[4], w[3], r), __builtin_amdgcn_alignbyte(w[5], w[4], r),
                           __builtin_amdgcn_alignbyte(w[6], w[5], r), __builtin_amdgcn_alignbyte(w[7], w[6], r));
            break;
    }
    return o;
}

}  // namespace

// ------------------------------------------------------------------ send: shards
// One wave per data row (g, i): shard = [size][cksum][payload][0 ...] over the full pitch.
__global__ void __launch_bounds__(256) k_build_shards(WireArgs a) {
    const uint64_t row = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (row >= a.groups * (uint64_t)a.k) return;
    const int lane = threadIdx.x & 63;
    const uint64_t g = row / (uint32_t)a.k;
    const int i = (int)(row - g * (uint32_t)a.k);
    const int size = a.sizes[row];
    const uint8_t* src = a.payload + a.offsets[row];
    uint8_t* dst = a.shards + g * a.group_stride + (uint64_t)i * a.pitch;
    const int head = a.checksum ? 4 : 2;
    const int chunks = (int)(a.pitch / 16);
    uint32_t sum = 0;
    uint4 first = make_uint4(0, 0, 0, 0);
    for (int q = lane; q < chunks; q += 64) {
        const int p0 = 16 * q - head;  // payload byte at chunk byte 0
        uint4 v = make_uint4(0, 0, 0, 0);
        if (q == 0) {
            if (size > 0) {
                const uint4 w = ldu16(src);  // payload bytes [0, 16)
                // shift the payload up by `head` bytes: chunk bytes [head, 16) = payload [0, 16 - head)
                v = window(make_uint4(0, 0, 0, 0), w, 16 - head);
                v = mask16(v, head, head + size);
                sum = sum16(v, sum);
            }
            put_byte(v, 0, (uint32_t)size & 0xFF);
            put_byte(v, 1, ((uint32_t)size >> 8) & 0xFF);
            first = v;
        } else if (p0 < size) {
            v = mask16(ldu16(src + p0), 0, size - p0);
            sum = sum16(v, sum);
        }
        if (q != 0) st16a(dst + 16 * q, v);
    }
    sum = wave_sum(sum);
    if (lane == 0) {
        if (a.checksum) {
            put_byte(first, 2, sum & 0xFF);
            put_byte(first, 3, (sum >> 8) & 0xFF);
        }
        st16a(dst, first);
    }
}

// ------------------------------------------------------------------ send: datagrams
// One wave per datagram (g, j): header + shard bytes [0, len), len = size + head for data
// rows, groupMax (the largest data shard of the group) for check rows.
template <int HDR>
__global__ void __launch_bounds__(256) k_emit_wire(WireArgs a) {
    const uint64_t slot = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    const int n = a.k + a.m;
    if (slot >= a.groups * (uint64_t)n) return;
    const int lane = threadIdx.x & 63;
    const uint64_t g = slot / (uint32_t)n;
    const int j = (int)(slot - g * (uint32_t)n);
    const int head = a.checksum ? 4 : 2;
    int gmax = 0;
    bool ok = true;
    for (int i = 0; i < a.k; ++i) {
        const int sz = a.sizes[g * a.k + i];
        ok = ok && sz >= 0 && sz + head <= (int)a.pitch;
        gmax = max(gmax, sz + head);
    }
    if (!ok) {  // a size the shard pitch cannot hold: the group is not packed
        if (lane == 0) a.wire_len[slot] = -1;
        return;
    }
    const int len = j < a.k ? a.sizes[g * a.k + j] + head : gmax;
    const uint8_t* sh = a.shards + g * a.group_stride + (uint64_t)j * a.pitch;
    uint8_t* out = a.wire + slot * a.wire_pitch;
    // shard byte sum (HDR == 13 carries it)
    uint32_t sum = 0;
    if (HDR == 13)
        for (int q = lane; 16 * q < len; q += 64) sum = sum16(mask16(*reinterpret_cast<const uint4*>(sh + 16 * q), 0, len - 16 * q), sum);
    sum = wave_sum(sum);
    const int total = HDR + len;
    for (int q = lane; 16 * q < total; q += 64) {
        // datagram bytes [16q, 16q + 16) = shard bytes [16q - HDR, 16q + 16 - HDR)
        uint4 v;
        if (q == 0) {
            v = window(make_uint4(0, 0, 0, 0), *reinterpret_cast<const uint4*>(sh), 16 - HDR);
            v = mask16(v, HDR, HDR + len);
            const uint32_t sent = a.seq[2 * g] + (uint32_t)j;
            const uint32_t src = a.seq[2 * g + 1] + (uint32_t)(j < a.k ? j : a.k - 1);
            const uint32_t ikn = ((uint32_t)n | ((uint32_t)a.k << 4) | ((uint32_t)j << 8)) & 0xFFFFu;
            put_byte(v, 0, HDR == 13 ? 0xED : 0xEC);
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                put_byte(v, 1 + b, sent >> (8 * b));
                put_byte(v, 5 + b, src >> (8 * b));
            }
            put_byte(v, 9, ikn);
            put_byte(v, 10, ikn >> 8);
            if (HDR == 13) {
                put_byte(v, 11, sum);
                put_byte(v, 12, sum >> 8);
            }
        } else {
            const uint4 lo = *reinterpret_cast<const uint4*>(sh + 16 * (q - 1));
            const uint4 hi = 16 * q < (int)a.pitch ? *reinterpret_cast<const uint4*>(sh + 16 * q) : make_uint4(0, 0, 0, 0);
            v = mask16(window(lo, hi, 16 - HDR), 0, total - 16 * q);
        }
        st16a(out + 16 * q, v);
    }
    if (lane == 0) a.wire_len[slot] = total;
}

// ------------------------------------------------------------------ receive: datagrams -> shards
// One wave per datagram slot (g, j).  Erased (mark = 1) when absent, not an FEC datagram,
// misrouted (header n/k/ik differ from the slot), or its shard checksum fails -- the
// cases in which network/NetFecCodec.cpp:200-213 drops it.
__global__ void __launch_bounds__(256) k_parse_wire(WireArgs a) {
    const uint64_t slot = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    const int n = a.k + a.m;
    if (slot >= a.groups * (uint64_t)n) return;
    const int lane = threadIdx.x & 63;
    const uint64_t g = slot / (uint32_t)n;
    const int j = (int)(slot - g * (uint32_t)n);
    const uint8_t* in = a.wire + slot * a.wire_pitch;
    uint8_t* sh = a.shards + g * a.group_stride + (uint64_t)j * a.pitch;
    const int len = a.wire_len[slot];
    int ok = len >= 11;
    uint4 h0 = make_uint4(0, 0, 0, 0);
    if (ok) h0 = *reinterpret_cast<const uint4*>(in);
    const uint32_t tag = get_byte(h0, 0);
    const int hdr = tag == 0xED ? 13 : 11;
    ok = ok && (tag == 0xEC || tag == 0xED) && len >= hdr;
    const uint32_t ikn = get_byte(h0, 9) | (get_byte(h0, 10) << 8);
    ok = ok && (int)(ikn & 0xF) == n && (int)((ikn >> 4) & 0xF) == a.k && (int)((ikn >> 8) & 0xF) == j;
    const int size = ok ? len - hdr : 0;
    if (ok && len > (int)a.wire_pitch) ok = 0;
    if (ok && size > (int)a.pitch) ok = 0;
    // rm_checksum (FecCodecBuf.cpp:42-61) over datagram bytes [13, len)
    if (ok && hdr == 13) {
        uint32_t sum = 0;
        for (int q = lane; 16 * q < len; q += 64)
            sum = sum16(mask16(*reinterpret_cast<const uint4*>(in + 16 * q), 13 - 16 * q, len - 16 * q), sum);
        sum = wave_sum(sum) & 0xFFFFu;
        ok = sum == (get_byte(h0, 11) | (get_byte(h0, 12) << 8));
    }
    // shard row = datagram bytes [hdr, len), zero-filled to the pitch
    const int chunks = (int)(a.pitch / 16);
    const int total_q = (len + 15) / 16;
    for (int q = lane; q < chunks; q += 64) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (ok && 16 * q < size) {
            const uint4 lo = *reinterpret_cast<const uint4*>(in + 16 * q);
            const uint4 hi = q + 1 < total_q ? *reinterpret_cast<const uint4*>(in + 16 * (q + 1)) : make_uint4(0, 0, 0, 0);
            v = mask16(window(lo, hi, hdr), 0, size - 16 * q);
        }
        st16a(sh + 16 * q, v);
    }
    if (lane == 0) {
        const uint8_t erased = ok ? 0 : 1;
        if (j < a.k) a.marks[g * a.k + j] = erased;
        else a.marks[a.groups * a.k + g * a.m + (j - a.k)] = erased;
        if (a.rx_size) a.rx_size[slot] = ok ? size : -1;
    }
}

// ------------------------------------------------------------------ receive: payload checks
// One wave per data row (g, i), after reconstruct: dec_src_pkt_info's size and checksum
// checks.  status = payload offset in the shard row (2 or 4), -1 dropped (bad size or
// checksum), -2 lost (erased and the group was not recoverable).
__global__ void __launch_bounds__(256) k_check_payloads(WireArgs a) {
    const uint64_t row = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (row >= a.groups * (uint64_t)a.k) return;
    const int lane = threadIdx.x & 63;
    const uint64_t g = row / (uint32_t)a.k;
    const int i = (int)(row - g * (uint32_t)a.k);
    const int n = a.k + a.m;
    // recoverability of the group (same rule as the reconstruct kernel)
    uint32_t mk = 0;
    if (lane < a.k) mk = a.marks[g * a.k + lane];
    else if (lane < n) mk = a.marks[a.groups * a.k + g * a.m + (lane - a.k)];
    const uint64_t mask = __ballot(mk != 0) & ((1ull << n) - 1ull);
    const bool lost = (mask >> i) & 1ull;
    const bool recoverable = __builtin_popcountll(~mask & ((1ull << n) - 1ull)) >= a.k;
    const uint8_t* sh = a.shards + g * a.group_stride + (uint64_t)i * a.pitch;
    const uint4 h0 = *reinterpret_cast<const uint4*>(sh);
    const int size = (int)(get_byte(h0, 0) | (get_byte(h0, 1) << 8));
    int status = a.checksum ? 4 : 2;
    if (lost && !recoverable) status = -2;
    else if (size >= a.dec_pkt_size || status + size > (int)a.pitch) status = -1;
    else if (a.checksum) {
        uint32_t sum = 0;
        for (int q = lane; 16 * q < 4 + size; q += 64)
            sum = sum16(mask16(*reinterpret_cast<const uint4*>(sh + 16 * q), 4 - 16 * q, 4 + size - 16 * q), sum);
        sum = wave_sum(sum) & 0xFFFFu;
        if (sum != (get_byte(h0, 2) | (get_byte(h0, 3) << 8))) status = -1;
    }
    if (lane == 0) {
        a.status[row] = status;
        a.psize[row] = size;
    }
}

// ------------------------------------------------------------------ send: fused
// Two launches for compile-time (K, M) replace build -> encode -> emit, so the
// [G][n][pitch] shard matrix never exists: HBM traffic is the payload in and the
// datagrams out.  GF arithmetic is bytewise, so check-shard bytes at any shard offset
// come from the data-shard bytes at the same offset; each lane therefore works on one
// 16-B DATAGRAM chunk t = shard bytes [16t - HDR, 16t + 16 - HDR) of all n rows at once,
// with no neighbour exchange.
//  k_pack_body   lanes for t >= 2, flat over (group, t), lpg lanes per group (a multiple
//                of 16): data chunks are straight payload loads; it stores all n datagram
//                chunks and 16-lane partial byte sums (two rows per u32) into `part`.
//  k_pack_head   two lanes per group for t = 0, 1: the only chunks that hold shard bytes
//                0-3 (size, payload checksum) and the datagram header with its checksum,
//                both of which need the whole group's sums.
template <int K, int M>
__device__ __forceinline__ void encode_col(const uint4 (&x)[K], uint4 (&acc)[M], const uint32_t* __restrict__ tab) {
#pragma unroll
    for (int r = 0; r < M; ++r) acc[r] = make_uint4(0, 0, 0, 0);
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
        Sel sl[4];
        sel16(sl, x[K - 1]);
#pragma unroll
        for (int r = 0; r < M; ++r) gf_mac16(acc[r], sl, tab + (r * K + K - 1) * QFEC_TAB_STRIDE);
    }
}

// sum over each aligned 16-lane row, result in every lane of the row (DPP, no LDS)
__device__ __forceinline__ uint32_t row16_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    return v;
}
// v + the value of lane ^ 1
__device__ __forceinline__ uint32_t pair_sum(uint32_t v) {
    return v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}

// A group is packed only if every size is in [0, shard_pitch - head]; otherwise its n
// wire_len entries are -1 and none of its datagram bytes are written.
template <int K, int HEAD>
__device__ __forceinline__ bool group_sizes(const int32_t* __restrict__ sizes, uint64_t g, int pitch, int (&size)[K],
                                            int& gmax) {
    bool ok = true;
    gmax = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        size[i] = sizes[g * K + i];
        ok = ok && size[i] >= 0 && size[i] + HEAD <= pitch;
        gmax = max(gmax, size[i] + HEAD);
    }
    return ok;
}

// UNI: lpg is a multiple of 64, so a wave never straddles groups and the group's sizes,
// offsets and row addresses are wave-uniform (SGPRs); otherwise per lane.
// One lane of the body: datagram chunk t = 2 + rem of group g (live: g exists).  PART_SC1:
// write the partial sums write-through (agent scope), for a same-launch reader.
template <int K, int M, int HDR, bool PART_SC1>
__device__ __forceinline__ void body_lane(const WireArgs& a, const uint8_t* __restrict__ payload,
                                          const int64_t* __restrict__ offsets, const int32_t* __restrict__ sizes,
                                          const uint32_t* __restrict__ tab, uint32_t* __restrict__ part,
                                          uint64_t g, uint32_t rem, bool live, uint32_t lpg) {
    constexpr int N = K + M, HEAD = HDR == 13 ? 4 : 2, P = (N + 1) / 2;
    const int t = 2 + (int)rem;
    const int p = 16 * t - HDR - HEAD;  // payload offset of this chunk's first byte (>= 32 - 17)
    int size[K], gmax = 0;
    bool ok = false;
    if (live) ok = group_sizes<K, HEAD>(sizes, g, (int)a.pitch, size, gmax);
    const bool act = ok && 16 * t < HDR + gmax;
    uint8_t* out = a.wire + g * (uint64_t)N * a.wire_pitch + 16 * t;
    // all K loads back to back (no per-row branch in between): the address is clamped to
    // the packet's end, whose 16 following bytes are readable by contract, and masked after
    uint4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = make_uint4(0, 0, 0, 0);
    if (ok) {
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = ldu16(payload + offsets[g * K + i] + min(p, size[i]));
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = mask16(x[i], 0, size[i] - p);
    }
    uint32_t ps[P];
#pragma unroll
    for (int q = 0; q < P; ++q) ps[q] = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        if (act && p < size[i]) stw(out + (uint64_t)i * a.wire_pitch, x[i], a.store_nt & 1);
        const uint32_t s = sum16(x[i], 0);
        ps[i >> 1] += (i & 1) ? s << 16 : s;
    }
    uint4 acc[M];
#pragma unroll
    for (int r = 0; r < M; ++r) acc[r] = make_uint4(0, 0, 0, 0);
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
        Sel sl[4];
        sel16(sl, x[K - 1]);
#pragma unroll
        for (int r = 0; r < M; ++r) gf_mac16(acc[r], sl, tab + (r * K + K - 1) * QFEC_TAB_STRIDE);
    }
#pragma unroll
    for (int j = 0; j < M; ++j) {
        // check-shard bytes past groupMax are zero: every data chunk is zero there
        if (act) stw(out + (uint64_t)(K + j) * a.wire_pitch, acc[j], a.store_nt & 1);
        const uint32_t s = sum16(acc[j], 0);
        ps[(K + j) >> 1] += ((K + j) & 1) ? s << 16 : s;
    }
    // per-lane sums are <= 16 * 255, a 16-lane row's <= 65280: two rows share a u32 exactly
    const uint32_t R = lpg >> 4;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        const uint32_t v = row16_sum(ps[q]);
        if (live && (rem & 15) == 0) {
            uint32_t* dst = part + (g * R + (rem >> 4)) * P + q;
            if (PART_SC1) __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else *dst = v;
        }
    }
}

template <int K, int M, int HDR, bool UNI>
__global__ void __launch_bounds__(256) k_pack_body(WireArgs a, const uint8_t* __restrict__ payload,
                                                   const int64_t* __restrict__ offsets,
                                                   const int32_t* __restrict__ sizes,
                                                   const uint32_t* __restrict__ tab, uint32_t* __restrict__ part,
                                                   uint64_t g0, uint32_t lanes, uint32_t lpg, DivMagic rows_div) {
    const uint32_t flat = blockIdx.x * 256u + threadIdx.x;
    const bool live = flat < lanes;  // whole 16-lane rows (UNI: waves) are live or not
    uint32_t gl;
    if (UNI) {
        if (!live) return;
        gl = __builtin_amdgcn_readfirstlane((uint32_t)fast_div(flat >> 6, rows_div));
    } else {
        gl = live ? (uint32_t)fast_div(flat >> 4, rows_div) : 0;
    }
    body_lane<K, M, HDR, false>(a, payload, offsets, sizes, tab, part, g0 + gl, flat - gl * lpg, live, lpg);
}

// One lane of the head: datagram chunk t (0 or 1) of group g; lanes 2j, 2j + 1 are a pair
// (same g, same `live`).  PART_SC1: read the partial sums write-through (agent scope).
template <int K, int M, int HDR, bool PART_SC1>
__device__ __forceinline__ void head_lane(const WireArgs& a, const uint8_t* __restrict__ payload,
                                          const int64_t* __restrict__ offsets, const int32_t* __restrict__ sizes,
                                          const uint32_t* __restrict__ tab, const uint32_t* __restrict__ part,
                                          const uint32_t* __restrict__ seq, uint8_t* __restrict__ wire,
                                          int32_t* __restrict__ wire_len, uint64_t g, int t, bool live, uint32_t lpg) {
    constexpr int N = K + M, HEAD = HDR == 13 ? 4 : 2, P = (N + 1) / 2;
    int size[K], gmax = 0;
    bool ok = false;
    if (live) ok = group_sizes<K, HEAD>(sizes, g, (int)a.pitch, size, gmax);
    // every global load up front, addresses clamped to the packet (+16 readable bytes)
    uint4 raw0[K], raw1[K];
    uint32_t tot[N], sent0 = 0, src0 = 0;
#pragma unroll
    for (int r = 0; r < N; ++r) tot[r] = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) raw0[i] = raw1[i] = make_uint4(0, 0, 0, 0);
    if (ok) {
        sent0 = seq[2 * g];
        src0 = seq[2 * g + 1];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const uint8_t* src = payload + offsets[g * K + i];
            raw0[i] = ldu16(src);
            raw1[i] = ldu16(src + min(16 - HEAD, size[i]));
        }
        // the body's 16-lane partial sums: R = lpg / 16 rows of P words
        const uint32_t R = lpg >> 4;
        const uint32_t* pg = part + g * R * P;
        for (uint32_t r0 = 0; r0 < R; r0 += 4) {
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const uint32_t rr = min(r0 + u, R - 1), use = r0 + u < R;
#pragma unroll
                for (int q = 0; q < P; ++q) {
                    uint32_t v = 0;
                    if (use)
                        v = PART_SC1 ? __hip_atomic_load(pg + rr * P + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : pg[rr * P + q];
                    tot[2 * q] += v & 0xFFFF;
                    if (2 * q + 1 < N) tot[2 * q + 1] += v >> 16;
                }
            }
        }
    }
    // this lane's datagram chunk of every data row (t = 0: shard bytes [0, 16 - HDR) after
    // the header; t = 1: shard bytes [16 - HDR, 32 - HDR)), checksum bytes still zero
    uint4 dw[K];
    uint32_t psum[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        uint4 c0 = mask16(window(make_uint4(0, 0, 0, 0), raw0[i], 16 - HEAD), HEAD, HEAD + size[i]);
        put_byte(c0, 0, (uint32_t)size[i]);
        put_byte(c0, 1, (uint32_t)size[i] >> 8);
        const uint4 c1 = mask16(raw1[i], 0, size[i] - (16 - HEAD));
        const int len = size[i] + HEAD;
        const uint4 d0 = mask16(window(make_uint4(0, 0, 0, 0), c0, 16 - HDR), HDR, HDR + len);
        const uint4 d1 = mask16(window(c0, c1, 16 - HDR), 0, HDR + len - 16);
        dw[i] = pick16(t == 0, d0, d1);
        psum[i] = sum16(dw[i], 0) - (t == 0 ? ((uint32_t)size[i] & 0xFF) + (((uint32_t)size[i] >> 8) & 0xFF) : 0u);
    }
#pragma unroll
    for (int i = 0; i < K; ++i) {
        psum[i] = (pair_sum(psum[i]) + tot[i]) & 0xFFFF;
        if (HEAD == 4) {  // shard bytes 2, 3: datagram chunk 0 byte 15, chunk 1 byte 0
            uint4 p0 = dw[i], p1 = dw[i];
            put_byte(p0, 15, psum[i]);
            put_byte(p1, 0, psum[i] >> 8);
            dw[i] = pick16(t == 0, p0, p1);
        }
    }
    uint4 pw[M];
    encode_col<K, M>(dw, pw, tab);
    uint32_t qsum[M];
#pragma unroll
    for (int j = 0; j < M; ++j) qsum[j] = (pair_sum(sum16(pw[j], 0)) + tot[K + j]) & 0xFFFF;
    if (!live) return;
    uint8_t* out = wire + g * (uint64_t)N * a.wire_pitch + 16 * t;
#pragma unroll
    for (int r = 0; r < N; ++r) {
        const int len = r < K ? size[r] + HEAD : gmax;
        const uint4 v = r < K ? dw[r] : pw[r - K];
        uint4 h = v;
        const uint32_t sent = sent0 + (uint32_t)r;
        const uint32_t srcno = src0 + (uint32_t)(r < K ? r : K - 1);
        const uint32_t ikn = ((uint32_t)N | ((uint32_t)K << 4) | ((uint32_t)r << 8)) & 0xFFFFu;
        put_byte(h, 0, HDR == 13 ? 0xED : 0xEC);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            put_byte(h, 1 + b, sent >> (8 * b));
            put_byte(h, 5 + b, srcno >> (8 * b));
        }
        put_byte(h, 9, ikn);
        put_byte(h, 10, ikn >> 8);
        if (HDR == 13) {
            // datagram checksum: byte sum of shard [0, len)
            const uint32_t d = r < K ? psum[r] + ((uint32_t)size[r] & 0xFF) + (((uint32_t)size[r] >> 8) & 0xFF) +
                                           (psum[r] & 0xFF) + (psum[r] >> 8)
                                     : qsum[r - K];
            put_byte(h, 11, d);
            put_byte(h, 12, d >> 8);
        }
        if (ok && (t == 0 || 16 < HDR + len)) stw(out + (uint64_t)r * a.wire_pitch, pick16(t == 0, h, v), a.store_nt & 2);
        if (t == 0) wire_len[g * N + r] = ok ? HDR + len : -1;
    }
}

template <int K, int M, int HDR>
__global__ void __launch_bounds__(256) k_pack_head(WireArgs a, const uint8_t* __restrict__ payload,
                                                   const int64_t* __restrict__ offsets,
                                                   const int32_t* __restrict__ sizes,
                                                   const uint32_t* __restrict__ tab,
                                                   const uint32_t* __restrict__ part,
                                                   const uint32_t* __restrict__ seq, uint8_t* __restrict__ wire,
                                                   int32_t* __restrict__ wire_len, uint64_t g0, uint32_t lanes,
                                                   uint32_t lpg) {
    const uint32_t flat = blockIdx.x * 256u + threadIdx.x;
    head_lane<K, M, HDR, false>(a, payload, offsets, sizes, tab, part, seq, wire, wire_len, g0 + (flat >> 1),
                                (int)(flat & 1), flat < lanes, lpg);
}

// One launch: body lanes in batches of 8 blocks dealt to one XCD (blocks b, b + 8, ...,
// b + 56 of each 64); a batch holds gpb whole groups (gpb * lpg <= 2048 lanes).  Each block
// publishes its partial sums write-through, waits for its stores, and bumps the batch
// counter; the block whose add is the batch's last runs the batch's heads (2 lanes per
// group) while the payload lines they re-read are still in that XCD's L2.
template <int K, int M, int HDR, bool UNI>
__global__ void __launch_bounds__(256) k_pack_one(WireArgs a, const uint8_t* __restrict__ payload,
                                                  const int64_t* __restrict__ offsets,
                                                  const int32_t* __restrict__ sizes,
                                                  const uint32_t* __restrict__ tab, uint32_t* __restrict__ part,
                                                  uint32_t* __restrict__ counters, uint32_t lpg, DivMagic rows_div,
                                                  uint32_t gpb, uint64_t nbatch) {
    __shared__ uint32_t s_last;
    const uint32_t b = blockIdx.x;
    const uint64_t beta = (uint64_t)(b >> 6) * 8 + (b & 7);
    const uint32_t lib = ((b >> 3) & 7) * 256u + threadIdx.x;  // lane in batch
    const uint32_t gib = UNI ? __builtin_amdgcn_readfirstlane((uint32_t)fast_div(lib >> 6, rows_div))
                             : (uint32_t)fast_div(lib >> 4, rows_div);
    const uint64_t g = beta * gpb + gib;
    const bool live = beta < nbatch && gib < gpb && g < a.groups;
    body_lane<K, M, HDR, true>(a, payload, offsets, sizes, tab, part, live ? g : 0, lib - gib * lpg, live, lpg);
    if (beta >= nbatch) return;  // whole block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(counters + beta, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 7;
    __syncthreads();
    if (!s_last || threadIdx.x >= 64) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint64_t gend = min((uint64_t)gpb, a.groups - beta * gpb);
    for (uint32_t h0 = 0; h0 < 2 * gend; h0 += 64) {
        const uint32_t h = h0 + threadIdx.x;
        head_lane<K, M, HDR, true>(a, payload, offsets, sizes, tab, part, a.seq, a.wire, a.wire_len,
                                   beta * gpb + (h >> 1), (int)(h & 1), h < 2 * gend, lpg);
    }
}

// ------------------------------------------------------------------ launchers
static inline unsigned waves_grid(uint64_t waves) { return (unsigned)((waves + 3) / 4); }

hipError_t launch_build_shards(const WireArgs& a, hipStream_t s) {
    const uint64_t rows = a.groups * (uint64_t)a.k;
    if (!rows) return hipSuccess;
    hipLaunchKernelGGL(k_build_shards, dim3(waves_grid(rows)), dim3(256), 0, s, a);
    return hipGetLastError();
}

template <int K, int M, int HDR>
hipError_t pack_fused_shape(const WireArgs& a, const uint32_t* tab, uint32_t* part, hipStream_t s) {
    // lanes per group for t >= 2 cover the longest datagram the shard pitch allows
    const uint32_t tn = (uint32_t)((HDR + a.pitch + 15) / 16);
    uint32_t lpg = std::max(16u, (tn - 2 + 15) / 16 * 16);
    const int uni_mode = tuning().wire_uni;
    if (uni_mode == 2) lpg = (lpg + 63) / 64 * 64;
    const bool uni = uni_mode != 0 && lpg % 64 == 0;
    const DivMagic rows_div = make_div_magic(uni ? lpg / 64 : lpg / 16);
    const uint32_t gpb = 2048 / lpg;
    if (tuning().wire_fused == 2 && gpb >= 1) {
        const uint64_t nbatch = (a.groups + gpb - 1) / gpb;
        const uint32_t P = (uint32_t)(a.k + a.m + 1) / 2;
        uint32_t* counters = part + a.groups * (lpg / 16) * P;
        hipError_t e = hipMemsetAsync(counters, 0, nbatch * 4, s);
        if (e != hipSuccess) return e;
        const uint64_t blocks = (nbatch + 7) / 8 * 64;
        if (blocks >= (1ull << 31)) return hipErrorInvalidValue;
        if (uni)
            hipLaunchKernelGGL((k_pack_one<K, M, HDR, true>), dim3((unsigned)blocks), dim3(256), 0, s, a, a.payload,
                               a.offsets, a.sizes, tab, part, counters, lpg, rows_div, gpb, nbatch);
        else
            hipLaunchKernelGGL((k_pack_one<K, M, HDR, false>), dim3((unsigned)blocks), dim3(256), 0, s, a, a.payload,
                               a.offsets, a.sizes, tab, part, counters, lpg, rows_div, gpb, nbatch);
        return hipGetLastError();
    }
    const uint64_t per = ((uint64_t)1 << 30) / lpg;  // groups per launch: lanes < 2^30
    for (uint64_t g0 = 0; g0 < a.groups; g0 += per) {
        const uint64_t gn = std::min(per, a.groups - g0);
        const uint32_t lanes = (uint32_t)(gn * lpg);
        if (uni)
            hipLaunchKernelGGL((k_pack_body<K, M, HDR, true>), dim3((lanes + 255) / 256), dim3(256), 0, s, a,
                               a.payload, a.offsets, a.sizes, tab, part, g0, lanes, lpg, rows_div);
        else
            hipLaunchKernelGGL((k_pack_body<K, M, HDR, false>), dim3((lanes + 255) / 256), dim3(256), 0, s, a,
                               a.payload, a.offsets, a.sizes, tab, part, g0, lanes, lpg, rows_div);
        const uint32_t hl = (uint32_t)(2 * gn);
        hipLaunchKernelGGL((k_pack_head<K, M, HDR>), dim3((hl + 255) / 256), dim3(256), 0, s, a, a.payload, a.offsets,
                           a.sizes, tab, (const uint32_t*)part, a.seq, a.wire, a.wire_len, g0, hl, lpg);
    }
    return hipGetLastError();
}

#define QFEC_PACK_CASE(KK, MM)                                                                              \
    if (a.k == KK && a.m == MM) {                                                                           \
        *launched = true;                                                                                   \
        return a.checksum ? pack_fused_shape<KK, MM, 13>(a, tab, part, s)                                   \
                          : pack_fused_shape<KK, MM, 11>(a, tab, part, s);                                  \
    }

// `part` needs pack_part_words(pitch, n) u32 per group; the caller's shard buffer holds it
hipError_t launch_pack_fused(const WireArgs& a, const uint32_t* tab, uint32_t* part, hipStream_t s, bool* launched) {
    *launched = false;
    if (!a.groups) return hipSuccess;
    QFEC_PACK_CASE(10, 3)
    QFEC_PACK_CASE(4, 1)
    QFEC_PACK_CASE(4, 2)
    QFEC_PACK_CASE(2, 2)
    QFEC_PACK_CASE(3, 1)
    QFEC_PACK_CASE(3, 2)
    QFEC_PACK_CASE(5, 1)
    QFEC_PACK_CASE(5, 3)
    QFEC_PACK_CASE(7, 1)
    QFEC_PACK_CASE(8, 4)
    return hipSuccess;
}
#undef QFEC_PACK_CASE

hipError_t launch_emit_wire(const WireArgs& a, hipStream_t s) {
    const uint64_t slots = a.groups * (uint64_t)(a.k + a.m);
    if (!slots) return hipSuccess;
    if (a.checksum) hipLaunchKernelGGL((k_emit_wire<13>), dim3(waves_grid(slots)), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_emit_wire<11>), dim3(waves_grid(slots)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_parse_wire(const WireArgs& a, hipStream_t s) {
    const uint64_t slots = a.groups * (uint64_t)(a.k + a.m);
    if (!slots) return hipSuccess;
    hipLaunchKernelGGL(k_parse_wire, dim3(waves_grid(slots)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_check_payloads(const WireArgs& a, hipStream_t s) {
    const uint64_t rows = a.groups * (uint64_t)a.k;
    if (!rows) return hipSuccess;
    hipLaunchKernelGGL(k_check_payloads, dim3(waves_grid(rows)), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace qfec
