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

#include "qfec_wire_device.hpp"

namespace qfec {


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
// For compile-time (K, M), build -> encode -> emit collapse into one body launch (plus a
// tiny head launch with checksums), so the [G][n][pitch] shard matrix never exists: HBM
// traffic is the payload in and the datagrams out.  GF arithmetic is bytewise, so check-shard
// bytes at any shard offset come from the data-shard bytes at the same offset; each lane
// works on one 16-B DATAGRAM chunk t = shard bytes [16t - HDR, 16t + 16 - HDR) of all n
// rows at once, with no neighbour exchange.
//
//  k_pack_body  flat over (group, t), lpg lanes per group (a multiple of 16).  HDR 11 (no
//               checksums): every chunk, header included.  HDR 13: every chunk but 0, with
//               shard byte 3 (the high checksum byte, datagram byte 16) left zero; 16-lane
//               partial byte sums (two rows per u32) go to `part`.
//  k_pack_head  HDR 13 only, one lane per group: shard bytes 0-3 are the sizes and payload
//               checksums, so check-shard bytes 0-3 are a K-term GF dot product of those
//               dwords -- no payload is read.  Writes chunk 0 (header, datagram checksum,
//               shard bytes 0-2) and byte 16 of every datagram.
template <int K, int M>
__device__ __forceinline__ void encode_cols(const uint4 (&x)[K], uint4 (&acc)[M], const uint32_t* __restrict__ tab) {
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

// the same over 8-byte columns (k_pack_wave64 with 8-B lanes)
template <int K, int M>
__device__ __forceinline__ void encode_cols8(const uint2 (&x)[K], uint2 (&acc)[M], const uint32_t* __restrict__ tab) {
#pragma unroll
    for (int r = 0; r < M; ++r) acc[r] = make_uint2(0, 0);
#pragma unroll
    for (int c = 0; c + 1 < K; c += 2) {
        const Sel a0 = gf_sel(x[c].x), a1 = gf_sel(x[c].y), b0 = gf_sel(x[c + 1].x), b1 = gf_sel(x[c + 1].y);
#pragma unroll
        for (int r = 0; r < M; ++r) {
            const uint32_t* ta = tab + (r * K + c) * QFEC_TAB_STRIDE;
            const uint32_t* tb = tab + (r * K + c + 1) * QFEC_TAB_STRIDE;
            acc[r].x = mac2(acc[r].x, a0, b0, ta, tb);
            acc[r].y = mac2(acc[r].y, a1, b1, ta, tb);
        }
    }
    if (K & 1) {
        const Sel a0 = gf_sel(x[K - 1].x), a1 = gf_sel(x[K - 1].y);
#pragma unroll
        for (int r = 0; r < M; ++r) {
            const uint32_t* t = tab + (r * K + K - 1) * QFEC_TAB_STRIDE;
            acc[r].x ^= gf_mul4(a0, t[0], t[1], t[2], t[3], t[4]);
            acc[r].y ^= gf_mul4(a1, t[0], t[1], t[2], t[3], t[4]);
        }
    }
}

__device__ __forceinline__ uint2 ldu8(const uint8_t* p) {
    uint2 v;
    __builtin_memcpy(&v, p, 8);
    return v;
}
__device__ __forceinline__ uint2 mask8(uint2 v, int lo, int hi) {
    v.x &= byte_mask(lo, hi, 0);
    v.y &= byte_mask(lo, hi, 1);
    return v;
}
__device__ __forceinline__ uint32_t sum8(const uint2& v, uint32_t acc) {
    return __builtin_amdgcn_sad_u8(v.y, 0u, __builtin_amdgcn_sad_u8(v.x, 0u, acc));
}

// sum over each aligned 16-lane row, result in every lane of the row (DPP, no LDS)
__device__ __forceinline__ uint32_t row16_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    return v;
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

// datagram header bytes 0-10 (+ 11-12 with HDR 13) into chunk 0 of row r
template <int HDR>
__device__ __forceinline__ void put_header(uint4& v, uint32_t sent, uint32_t srcno, uint32_t ikn, uint32_t dsum) {
    put_byte(v, 0, HDR == 13 ? 0xED : 0xEC);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        put_byte(v, 1 + b, sent >> (8 * b));
        put_byte(v, 5 + b, srcno >> (8 * b));
    }
    put_byte(v, 9, ikn);
    put_byte(v, 10, ikn >> 8);
    if (HDR == 13) {
        put_byte(v, 11, dsum);
        put_byte(v, 12, dsum >> 8);
    }
}

template <int K, int M, int HDR, bool LINE>
__global__ void __launch_bounds__(256) k_pack_body(WireArgs a, const uint8_t* __restrict__ payload,
                                                   const int64_t* __restrict__ offsets,
                                                   const int32_t* __restrict__ sizes,
                                                   const uint32_t* __restrict__ seq,
                                                   const uint32_t* __restrict__ tab, uint32_t* __restrict__ part,
                                                   uint64_t g0, uint32_t lanes, uint32_t lpg, DivMagic lpg_div,
                                                   uint64_t row0) {
    constexpr int N = K + M, HEAD = HDR == 13 ? 4 : 2, P = (N + 1) / 2;
    // first chunk of the body: 1 (HDR 13: k_pack_head writes chunk 0 and byte 16), 4 (HDR 13,
    // LINE: k_pack_line0 writes the whole first 64-B line), 0 (HDR 11: the body writes all)
    constexpr int TS = HDR == 13 ? (LINE ? 4 : 1) : 0;
    constexpr int PS = 16 * TS - HDR - HEAD;  // its payload offset (< 0 unless LINE with HDR 13)
    const uint32_t flat = blockIdx.x * 256u + threadIdx.x;
    const bool live = flat < lanes;  // dead lanes still join the row sums (with zeros)
    const uint32_t gl = (uint32_t)fast_div(flat, lpg_div);
    const uint32_t rem = flat - gl * lpg;
    const uint64_t g = g0 + gl;
    const int t = TS + (int)rem;
    const bool first = PS < 0 && t == TS;  // holds shard byte 0 (HDR 11) / byte 3 (HDR 13)
    const int p = 16 * t - HDR - HEAD;   // payload offset of this chunk's first byte
    int size[K], gmax = 0;
    bool ok = false;
    if (live) ok = group_sizes<K, HEAD>(sizes, g, (int)a.pitch, size, gmax);
    // LINE: every chunk up to the (64-B multiple) wire pitch is stored, zeros past a datagram,
    // so each 64-B line of a row is written whole by one store instruction
    const bool act = ok && (LINE || 16 * t < HDR + gmax);
    uint8_t* out = a.wire + g * (uint64_t)N * a.wire_pitch + 16 * t;
    // all K loads back to back, addresses clamped into the packet (+16 readable bytes)
    uint4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = make_uint4(0, 0, 0, 0);
    if (ok) {
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = ldu16(payload + offsets[g * K + i] + min(max(p, 0), size[i]));
#pragma unroll
        for (int i = 0; i < K; ++i) {
            // the first chunk's payload starts -PS bytes in: shift it up
            const uint4 sh = window(make_uint4(0, 0, 0, 0), x[i], 16 + PS);
            x[i] = mask16(pick16(first, sh, x[i]), first ? -PS : 0, size[i] - p);
            if (HDR == 11) {  // shard bytes 0-1 (size) at chunk bytes 11-12 of the first chunk
                uint4 y = x[i];
                put_byte(y, 11, (uint32_t)size[i]);
                put_byte(y, 12, (uint32_t)size[i] >> 8);
                x[i] = pick16(first, y, x[i]);
            }
        }
    }
    uint32_t ps[P];
#pragma unroll
    for (int q = 0; q < P; ++q) ps[q] = 0;
    if (HDR == 13) {
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const uint32_t s = sum16(x[i], 0);  // payload bytes only
            ps[i >> 1] += (i & 1) ? s << 16 : s;
        }
    }
    uint4 acc[M];
    encode_cols<K, M>(x, acc, tab);
#pragma unroll
    for (int r = 0; r < M; ++r) pin16(acc[r]);  // no sinking of a row's MAC into its store branch
    uint32_t sent0 = 0, src0 = 0;
    if (HDR == 11 && act && first) {
        sent0 = seq[2 * g];
        src0 = seq[2 * g + 1];
    }
#pragma unroll
    for (int r = 0; r < N; ++r) {
        uint4 v = r < K ? x[r] : acc[r - K];
        const int len = r < K ? size[r] + HEAD : gmax;
        if (HDR == 11 && first) {
            uint4 h = v;
            put_header<11>(h, sent0 + (uint32_t)r, src0 + (uint32_t)(r < K ? r : K - 1),
                           ((uint32_t)N | ((uint32_t)K << 4) | ((uint32_t)r << 8)) & 0xFFFFu, 0);
            v = pick16(true, h, v);
        }
        if (act && (LINE || 16 * t < HDR + len)) stw(out + (uint64_t)r * a.wire_pitch, v, a.store_nt & 1);
        if (HDR == 11 && act && first) a.wire_len[g * N + r] = HDR + len;
        if (HDR == 13 && r >= K) {
            const uint32_t s = sum16(v, 0);  // check-shard bytes 0-3 are the head's: zero here
            ps[r >> 1] += (r & 1) ? s << 16 : s;
        }
    }
    if (HDR == 11) {
        if (live && !ok && first)
            for (int r = 0; r < N; ++r) a.wire_len[g * N + r] = -1;
        return;
    }
    // Per-lane sums are <= 16 * 255, a 16-lane row's <= 65280: two rows share a u32 exactly.
    // lpg >= 16 lanes per group, so a 16-lane row holds at most two groups (its first and
    // its last): one sum for each, slot 0 and slot 1 of the row's record.
    const uint32_t gf = (uint32_t)fast_div(flat & ~15u, lpg_div), gla = (uint32_t)fast_div(flat | 15u, lpg_div);
    uint32_t* rec = part + (row0 + (flat >> 4)) * 2 * P;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        const uint32_t v0 = row16_sum(gl == gf ? ps[q] : 0u);
        const uint32_t v1 = row16_sum(gl == gla && gla != gf ? ps[q] : 0u);
        if (live && (flat & 15) == 0) {
            rec[q] = v0;
            rec[P + q] = v1;
        }
    }
}

// HDR 13 only.  One lane per group, no payload reads (see the section comment).
template <int K, int M>
__global__ void __launch_bounds__(256) k_pack_head(WireArgs a, const int32_t* __restrict__ sizes,
                                                   const uint32_t* __restrict__ tab,
                                                   const uint32_t* __restrict__ part,
                                                   const uint32_t* __restrict__ seq, uint8_t* __restrict__ wire,
                                                   int32_t* __restrict__ wire_len, uint64_t g0, uint32_t lanes,
                                                   uint32_t lpg, uint64_t row0) {
    constexpr int N = K + M, HDR = 13, HEAD = 4, P = (N + 1) / 2;
    const uint32_t flat = blockIdx.x * 256u + threadIdx.x;
    if (flat >= lanes) return;
    const uint64_t g = g0 + flat;
    int size[K], gmax = 0;
    const bool ok = group_sizes<K, HEAD>(sizes, g, (int)a.pitch, size, gmax);
    if (!ok) {
#pragma unroll
        for (int r = 0; r < N; ++r) wire_len[g * N + r] = -1;
        return;
    }
    uint32_t tot[N];
#pragma unroll
    for (int r = 0; r < N; ++r) tot[r] = 0;
    // the body's 16-lane rows holding this group's lanes [flat0, flat0 + lpg)
    const uint64_t flat0 = (uint64_t)flat * lpg;
    for (uint64_t row = flat0 >> 4; row <= (flat0 + lpg - 1) >> 4; ++row) {
        const uint32_t* rec = part + (row0 + row) * 2 * P + ((row << 4) >= flat0 ? 0 : P);
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const uint32_t v = rec[q];
            tot[2 * q] += v & 0xFFFF;
            if (2 * q + 1 < N) tot[2 * q + 1] += v >> 16;
        }
    }
    const uint32_t sent0 = seq[2 * g], src0 = seq[2 * g + 1];
    // shard bytes 0-3 of the data rows: [size lo][size hi][cksum lo][cksum hi]
    uint32_t d[K];
#pragma unroll
    for (int i = 0; i < K; ++i) d[i] = ((uint32_t)size[i] & 0xFFFFu) | ((tot[i] & 0xFFFFu) << 16);
    uint8_t* out = wire + g * (uint64_t)N * a.wire_pitch;
#pragma unroll
    for (int r = 0; r < N; ++r) {
        uint32_t w;  // shard bytes 0-3 of row r
        uint32_t dsum;
        if (r < K) {
            w = d[r];
            dsum = tot[r] + (w & 0xFF) + ((w >> 8) & 0xFF) + ((w >> 16) & 0xFF) + (w >> 24);
        } else {
            w = 0;
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const uint32_t* e = tab + ((r - K) * K + i) * QFEC_TAB_STRIDE;
                w ^= gf_mul4(gf_sel(d[i]), e[0], e[1], e[2], e[3], e[4]);
            }
            dsum = tot[r] + (w & 0xFF) + ((w >> 8) & 0xFF) + ((w >> 16) & 0xFF) + (w >> 24);
        }
        const int len = r < K ? size[r] + HEAD : gmax;
        // chunk 0 = header (13) + shard bytes 0-2, masked to the datagram length
        uint4 v = make_uint4(0, 0, 0, w << 8);
        put_header<HDR>(v, sent0 + (uint32_t)r, src0 + (uint32_t)(r < K ? r : K - 1),
                        ((uint32_t)N | ((uint32_t)K << 4) | ((uint32_t)r << 8)) & 0xFFFFu, dsum);
        v = mask16(v, 0, HDR + len);
        stw(out + (uint64_t)r * a.wire_pitch, v, a.store_nt & 2);
        if (HDR + len > 16) out[(uint64_t)r * a.wire_pitch + 16] = (uint8_t)(w >> 24);
        wire_len[g * N + r] = HDR + len;
    }
}

// HDR 13 with LINE bodies: the first 64-B line (datagram chunks 0-3) of every row, one quad of
// lanes per group, lane q = chunk q, so each row's line 0 is one store instruction.  Chunk 0
// is the header + shard bytes 0-2, chunk 1 starts with shard byte 3, chunks 1-3 carry payload
// bytes 0-46 (and their check-shard bytes); the row sums are the body's partial records plus
// the quad's own chunks, reduced across the quad.
__device__ __forceinline__ uint32_t quad_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    return v;
}

template <int K, int M>
__global__ void __launch_bounds__(256) k_pack_line0(WireArgs a, const uint8_t* __restrict__ payload,
                                                    const int64_t* __restrict__ offsets,
                                                    const int32_t* __restrict__ sizes,
                                                    const uint32_t* __restrict__ tab,
                                                    const uint32_t* __restrict__ part,
                                                    const uint32_t* __restrict__ seq, uint8_t* __restrict__ wire,
                                                    int32_t* __restrict__ wire_len, uint64_t g0, uint32_t groups,
                                                    uint32_t lpg, uint64_t row0) {
    constexpr int N = K + M, HDR = 13, HEAD = 4, P = (N + 1) / 2;
    const uint32_t flat = blockIdx.x * 256u + threadIdx.x;
    const uint32_t gl = flat >> 2;
    const int q = (int)(flat & 3u);
    const bool live = gl < groups;  // a quad is live or dead as a whole; dead quads still
                                    // run the DPP reductions (no early return inside a quad)
    const uint64_t g = g0 + (live ? gl : 0u);
    // every load that does not depend on another is issued first: sizes, offsets, seq and the
    // body's partial-sum records of this group (one 16-lane record row per quad lane and pass)
    int size[K], gmax = 0;
    int64_t off[K];
    bool ok = false;
    uint32_t tot[N];
#pragma unroll
    for (int r = 0; r < N; ++r) tot[r] = 0;
    uint32_t sent0 = 0, src0 = 0;
    if (live) {
        ok = group_sizes<K, HEAD>(sizes, g, (int)a.pitch, size, gmax);
#pragma unroll
        for (int i = 0; i < K; ++i) off[i] = offsets[g * K + i];
        sent0 = seq[2 * g];
        src0 = seq[2 * g + 1];
        const uint64_t flat0 = (uint64_t)gl * lpg;
        for (uint64_t row = (flat0 >> 4) + (uint64_t)q; row <= (flat0 + lpg - 1) >> 4; row += 4) {
            const uint32_t* rec = part + (row0 + row) * 2 * P + ((row << 4) >= flat0 ? 0 : P);
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const uint32_t v = rec[j];
                tot[2 * j] += v & 0xFFFF;
                if (2 * j + 1 < N) tot[2 * j + 1] += v >> 16;
            }
        }
    }
    // chunk q: datagram bytes [16q, 16q + 16), payload offset p = 16q - 17
    const int p = 16 * q - HDR - HEAD;
    uint4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = make_uint4(0, 0, 0, 0);
    if (ok && q > 0) {
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = ldu16(payload + off[i] + min(max(p, 0), size[i]));
#pragma unroll
        for (int i = 0; i < K; ++i) {  // chunk 1: payload byte 0 sits at chunk byte 1
            const uint4 sh = window(make_uint4(0, 0, 0, 0), x[i], 15);
            x[i] = mask16(pick16(q == 1, sh, x[i]), q == 1 ? 1 : 0, size[i] - p);
        }
    }
    uint4 acc[M];
    encode_cols<K, M>(x, acc, tab);
    // row sums: own chunk (payload / check bytes; shard bytes 0-3 are still zero here) plus the
    // body's 16-lane records of this group, spread over the quad's lanes
#pragma unroll
    for (int r = 0; r < N; ++r) tot[r] += sum16(r < K ? x[r] : acc[r - K], 0);
#pragma unroll
    for (int r = 0; r < N; ++r) tot[r] = quad_sum(tot[r]);
    if (!live) return;
    if (!ok) {
        if (q == 0)
            for (int r = 0; r < N; ++r) wire_len[g * N + r] = -1;
        return;
    }
    uint32_t d[K];  // shard bytes 0-3 of the data rows: [size lo][size hi][cksum lo][cksum hi]
#pragma unroll
    for (int i = 0; i < K; ++i) d[i] = ((uint32_t)size[i] & 0xFFFFu) | ((tot[i] & 0xFFFFu) << 16);
    uint8_t* out = wire + g * (uint64_t)N * a.wire_pitch + 16 * q;
#pragma unroll
    for (int r = 0; r < N; ++r) {
        uint32_t w = d[r < K ? r : 0];  // shard bytes 0-3 of row r
        if (r >= K) {
            w = 0;
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const uint32_t* e = tab + ((r - K) * K + i) * QFEC_TAB_STRIDE;
                w ^= gf_mul4(gf_sel(d[i]), e[0], e[1], e[2], e[3], e[4]);
            }
        }
        const uint32_t dsum = tot[r] + (w & 0xFF) + ((w >> 8) & 0xFF) + ((w >> 16) & 0xFF) + (w >> 24);
        uint4 v = r < K ? x[r] : acc[r - K];
        if (q == 0) {
            v = make_uint4(0, 0, 0, w << 8);
            put_header<HDR>(v, sent0 + (uint32_t)r, src0 + (uint32_t)(r < K ? r : K - 1),
                            ((uint32_t)N | ((uint32_t)K << 4) | ((uint32_t)r << 8)) & 0xFFFFu, dsum);
        } else if (q == 1) {
            put_byte(v, 0, w >> 24);
        }
        stw(out + (uint64_t)r * a.wire_pitch, v, a.store_nt & 2);
        if ((r & 3) == q) wire_len[g * N + r] = HDR + (r < K ? size[r] + HEAD : gmax);
    }
}

// ------------------------------------------------------------------ receive: fused
// For compile-time (K, M), parse -> reconstruct -> check collapse into one launch, one wave
// per group: HBM traffic is the received datagrams in and the k data rows out (check-shard
// rows of d_shards are not written on this path).
//  1. lanes j < n parse datagram j's header (unpack_fec_head's tests, FecCodecBuf.cpp:334-411)
//  2. survivors = the first k rows in group order whose header is good -- optimistic: their
//     shard checksums are verified in step 4 and a bad one restarts the group without it,
//     so the final survivors are the first k VALID rows (NetFecCodec.cpp:504-528).
//  3. passes over the shard columns (16 B per lane, then one 4-B-per-lane tail pass when
//     fewer than 17 chunks remain): survivor chunks are loaded straight from the datagrams
//     (unaligned), lost data rows decoded with the record's perm tables, the k data rows
//     stored, and shard / payload byte sums accumulated.
//  4. wave sums -> datagram checksum verdicts, then dec_src_pkt_info's status per data row.
__device__ __forceinline__ uint32_t wave_total(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// ------------------------------------------------------------------ send: one wave per group
// HDR 13 with a 1088-B wire pitch (1 KiB payloads): the body's chunks 4..67 are exactly 64
// lanes, so with groups wave-aligned each wave holds one whole group and can finish its first
// 64-B line itself: wave sums of the body's chunks, then lanes 0..15
// take dword i of line 0 of every row -- header, shard bytes 0-3, payload bytes 0..46 and
// their check bytes (a dword-wide encode) -- and store each row's line 0 as one instruction.
// This replaces k_pack_line0's scattered second pass (13 lines 1088 B apart per group).
// sum over the lanes of each group of 64 / GPW lanes, in every lane of the group
template <int GPW>
__device__ __forceinline__ uint32_t group_total(uint32_t v) {
    if constexpr (GPW == 1) {
        return wave_total(v);
    } else {  // GPW 2: 16-lane rows, then the row pair of each 32-lane half
        v = row16_sum(v);
        return v + (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);  // lane ^ 16
    }
}

// FP (frame prefix 4 or 12, qfec_pack_frames): the same pass emits ProtocolUdp frames
// instead of bare datagrams -- frame = [mask][c][cmd][proto]([conv][hid])[datagram], bytes 1..
// XORed with mask ^ gmask ^ 0x5a (network/ProtocolBasic.cpp:111-150, SessionDesc.cpp:69-77).
// Lane ln then owns frame chunk 4 + ln, i.e. datagram bytes shifted down by FP (the payload
// loads are unaligned anyway); line 0's dword ln is datagram dword ln - FP/4, the prefix below
// it.  The frame checksum is the datagram's byte sum (header + the shard sum the wave already
// has) plus the prefix bytes, so no byte is read twice.  Bytes of a row past its frame are 0.
#ifndef FRAME_WAVES
#define FRAME_WAVES 3  // waves per SIMD the one-pass frame send is compiled for (A/B: 4 spills)
#endif
//
// NP (GPW 1 only): passes over the body's chunks.  NP 1 covers wire pitches up to 1088 (body
// chunks 4 .. wire_pitch / 16 - 1, lanes past them idle); NP 2 covers 1104 .. 2112, e.g. the
// 1472-B pitch of 1400-B (MTU-size) payloads: pass 0 chunks 4..67, pass 1 chunks 68.. on the
// first wire_pitch / 16 - 68 lanes.  Row sums accumulate over the passes, so line 0 is
// unchanged.
//
// LW 8 (wire pitches 1104 .. 1600): 8-byte lanes, NP passes over the 8-B chunks 8 .. wire_pitch
// / 8 - 1 (1088: two full passes; 1472: 64 + 64 + 48 lanes), fewer registers per pass.
template <int K, int M, int GPW, int FP = 0, int NP = 1, int LW = 16, int WV = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WV ? WV : LW == 8 ? (NP >= 3 ? 4 : 6) : FP ? FRAME_WAVES : 4))) k_pack_wave64(WireArgs a, const uint8_t* __restrict__ payload,
                                                     const int64_t* __restrict__ offsets,
                                                     const int32_t* __restrict__ sizes,
                                                     const uint32_t* __restrict__ seq,
                                                     const uint32_t* __restrict__ tab, uint64_t groups,
                                                     FrameSend fs) {
    constexpr int N = K + M, HDR = 13, HEAD = 4, LPG = 64 / GPW;  // lanes per group
    constexpr int FD = FP / 4;                                      // prefix dwords of line 0
    static_assert(FP == 0 || FP == 4 || FP == 12, "frame prefix");
    static_assert(NP == 1 || GPW == 1, "passes");
    static_assert(LW == 16 || (LW == 8 && GPW == 1), "lane width");
    const int lane = threadIdx.x & 63;
    const int ln = GPW == 1 ? lane : lane % LPG;  // lane within its group: chunk 4 + ln (+ 64 per pass)
    const uint64_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));  // wave-uniform
    if (w * GPW >= groups) return;  // whole waves
    // GPW 1: g is wave-uniform (scalar loads of sizes / offsets); GPW 2: two groups per wave,
    // a dead second group still joins the cross-lane sums
    const uint64_t g = GPW == 1 ? w : w * GPW + (uint64_t)(lane / LPG);
    const bool live = GPW == 1 || g < groups;
    const int tend = GPW == 1 ? (int)(a.wire_pitch / 16) : 4 + LPG;  // body chunks end here
    int size[K], gmax = 0;
    bool ok = false;
    if (live) ok = group_sizes<K, HEAD>(sizes, g, (int)a.pitch, size, gmax);
    if (GPW == 1 && !ok) {
        if (lane < N) a.wire_len[g * N + lane] = -1;
        return;
    }
    int64_t off[K];
#pragma unroll
    for (int i = 0; i < K; ++i) off[i] = ok ? offsets[g * K + i] : 0;
    uint8_t* out_g = a.wire + g * (uint64_t)N * a.wire_pitch;
    // FP: the group's N mask bytes, from the aligned dwords that hold them (scalar loads for
    // GPW 1; an aligned dword never reaches past the page its first byte is on); row r's XOR
    // word is formed where it is used, so no N registers stay live across the encode
    uint32_t mw5[FP ? 5 : 1];
    int msh = 0;
    if constexpr (FP != 0) {
        const uint64_t b0 = g * (uint64_t)N;
        const uint32_t* mw = reinterpret_cast<const uint32_t*>(fs.mask + (b0 & ~(uint64_t)3));
        msh = (int)(b0 & 3);
#pragma unroll
        for (int d = 0; d < 5; ++d) mw5[d] = 4 * d < msh + N ? mw[d] : 0u;
    }
    auto mm_of = [&](int r) -> uint32_t {  // (mask ^ gmask ^ 0x5a) in every byte
        if constexpr (FP == 0) {
            return 0u;
        } else {
            const int bpos = msh + r;
            const uint32_t byte = (mw5[bpos >> 2] >> (8 * (bpos & 3))) ^ fs.gmask ^ 0x5Au;
            return (byte & 0xFFu) * 0x01010101u;
        }
    };
    uint32_t ps[N];  // per-lane byte sums of each row's chunks (payload / check bytes)
#pragma unroll
    for (int r = 0; r < N; ++r) ps[r] = 0;
    if constexpr (LW == 8) {
        const int tend8 = (int)(a.wire_pitch / 8);
#pragma unroll
        for (int pp = 0; pp < NP; ++pp) {
            const int t = 8 + ln + 64 * pp;
            const bool act = ok && t < tend8;
            const int p = 8 * t - FP - HDR - HEAD;  // payload offset of this chunk's first byte (>= 35)
            uint2 x[K];
#pragma unroll
            for (int i = 0; i < K; ++i) x[i] = make_uint2(0, 0);
            if (act) {
#pragma unroll
                for (int i = 0; i < K; ++i) x[i] = ldu8(payload + off[i] + min(p, size[i]));
#pragma unroll
                for (int i = 0; i < K; ++i) x[i] = mask8(x[i], 0, size[i] - p);
            }
#pragma unroll
            for (int i = 0; i < K; ++i) ps[i] = sum8(x[i], ps[i]);
            uint2 acc[M];
            encode_cols8<K, M>(x, acc, tab);
#pragma unroll
            for (int r = 0; r < M; ++r) asm volatile("" : "+v"(acc[r].x), "+v"(acc[r].y));
            uint8_t* out = out_g + 8 * t;
#pragma unroll
            for (int r = 0; r < N; ++r) {
                uint2 v = r < K ? x[r] : acc[r - K];
                if (r >= K) ps[r] = sum8(v, ps[r]);
                if constexpr (FP != 0) {  // XOR the frame's bytes only: padding past it stays 0
                    const int total = FP + HDR + (r < K ? size[r] + HEAD : gmax);
                    uint64_t klo, khi;
                    int rel = total - 8 * t;
                    asm volatile("" : "+v"(rel));
                    keep_words(rel, klo, khi);
                    const uint32_t mr = mm_of(r);
                    const uint64_t xl = (((uint64_t)mr << 32) | mr) & klo;
                    v = make_uint2(v.x ^ (uint32_t)xl, v.y ^ (uint32_t)(xl >> 32));
                }
                if (act) {
                    uint2* dst = reinterpret_cast<uint2*>(out + (uint64_t)r * a.wire_pitch);
                    if (a.store_nt & 1) {
                        const u32x2 w2 = {v.x, v.y};
                        __builtin_nontemporal_store(w2, reinterpret_cast<u32x2*>(dst));
                    } else {
                        *dst = v;
                    }
                }
            }
        }
    } else {
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
        const int t = 4 + ln + 64 * pp;
        const bool act = ok && t < tend;         // idle lanes carry zeros: they add nothing to the sums
        const int p = 16 * t - FP - HDR - HEAD;  // payload offset of this chunk's first byte (>= 35)
        uint4 x[K];
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = make_uint4(0, 0, 0, 0);
        if (act) {
#pragma unroll
            for (int i = 0; i < K; ++i) x[i] = ldu16(payload + off[i] + min(p, size[i]));
#pragma unroll
            for (int i = 0; i < K; ++i) x[i] = mask16(x[i], 0, size[i] - p);
        }
#pragma unroll
        for (int i = 0; i < K; ++i) ps[i] = sum16(x[i], ps[i]);
        uint4 acc[M];
        encode_cols<K, M>(x, acc, tab);
#pragma unroll
        for (int r = 0; r < M; ++r) pin16(acc[r]);
        uint8_t* out = out_g + 16 * t;
#pragma unroll
        for (int r = 0; r < N; ++r) {
            uint4 v = r < K ? x[r] : acc[r - K];
            if (r >= K) ps[r] = sum16(v, ps[r]);
            if constexpr (FP != 0) {  // XOR the frame's bytes only: padding past it stays 0
                const int total = FP + HDR + (r < K ? size[r] + HEAD : gmax);
                uint64_t klo, khi;  // bytes of this chunk below the frame's end
                int rel = total - 16 * t;
                asm volatile("" : "+v"(rel));  // formed here, after the encode: not hoisted into it
                keep_words(rel, klo, khi);
                const uint32_t mr = mm_of(r);
                const uint64_t m2 = ((uint64_t)mr << 32) | mr;
                const uint64_t xl = m2 & klo, xh = m2 & khi;
                v = make_uint4(v.x ^ (uint32_t)xl, v.y ^ (uint32_t)(xl >> 32), v.z ^ (uint32_t)xh, v.w ^ (uint32_t)(xh >> 32));
            }
            if (act) stw(out + (uint64_t)r * a.wire_pitch, v, a.store_nt & 1);
        }
    }
    }
    // ---- line 0
    // line 0's payload dwords (lanes ln 0..15: frame bytes 4 ln .. 4 ln + 3 = datagram dword
    // dl = ln - FD; payload byte 4 dl - 17 at its first byte)
    const int dl = ln - FD;
    const int q = 4 * dl - HDR - HEAD;
    uint32_t pay[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        pay[i] = 0;
        if (ok && dl >= 4 && ln < 16) __builtin_memcpy(&pay[i], payload + off[i] + min(max(q, 0), size[i]), 4);
    }
#pragma unroll
    for (int i = 0; i < K; ++i) {
        // byte j of the dword holds payload byte q + j (dword 4: loaded from payload byte 0 and
        // shifted up one byte); keep the bytes below the payload's size
        const uint32_t v = dl == 4 ? pay[i] << 8 : pay[i];
        const int nb = min(max(size[i] - q, 0), 4);
        pay[i] = nb >= 4 ? v : v & ((1u << (8 * nb)) - 1u);
    }
    uint32_t tot[N];  // payload sums of the data rows, check-byte sums of the check rows
#pragma unroll
    for (int i = 0; i < K; ++i) tot[i] = group_total<GPW>(ps[i] + __builtin_amdgcn_sad_u8(pay[i], 0u, 0u));
    // shard view of line 0's dwords: data row i = [size][cksum] at shard bytes 0-3, then payload
    uint32_t sh[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const uint32_t wd = ((uint32_t)size[i] & 0xFFFFu) | ((tot[i] & 0xFFFFu) << 16);  // shard bytes 0-3
        sh[i] = !ok || dl < 3 ? 0u : dl == 3 ? wd << 8 : dl == 4 ? (wd >> 24) | pay[i] : pay[i];
    }
    uint32_t par[M];  // check rows' shard view: a dword-wide encode of the data rows'
#pragma unroll
    for (int j = 0; j < M; ++j) par[j] = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const Sel sl = gf_sel(sh[i]);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const uint32_t* e = tab + (j * K + i) * QFEC_TAB_STRIDE;
            par[j] ^= gf_mul4(sl, e[0], e[1], e[2], e[3], e[4]);
        }
    }
#pragma unroll
    for (int j = 0; j < M; ++j)
        tot[K + j] = group_total<GPW>(ps[K + j] + (ln < 16 ? __builtin_amdgcn_sad_u8(par[j], 0u, 0u) : 0u));
    if (!ok) {  // (GPW 2) a void or dead group: no datagram bytes, lengths -1
        if (live && ln < N) a.wire_len[g * N + ln] = -1;
        return;
    }
    const uint32_t sent0 = seq[2 * g], src0 = seq[2 * g + 1];
    uint32_t fcmd = 0, fproto = 0;
    if constexpr (FP != 0) {
        fcmd = (fs.cmd & 0x1Fu) | 0xA0u;
        fproto = fs.protocol & 0xFFu;
    }
#pragma unroll
    for (int r = 0; r < N; ++r) {
        uint32_t dsum;
        const uint32_t v = r < K ? sh[r] : par[r - K];
        if (r < K) {
            const uint32_t wd = ((uint32_t)size[r] & 0xFFFFu) | ((tot[r] & 0xFFFFu) << 16);
            dsum = tot[r] + (wd & 0xFF) + ((wd >> 8) & 0xFF) + ((wd >> 16) & 0xFF) + (wd >> 24);
        } else {
            dsum = tot[r];  // check shard bytes 0-3 are in par's dwords 3-4, summed above
        }
        const uint32_t sent = sent0 + (uint32_t)r, src = src0 + (uint32_t)(r < K ? r : K - 1);
        const uint32_t ikn = ((uint32_t)N | ((uint32_t)K << 4) | ((uint32_t)r << 8)) & 0xFFFFu;
        uint32_t d = v;
        if (dl == 0) d = 0xEDu | (sent << 8);
        else if (dl == 1) d = (sent >> 24) | (src << 8);
        else if (dl == 2) d = (src >> 24) | (ikn << 8) | ((dsum & 0xFFu) << 24);
        else if (dl == 3) d = ((dsum >> 8) & 0xFFu) | v;
        if constexpr (FP != 0) {
            const int total = FP + HDR + (r < K ? size[r] + HEAD : gmax);
            uint32_t conv = 0, hid = 0;
            if (FP == 12) {
                conv = fs.conv_hid[2 * (g * N + r)];
                hid = fs.conv_hid[2 * (g * N + r) + 1];
            }
            // CheckSum over frame bytes 2.. (ProtocolBasic.cpp:80-87): cmd, protocol, the Session
            // prefix and every datagram byte -- the header's bytes plus the shard sum dsum
            const uint32_t hsum = 0xEDu + __builtin_amdgcn_sad_u8(sent, 0u, 0u) + __builtin_amdgcn_sad_u8(src, 0u, 0u) +
                                  (ikn & 0xFFu) + (ikn >> 8) + (dsum & 0xFFu) + ((dsum >> 8) & 0xFFu);
            const uint32_t fsum = fcmd + fproto + __builtin_amdgcn_sad_u8(conv, 0u, 0u) +
                                  __builtin_amdgcn_sad_u8(hid, 0u, 0u) + hsum + dsum;
            const uint32_t c = ~((fsum >> 16) + (fsum & 0xFFFFu)) & 0xFFu;
            if (ln == 0) d = (c | (fcmd << 8) | (fproto << 16)) << 8;
            else if (FP == 12 && ln == 1) d = conv;
            else if (FP == 12 && ln == 2) d = hid;
            d ^= mm_of(r) & byte_mask(ln == 0 ? 1 : 0, total - 4 * ln, 0);
            if (ln == 0) d |= (mw5[(msh + r) >> 2] >> (8 * ((msh + r) & 3))) & 0xFFu;  // the raw mask byte
        }
        if (ln < 16) {
            uint32_t* dst = reinterpret_cast<uint32_t*>(out_g + (uint64_t)r * a.wire_pitch + 4 * ln);
            if (a.store_nt & 2) __builtin_nontemporal_store(d, dst);
            else *dst = d;
        }
    }
    if (ln < N) a.wire_len[g * N + ln] = FP + HDR + (ln < K ? size[ln] + HEAD : gmax);
}

// The fused receive (qfec_unpack_datagrams / qfec_unpack_frames) is k_rx in qfec_rx.hip.


// ------------------------------------------------------------------ launchers

hipError_t launch_build_shards(const WireArgs& a, hipStream_t s) {
    const uint64_t rows = a.groups * (uint64_t)a.k;
    if (!rows) return hipSuccess;
    hipLaunchKernelGGL(k_build_shards, dim3(waves_grid(rows)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// the one-wave send's mapping for a wire (or frame) pitch that is the 64-B multiple above the row:
// 1 one group per wave, one pass (1088 B); 2 two groups per wave (576 B); 10 one group per wave on
// 8-B lanes (1104..1600 B); 0 none.  (16-B lanes in two passes above 1088 B, a retired A/B, ran
// 841 us against 782 for the body + line-0 pair at 1472 B: profiles/r03_wire/r03n_mtu_ab.txt)
static int send_wave_gpw(uint64_t wire_pitch) {
    // above 1088 B: 8-B lanes in three passes (1472 B, RS(10,13) x 100k: 737 against 781 us for
    // the body + line-0 pair); at 1088 B 16-B lanes, one pass (497 against 545 us on 8-B lanes)
    if (wire_pitch > 1088 && wire_pitch <= 1600) return 10;
    if (wire_pitch == 576) return 2;
    if (wire_pitch == 1088) return 1;
    return 0;
}

template <int K, int M, int HDR>
hipError_t pack_fused_shape(const WireArgs& a, const uint32_t* tab, uint32_t* part, hipStream_t s) {
    // body lanes per group cover chunks [TS, tn): the longest datagram the shard pitch allows;
    // groups are packed back to back (no rounding), partial sums go per 16-lane row.
    // LINE (when the wire pitch is the 64-B multiple just above HDR + shard pitch): chunks
    // [TS, wire_pitch / 16), so lanes per group is a multiple of 4 and every
    // 64-B line of a row is one store instruction (a line written in two parts costs the
    // memory a read-modify-write: tools/wrskel.hip, profiles/r02zn_wrskel.txt)
    const bool line = a.wire_pitch % 64 == 0 &&
                      a.wire_pitch == (HDR + a.pitch + 63) / 64 * 64 && a.wire_pitch / 16 >= (HDR == 13 ? 20u : 16u);
    // one wave per group (k_pack_wave64): the body's chunks 4.. are 64 lanes at a 1088-B wire
    // pitch (one pass), 32 at 576 B (two groups per wave), up to 128 in two passes above 1088 B
    // (1472 B: 1400-B payloads)
    const int gpw = send_wave_gpw(a.wire_pitch);
    if (HDR == 13 && line && gpw) {
        for (uint64_t g0 = 0; g0 < a.groups; g0 += ((uint64_t)1 << 28)) {
            const uint64_t gn = std::min((uint64_t)1 << 28, a.groups - g0);
            WireArgs b = a;
            b.wire = a.wire + g0 * (uint64_t)(K + M) * a.wire_pitch;
            b.wire_len = a.wire_len + g0 * (K + M);
            const dim3 grid((unsigned)((gn + 4 * (gpw == 2 ? 2 : 1) - 1) / (4 * (gpw == 2 ? 2 : 1))));
            if (gpw == 1)
                hipLaunchKernelGGL((k_pack_wave64<K, M, 1>), grid, dim3(256), 0, s, b, a.payload, a.offsets + g0 * K,
                                   a.sizes + g0 * K, a.seq + 2 * g0, tab, gn, FrameSend{});
            else if (gpw == 10)
                hipLaunchKernelGGL((k_pack_wave64<K, M, 1, 0, 3, 8>), grid, dim3(256), 0, s, b, a.payload,
                                   a.offsets + g0 * K, a.sizes + g0 * K, a.seq + 2 * g0, tab, gn, FrameSend{});
            else
                hipLaunchKernelGGL((k_pack_wave64<K, M, 2>), grid, dim3(256), 0, s, b, a.payload, a.offsets + g0 * K,
                                   a.sizes + g0 * K, a.seq + 2 * g0, tab, gn, FrameSend{});
        }
        return hipGetLastError();
    }
    const uint32_t TS = HDR == 13 ? (line ? 4 : 1) : 0;
    const uint32_t tn = line ? (uint32_t)(a.wire_pitch / 16) : (uint32_t)((HDR + a.pitch + 15) / 16);
    const uint32_t lpg = std::max(16u, tn - TS);
    const DivMagic lpg_div = make_div_magic(lpg);
    // groups per body + head launch pair (keeps g0 * lpg % 16 == 0)
    uint64_t per = (((uint64_t)1 << 30) / lpg) & ~(uint64_t)15;
    per = std::max(per, (uint64_t)16);
    for (uint64_t g0 = 0; g0 < a.groups; g0 += per) {
        const uint64_t gn = std::min(per, a.groups - g0);
        const uint32_t lanes = (uint32_t)(gn * lpg);  // the grid covers whole 16-lane rows past it
        const uint64_t row0 = g0 * lpg / 16;
        if (line)
            hipLaunchKernelGGL((k_pack_body<K, M, HDR, true>), dim3((lanes + 255) / 256), dim3(256), 0, s, a, a.payload,
                               a.offsets, a.sizes, a.seq, tab, part, g0, lanes, lpg, lpg_div, row0);
        else
            hipLaunchKernelGGL((k_pack_body<K, M, HDR, false>), dim3((lanes + 255) / 256), dim3(256), 0, s, a, a.payload,
                               a.offsets, a.sizes, a.seq, tab, part, g0, lanes, lpg, lpg_div, row0);
        if (HDR == 13 && line)
            hipLaunchKernelGGL((k_pack_line0<K, M>), dim3((unsigned)((gn * 4 + 255) / 256)), dim3(256), 0, s, a,
                               a.payload, a.offsets, a.sizes, tab, (const uint32_t*)part, a.seq, a.wire, a.wire_len,
                               g0, (uint32_t)gn, lpg, row0);
        else if (HDR == 13)
            hipLaunchKernelGGL((k_pack_head<K, M>), dim3((unsigned)((gn + 255) / 256)), dim3(256), 0, s, a, a.sizes,
                               tab, (const uint32_t*)part, a.seq, a.wire, a.wire_len, g0, (uint32_t)gn, lpg, row0);
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

// qfec_pack_frames: datagrams and their ProtocolUdp frames in one pass (k_pack_wave64 with a
// frame prefix) where the frame pitch is the 64-B multiple just above prefix + 13 + shard pitch
// and a group fills a wave (1088 B) or half of one (576 B); *launched = false otherwise
template <int K, int M>
hipError_t pack_frames_shape(const WireArgs& a, const FrameSend& fs, int fp, const uint32_t* tab, hipStream_t s,
                             bool* launched) {
    const uint64_t fpitch = a.wire_pitch;
    // frames above 1088 B take the two-pass wave whenever the one-wave send is on: the other way
    // is two calls (datagrams, then frames), 1 577 against 851 us at 1472 B (r03n)
    int gpw = send_wave_gpw(fpitch);
    if (!gpw && fpitch > 1088 && fpitch <= 2112) gpw = 5;
    if (!a.checksum || !gpw || fpitch != (fp + 13 + a.pitch + 63) / 64 * 64) return hipSuccess;
    *launched = true;
    for (uint64_t g0 = 0; g0 < a.groups; g0 += ((uint64_t)1 << 28)) {
        const uint64_t gn = std::min((uint64_t)1 << 28, a.groups - g0);
        WireArgs b = a;
        b.wire = a.wire + g0 * (uint64_t)(K + M) * fpitch;
        b.wire_len = a.wire_len + g0 * (K + M);
        FrameSend f = fs;
        f.mask = fs.mask + g0 * (K + M);
        if (fs.conv_hid) f.conv_hid = fs.conv_hid + 2 * g0 * (K + M);
        const dim3 grid((unsigned)((gn + 4 * (gpw == 2 ? 2 : 1) - 1) / (4 * (gpw == 2 ? 2 : 1))));
#define QFEC_PF(GPW, FP, NP)                                                                                          \
    hipLaunchKernelGGL((k_pack_wave64<K, M, GPW, FP, NP>), grid, dim3(256), 0, s, b, a.payload, a.offsets + g0 * K, \
                       a.sizes + g0 * K, a.seq + 2 * g0, tab, gn, f)
#define QFEC_PF8(FP, NP)                                                                                          \
    hipLaunchKernelGGL((k_pack_wave64<K, M, 1, FP, NP, 8>), grid, dim3(256), 0, s, b, a.payload, a.offsets + g0 * K, \
                       a.sizes + g0 * K, a.seq + 2 * g0, tab, gn, f)
        if (gpw == 10 && fp == 4) QFEC_PF8(4, 3);
        else if (gpw == 10) QFEC_PF8(12, 3);
        else if (gpw == 1 && fp == 4) QFEC_PF(1, 4, 1);
        else if (gpw == 1) QFEC_PF(1, 12, 1);
        else if (gpw == 5 && fp == 4) QFEC_PF(1, 4, 2);
        else if (gpw == 5) QFEC_PF(1, 12, 2);
        else if (fp == 4) QFEC_PF(2, 4, 1);
        else QFEC_PF(2, 12, 1);
#undef QFEC_PF
#undef QFEC_PF8
    }
    return hipGetLastError();
}

hipError_t launch_pack_frames(const WireArgs& a, const FrameSend& fs, int fp, const uint32_t* tab, hipStream_t s,
                              bool* launched) {
    *launched = false;
    if (!a.groups) return hipSuccess;
#define QFEC_PFC(KK, MM) \
    if (a.k == KK && a.m == MM) return pack_frames_shape<KK, MM>(a, fs, fp, tab, s, launched);
    QFEC_PFC(10, 3)
    QFEC_PFC(4, 1)
    QFEC_PFC(4, 2)
    QFEC_PFC(2, 2)
    QFEC_PFC(3, 1)
    QFEC_PFC(3, 2)
    QFEC_PFC(5, 1)
    QFEC_PFC(5, 3)
    QFEC_PFC(7, 1)
    QFEC_PFC(8, 4)
#undef QFEC_PFC
    return hipSuccess;
}

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
