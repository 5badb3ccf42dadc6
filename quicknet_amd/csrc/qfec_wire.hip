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
    for (int i = 0; i < a.k; ++i) gmax = max(gmax, a.sizes[g * a.k + i] + head);
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

// ------------------------------------------------------------------ launchers
static inline unsigned waves_grid(uint64_t waves) { return (unsigned)((waves + 3) / 4); }

hipError_t launch_build_shards(const WireArgs& a, hipStream_t s) {
    const uint64_t rows = a.groups * (uint64_t)a.k;
    if (!rows) return hipSuccess;
    hipLaunchKernelGGL(k_build_shards, dim3(waves_grid(rows)), dim3(256), 0, s, a);
    return hipGetLastError();
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
