// qfec_wire_device.hpp -- device helpers of the datagram and framing kernels (qfec_wire.hip,
// qfec_rx.hip, qfec_frame.hip): unaligned 16-B loads, byte masks, byte sums, wave sums, XOR words.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

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

// lanes of one wave hand data to each other through LDS: make the order explicit (a release /
// acquire pair at wavefront scope around a wave barrier; no workgroup barrier is needed)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint4 xor16(uint4 v, uint32_t mm) {
    return make_uint4(v.x ^ mm, v.y ^ mm, v.z ^ mm, v.w ^ mm);
}

// 16-byte keep mask for the chunk's bytes below n (n clamped to 0..16), as two 64-bit words
__device__ __forceinline__ void keep_words(int n, uint64_t& lo, uint64_t& hi) {
    const int c = min(max(n, 0), 16);
    lo = c >= 8 ? ~0ull : (1ull << (8 * c)) - 1ull;
    hi = c >= 16 ? ~0ull : c <= 8 ? 0ull : (1ull << (8 * (c - 8))) - 1ull;
}

// XOR with mm only the chunk's bytes below n: a frame's padding stays zero
__device__ __forceinline__ uint4 xor16n(uint4 v, uint32_t mm, int n) {
    return make_uint4(v.x ^ (mm & byte_mask(0, n, 0)), v.y ^ (mm & byte_mask(0, n, 1)), v.z ^ (mm & byte_mask(0, n, 2)),
                      v.w ^ (mm & byte_mask(0, n, 3)));
}

// datagram store: non-temporal or write-back (WireArgs::store_nt), wave-uniform flag
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

static inline unsigned waves_grid(uint64_t waves) { return (unsigned)((waves + 3) / 4); }

}  // namespace qfec
