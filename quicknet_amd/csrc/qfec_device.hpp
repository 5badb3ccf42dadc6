// qfec_device.hpp -- device helpers shared by the HIP kernels of libqfec (gfx950).
// GF(2^8) multiply by a constant four bytes per v_perm_b32 (see qfec_kernels.hip header),
// streamed loads/stores, division by a runtime constant.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qfec_internal.hpp"

namespace qfec {

// ------------------------------------------------------------------ GF helpers

// selector words for the three partial products of the 4 bytes in x
struct Sel {
    uint32_t a, b, c;
};

__device__ __forceinline__ Sel gf_sel(uint32_t x) {
    Sel s;
    s.a = x & 0x07070707u;
    s.b = (x >> 3) & 0x07070707u;
    s.c = (x >> 6) & 0x03030303u;
    return s;
}

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// the three partial products of c * x (t = the 5-dword perm table of c)
__device__ __forceinline__ uint32_t pp0(const Sel& s, uint32_t t0, uint32_t t1) { return __builtin_amdgcn_perm(t1, t0, s.a); }
__device__ __forceinline__ uint32_t pp1(const Sel& s, uint32_t t2, uint32_t t3) { return __builtin_amdgcn_perm(t3, t2, s.b); }
__device__ __forceinline__ uint32_t pp2(const Sel& s, uint32_t t4) { return __builtin_amdgcn_perm(t4, t4, s.c); }

// c * x for the four bytes described by s
__device__ __forceinline__ uint32_t gf_mul4(const Sel& s, uint32_t t0, uint32_t t1, uint32_t t2,
                                            uint32_t t3, uint32_t t4) {
    return xor3(pp0(s, t0, t1), pp1(s, t2, t3), pp2(s, t4));
}

// acc ^= c * x over 16 bytes: 3 v_perm_b32 + 2 v_bitop3 per dword
__device__ __forceinline__ void gf_mac16(uint4& acc, const Sel (&s)[4], const uint32_t* __restrict__ t) {
    const uint32_t t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3], t4 = t[4];
    acc.x = xor3(acc.x, pp0(s[0], t0, t1), pp1(s[0], t2, t3)) ^ pp2(s[0], t4);
    acc.y = xor3(acc.y, pp0(s[1], t0, t1), pp1(s[1], t2, t3)) ^ pp2(s[1], t4);
    acc.z = xor3(acc.z, pp0(s[2], t0, t1), pp1(s[2], t2, t3)) ^ pp2(s[2], t4);
    acc.w = xor3(acc.w, pp0(s[3], t0, t1), pp1(s[3], t2, t3)) ^ pp2(s[3], t4);
}

// acc ^= ca * xa ^ cb * xb over 16 bytes: 6 v_perm_b32 + 3 v_bitop3 per dword
__device__ __forceinline__ uint32_t mac2(uint32_t acc, const Sel& a, const Sel& b, const uint32_t* ta,
                                         const uint32_t* tb) {
    acc = xor3(acc, pp0(a, ta[0], ta[1]), pp1(a, ta[2], ta[3]));
    acc = xor3(acc, pp2(a, ta[4]), pp0(b, tb[0], tb[1]));
    return xor3(acc, pp1(b, tb[2], tb[3]), pp2(b, tb[4]));
}

__device__ __forceinline__ void gf_mac16x2(uint4& acc, const Sel (&sa)[4], const Sel (&sb)[4],
                                           const uint32_t* __restrict__ ta, const uint32_t* __restrict__ tb) {
    uint32_t a5[5], b5[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) { a5[i] = ta[i]; b5[i] = tb[i]; }
    acc.x = mac2(acc.x, sa[0], sb[0], a5, b5);
    acc.y = mac2(acc.y, sa[1], sb[1], a5, b5);
    acc.z = mac2(acc.z, sa[2], sb[2], a5, b5);
    acc.w = mac2(acc.w, sa[3], sb[3], a5, b5);
}

// opaque register barrier: uses of v after it cannot be hoisted above it
__device__ __forceinline__ void pin16(uint4& v) {
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}

__device__ __forceinline__ void sel16(Sel (&s)[4], const uint4& v) {
    s[0] = gf_sel(v.x);
    s[1] = gf_sel(v.y);
    s[2] = gf_sel(v.z);
    s[3] = gf_sel(v.w);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// streamed once: non-temporal (the shards are not re-read by this launch)
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
// written once, read by a later launch or the host: non-temporal store (measured on
// MI355X: the encode traffic shape streams at 6.3 TB/s with nt loads + nt stores against
// 5.7 TB/s with plain stores, tools/membench.hip)
__device__ __forceinline__ void st16(uint8_t* p, const uint4& v) {
    const u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

__device__ __forceinline__ uint64_t fast_div(uint64_t n, const DivMagic& d) {
    // n < 2^32 and d.mul < 2^33 (see make_div_magic); exact.
    return d.pow2 ? (n >> d.shift) : ((n * d.mul) >> (32 + d.shift));
}

}  // namespace qfec
