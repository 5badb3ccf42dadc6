// rxskel.hip -- the memory skeleton of the fused datagram receive (qfec_wire.hip k_unpack_*),
// no GF arithmetic: per group, read K datagram rows at byte offset HDR of rows of WP bytes and
// write K shard rows of PITCH bytes.  Which part of the receive's time the access pattern
// alone explains, per layout choice:
//   w2x8    2 waves per group (one workgroup), 8 B per lane + tail dwords (k_unpack_wg's map)
//   w1x16   1 wave per group, 16 B per lane + tail dwords, 2 passes (k_unpack_fused's map)
//   flat    lanes flat over (group, 16-B chunk): no per-group waves at all
// each at HDR = 13 (the wire format) and HDR = 16 (aligned, for comparison).
//   hipcc --offload-arch=gfx950 -O3 tools/rxskel.hip -o /tmp/rxskel && /tmp/rxskel
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int K = 10, N = 13;

__global__ void __launch_bounds__(256) k_w2x8(const uint8_t* __restrict__ wire, uint8_t* __restrict__ out, int wp,
                                              int pitch, int hdr) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, W = blockDim.x >> 6;
    const uint64_t g = blockIdx.x;
    const uint8_t* wg = wire + g * N * (uint64_t)wp + hdr;
    uint8_t* og = out + g * N * (uint64_t)pitch;
    const int pa = 512 * w + 8 * lane, pt = 512 * W + 256 * w + 4 * lane;
    u32x2 x[K];
    uint32_t t[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        if (pa < pitch) __builtin_memcpy(&x[c], wg + (uint64_t)c * wp + pa, 8);
        if (pt < pitch) __builtin_memcpy(&t[c], wg + (uint64_t)c * wp + pt, 4);
    }
#pragma unroll
    for (int c = 0; c < K; ++c) {
        if (pa < pitch) __builtin_nontemporal_store(x[c], reinterpret_cast<u32x2*>(og + (uint64_t)c * pitch + pa));
        if (pt < pitch) __builtin_nontemporal_store(t[c], reinterpret_cast<uint32_t*>(og + (uint64_t)c * pitch + pt));
    }
}

__global__ void __launch_bounds__(256) k_w1x16(const uint8_t* __restrict__ wire, uint8_t* __restrict__ out,
                                               uint64_t groups, int wp, int pitch, int hdr) {
    const int lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= groups) return;
    const uint8_t* wg = wire + g * N * (uint64_t)wp + hdr;
    uint8_t* og = out + g * N * (uint64_t)pitch;
    for (int p0 = 0; p0 < pitch; p0 += 1024) {
        const int pa = p0 + 16 * lane;
        u32x4 x[K];
#pragma unroll
        for (int c = 0; c < K; ++c)
            if (pa < pitch) __builtin_memcpy(&x[c], wg + (uint64_t)c * wp + pa, 16);
#pragma unroll
        for (int c = 0; c < K; ++c)
            if (pa < pitch) __builtin_nontemporal_store(x[c], reinterpret_cast<u32x4*>(og + (uint64_t)c * pitch + pa));
    }
}

// 1 wave per group, 16 B per lane over [0, 1024) + one tail dword per lane past it, one pass
__global__ void __launch_bounds__(256) k_w1x16t(const uint8_t* __restrict__ wire, uint8_t* __restrict__ out,
                                                uint64_t groups, int wp, int pitch, int hdr) {
    const int lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= groups) return;
    const uint8_t* wg = wire + g * N * (uint64_t)wp + hdr;
    uint8_t* og = out + g * N * (uint64_t)pitch;
    const int pa = 16 * lane, pt = 1024 + 4 * lane;
    u32x4 x[K];
    uint32_t t[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        if (pa < pitch) __builtin_memcpy(&x[c], wg + (uint64_t)c * wp + pa, 16);
        if (pt < pitch) __builtin_memcpy(&t[c], wg + (uint64_t)c * wp + pt, 4);
    }
#pragma unroll
    for (int c = 0; c < K; ++c) {
        if (pa < pitch) __builtin_nontemporal_store(x[c], reinterpret_cast<u32x4*>(og + (uint64_t)c * pitch + pa));
        if (pt < pitch) __builtin_nontemporal_store(t[c], reinterpret_cast<uint32_t*>(og + (uint64_t)c * pitch + pt));
    }
}

// 1 wave per group: rows into LDS (16 B per lane + tail dwords), then the group's K output rows
// written as ONE flat byte range, 1 KiB per wave instruction across row boundaries (full
// 64-B lines even when the row pitch is not a multiple of 64)
__global__ void __launch_bounds__(256) k_w1lds(const uint8_t* __restrict__ wire, uint8_t* __restrict__ out,
                                               uint64_t groups, int wp, int pitch, int hdr) {
    extern __shared__ uint8_t lds[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t g = (uint64_t)blockIdx.x * 4 + wv;
    if (g >= groups) return;
    uint8_t* L = lds + wv * K * pitch;
    const uint8_t* wg = wire + g * N * (uint64_t)wp + hdr;
    uint8_t* og = out + g * N * (uint64_t)pitch;
    const int pa = 16 * lane, pt = 1024 + 4 * lane;
    u32x4 x[K];
    uint32_t t[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        if (pa < pitch) __builtin_memcpy(&x[c], wg + (uint64_t)c * wp + pa, 16);
        if (pt < pitch) __builtin_memcpy(&t[c], wg + (uint64_t)c * wp + pt, 4);
    }
#pragma unroll
    for (int c = 0; c < K; ++c) {
        if (pa < pitch) *reinterpret_cast<u32x4*>(L + c * pitch + pa) = x[c];
        if (pt < pitch) *reinterpret_cast<uint32_t*>(L + c * pitch + pt) = t[c];
    }
    __builtin_amdgcn_s_waitcnt(0);  // (one wave: its own LDS writes are visible in order)
    const int total = K * pitch;
    for (int o = 16 * lane; o < total; o += 1024)
        __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(L + o), reinterpret_cast<u32x4*>(og + o));
}

// w1x16t, stores: MODE 0 all plain (L2 merges the two halves of a row-boundary line), 1 plain
// for the boundary lines only (each row's first 64 B and its tail dwords), nt elsewhere
template <int MODE>
__global__ void __launch_bounds__(256) k_w1x16t_st(const uint8_t* __restrict__ wire, uint8_t* __restrict__ out,
                                                   uint64_t groups, int wp, int pitch, int hdr) {
    const int lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= groups) return;
    const uint8_t* wg = wire + g * N * (uint64_t)wp + hdr;
    uint8_t* og = out + g * N * (uint64_t)pitch;
    const int pa = 16 * lane, pt = 1024 + 4 * lane;
    u32x4 x[K];
    uint32_t t[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        if (pa < pitch) __builtin_memcpy(&x[c], wg + (uint64_t)c * wp + pa, 16);
        if (pt < pitch) __builtin_memcpy(&t[c], wg + (uint64_t)c * wp + pt, 4);
    }
#pragma unroll
    for (int c = 0; c < K; ++c) {
        u32x4* d = reinterpret_cast<u32x4*>(og + (uint64_t)c * pitch + pa);
        if (pa < pitch) {
            if (MODE == 0 || lane < 4) *d = x[c];
            else __builtin_nontemporal_store(x[c], d);
        }
        if (pt < pitch) *reinterpret_cast<uint32_t*>(og + (uint64_t)c * pitch + pt) = t[c];
    }
}

// w1x16t with the K rows' tails gathered: lane l < 4K loads dword (l & 3) of row (l >> 2)'s tail,
// so all tails are ONE load and ONE store instruction instead of K each
__global__ void __launch_bounds__(256) k_w1x16c(const uint8_t* __restrict__ wire, uint8_t* __restrict__ out,
                                                uint64_t groups, int wp, int pitch, int hdr) {
    const int lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= groups) return;
    const uint8_t* wg = wire + g * N * (uint64_t)wp + hdr;
    uint8_t* og = out + g * N * (uint64_t)pitch;
    const int pa = 16 * lane;
    const int tr = lane >> 2, tp = 1024 + 4 * (lane & 3);
    const bool tact = tr < K && tp < pitch;
    u32x4 x[K];
    uint32_t t = 0;
#pragma unroll
    for (int c = 0; c < K; ++c)
        if (pa < pitch) __builtin_memcpy(&x[c], wg + (uint64_t)c * wp + pa, 16);
    if (tact) __builtin_memcpy(&t, wg + (uint64_t)tr * wp + tp, 4);
#pragma unroll
    for (int c = 0; c < K; ++c)
        if (pa < pitch) __builtin_nontemporal_store(x[c], reinterpret_cast<u32x4*>(og + (uint64_t)c * pitch + pa));
    if (tact) __builtin_nontemporal_store(t, reinterpret_cast<uint32_t*>(og + (uint64_t)tr * pitch + tp));
}

// lanes flat over (group, row, 16-B chunk)
__global__ void __launch_bounds__(256) k_flat(const uint8_t* __restrict__ wire, uint8_t* __restrict__ out,
                                              uint64_t items, int wp, int pitch, int hdr, int cpr) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= items) return;
    const uint64_t row = i / cpr;
    const int ch = (int)(i - row * cpr);
    const uint64_t g = row / K;
    const int c = (int)(row - g * K);
    u32x4 x;
    __builtin_memcpy(&x, wire + (g * N + c) * (uint64_t)wp + hdr + 16 * ch, 16);
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(out + (g * N + c) * (uint64_t)pitch + 16 * ch));
}

int main() {
    const uint64_t G = 100000;
    const int pitches[2] = {1040, 1088};
    for (int pi = 0; pi < 2; ++pi) {
        const int pitch = pitches[pi], wp = (pitch + 13 + 15) / 16 * 16 + 16;
        uint8_t *wire, *out;
        CHECK(hipMalloc(&wire, G * N * wp + 64));
        CHECK(hipMalloc(&out, G * N * pitch));
        CHECK(hipMemset(wire, 7, G * N * wp + 64));
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        const double bytes = 2.0 * G * K * pitch;  // (pitch 1088 / 1472: 64-B aligned rows, more bytes)
        for (int round = 0; round < 2; ++round) {
            for (int hdr : {13}) {
                for (int v = 0; v < 8; ++v) {
                    const unsigned W = (pitch + 767) / 768;
                    const int cpr = pitch / 16;
                    auto launch = [&]() {
                        if (v == 0) k_w2x8<<<(unsigned)G, 64 * W>>>(wire, out, wp, pitch, hdr);
                        else if (v == 1) k_w1x16<<<(unsigned)((G + 3) / 4), 256>>>(wire, out, G, wp, pitch, hdr);
                        else if (v == 5) k_w1x16t_st<0><<<(unsigned)((G + 3) / 4), 256>>>(wire, out, G, wp, pitch, hdr);
                        else if (v == 6) k_w1x16t_st<1><<<(unsigned)((G + 3) / 4), 256>>>(wire, out, G, wp, pitch, hdr);
                        else if (v == 4) k_w1lds<<<(unsigned)((G + 3) / 4), 256, 4 * K * pitch>>>(wire, out, G, wp, pitch, hdr);
                        else if (v == 7) k_w1x16c<<<(unsigned)((G + 3) / 4), 256>>>(wire, out, G, wp, pitch, hdr);
                        else if (v == 3) k_w1x16t<<<(unsigned)((G + 3) / 4), 256>>>(wire, out, G, wp, pitch, hdr);
                        else k_flat<<<(unsigned)((G * K * cpr + 255) / 256), 256>>>(wire, out, G * K * cpr, wp, pitch, hdr, cpr);
                    };
                    for (int w = 0; w < 3; ++w) launch();
                    CHECK(hipEventRecord(a, 0));
                    for (int r = 0; r < 20; ++r) launch();
                    CHECK(hipEventRecord(b, 0));
                    CHECK(hipEventSynchronize(b));
                    float ms = 0;
                    CHECK(hipEventElapsedTime(&ms, a, b));
                    ms /= 20;
                    const char* names[8] = {"w2x8 ", "w1x16", "flat ", "w1x16t", "w1lds", "w1x16t-plain", "w1x16t-edgeplain", "w1x16c (tails gathered)"};
                    if (round == 1)
                        printf("pitch %4d hdr %2d %s %8.1f us  %7.1f GB/s (read + write)\n", pitch, hdr, names[v],
                               ms * 1e3, bytes / (ms * 1e-3) / 1e9);
                }
            }
        }
        CHECK(hipFree(wire));
        CHECK(hipFree(out));
    }
    return 0;
}
