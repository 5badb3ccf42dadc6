// qfec_frame.hip -- ProtocolUdp framing on the device: k_frame_udp /
// k_unframe_udp and their two-rows-per-wave forms (qfec_frame_udp / qfec_unframe_udp), and the
// row gather the exact NetFecCodec layer uses (qfec_gather_rows).  Split out of qfec_wire.hip in round 6.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "qfec_wire_device.hpp"

namespace qfec {

// frames built in LDS and stored flat (k_frame_udp_rows<.., true>)
extern __shared__ uint4 rx_stage[];

// ------------------------------------------------------------------ ProtocolUdp framing
// The byte stage below FEC on every datagram:
//   Session::PacketOutput (network/SessionDesc.cpp:69-77): mask = _mask++, push hid, push conv
//   ProtocolUdp::SendPacket (network/ProtocolBasic.cpp:111-150): push protocol, push
//     (cmd & 0x1f) | 0xA0, push c = CheckSum(all of it) & 0xff, XOR all of it with
//     mask ^ gmask ^ 0x5a, push mask
// so frame = [mask][c][cmd][proto]([conv LE][hid LE])[data], bytes 1.. XORed, with
// CheckSum(x) = ~((s >> 16) + (s & 0xffff)), s = byte sum (ProtocolBasic.cpp:56-87).
// One wave per row, 32 bytes per lane per pass; chunk 0 (which holds c) is written last.

__global__ void __launch_bounds__(256) k_frame_udp(FrameArgs a) {
    const uint64_t row = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (row >= a.rows) return;
    const int lane = threadIdx.x & 63;
    const int P = a.session ? 12 : 4;
    const int len = a.in_len[row];
    const int total = P + len;
    const uint8_t* in = a.in + row * a.in_pitch;
    uint8_t* out = a.out + row * a.out_pitch;
    if (len < 0 || total > (int)a.out_pitch || len > (int)a.in_pitch) {
        for (int o = 16 * lane; o < (int)a.out_pitch; o += 1024) st16a(out + o, make_uint4(0, 0, 0, 0));
        if (lane == 0) a.out_len[row] = -1;
        return;
    }
    for (int o = 16 * ((total + 15) / 16) + 16 * lane; o < (int)a.out_pitch; o += 1024)  // zero padding
        st16a(out + o, make_uint4(0, 0, 0, 0));
    const uint32_t m = a.mask[row];
    const uint32_t x = (m ^ a.gmask ^ 0x5Au) & 0xFFu;
    const uint32_t mm = x * 0x01010101u;
    const int in_chunks = (int)(a.in_pitch / 16);
    uint32_t sum = 0;
    uint4 first = make_uint4(0, 0, 0, 0);
    for (int q0 = 2 * lane; 16 * q0 < total; q0 += 128) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = q0 + h;
            if (16 * q >= total) break;
            // frame bytes [16q, 16q + 16) = data bytes [16q - P, 16q + 16 - P)
            const uint4 lo = q >= 1 ? *reinterpret_cast<const uint4*>(in + 16 * (q - 1)) : make_uint4(0, 0, 0, 0);
            const uint4 hi = q < in_chunks ? *reinterpret_cast<const uint4*>(in + 16 * q) : make_uint4(0, 0, 0, 0);
            uint4 v = mask16(window(lo, hi, 16 - P), q == 0 ? P : 0, total - 16 * q);
            sum = sum16(v, sum);
            if (q == 0) {
                first = v;
            } else {
                st16a(out + 16 * q, xor16n(v, mm, total - 16 * q));
            }
        }
    }
    sum = wave_sum(sum);
    if (lane == 0) {
        const uint32_t cmd = (a.cmd & 0x1Fu) | 0xA0u, proto = a.protocol & 0xFFu;
        put_byte(first, 2, cmd);
        put_byte(first, 3, proto);
        uint32_t s2 = sum + cmd + proto;
        if (a.session) {
            const uint32_t conv = a.conv_hid[2 * row], hid = a.conv_hid[2 * row + 1];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                put_byte(first, 4 + b, conv >> (8 * b));
                put_byte(first, 8 + b, hid >> (8 * b));
                s2 += ((conv >> (8 * b)) & 0xFFu) + ((hid >> (8 * b)) & 0xFFu);
            }
        }
        const uint32_t c = ~((s2 >> 16) + (s2 & 0xFFFFu)) & 0xFFu;
        put_byte(first, 1, c);
        first = xor16n(first, mm, total);
        put_byte(first, 0, m);
        st16a(out, first);
        a.out_len[row] = total;
    }
}

// k_frame_udp over ROWS rows per wave with every load issued before any use: one row per wave
// keeps ~1 KB in flight per wave, too little to cover the
// memory latency at this kernel's occupancy; ROWS rows put ROWS times as many bytes in flight.
// Rows of at most 2 048 B (one pass of two 16-B chunks per lane); the host checks.
// STAGE (the launch uses ROWS 2 with STAGE): the ROWS output rows are built in LDS (zeroed first) and stored as one
// flat range, so no 64-B line of the output is written in two parts by one wave; rows with
// out_len -1 then read back zeros instead of being left untouched
template <int ROWS, bool STAGE = false>
__global__ void __launch_bounds__(256) k_frame_udp_rows(FrameArgs a) {
    const uint64_t row0 = ((uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6)) * ROWS;
    if (row0 >= a.rows) return;
    const int lane = threadIdx.x & 63;
    const int P = a.session ? 12 : 4;
    const int in_chunks = (int)(a.in_pitch / 16);
    int len[ROWS], total[ROWS];
    bool good[ROWS];
#pragma unroll
    for (int i = 0; i < ROWS; ++i) {
        len[i] = row0 + i < a.rows ? a.in_len[row0 + i] : -1;
        total[i] = P + len[i];
        good[i] = row0 + i < a.rows && len[i] >= 0 && total[i] <= (int)a.out_pitch && len[i] <= (int)a.in_pitch;
    }
    uint4* const region = STAGE ? rx_stage + (threadIdx.x >> 6) * (ROWS * a.out_pitch / 16) : nullptr;
    if constexpr (STAGE) {
        for (int o = lane; o < (int)(ROWS * a.out_pitch / 16); o += 64) region[o] = make_uint4(0, 0, 0, 0);
        wave_lds_sync();
    }
    uint4 lo[ROWS][2], hi[ROWS][2];
#pragma unroll
    for (int i = 0; i < ROWS; ++i) {
        const uint8_t* in = a.in + (row0 + i) * a.in_pitch;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = 2 * lane + h;
            lo[i][h] = hi[i][h] = make_uint4(0, 0, 0, 0);
            if (good[i] && 16 * q < total[i]) {
                if (q >= 1) lo[i][h] = *reinterpret_cast<const uint4*>(in + 16 * (q - 1));
                if (q < in_chunks) hi[i][h] = *reinterpret_cast<const uint4*>(in + 16 * q);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < ROWS; ++i) {
        const uint64_t row = row0 + i;
        if (row >= a.rows) break;
        uint8_t* out = STAGE ? reinterpret_cast<uint8_t*>(region) + i * a.out_pitch : a.out + row * a.out_pitch;
        if (!good[i]) {  // a rejected row reads back zeros (staged: the zeroed region)
            if (!STAGE) {
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (16 * (2 * lane + h) < (int)a.out_pitch) st16a(out + 16 * (2 * lane + h), make_uint4(0, 0, 0, 0));
            }
            if (lane == 0) a.out_len[row] = -1;
            continue;
        }
        const uint32_t m = a.mask[row];
        const uint32_t x = (m ^ a.gmask ^ 0x5Au) & 0xFFu;
        const uint32_t mm = x * 0x01010101u;
        uint32_t sum = 0;
        uint4 first = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = 2 * lane + h;
            if (16 * q >= total[i]) {  // padding up to the pitch is zero (staged: already)
                if (!STAGE && 16 * q < (int)a.out_pitch) st16a(out + 16 * q, make_uint4(0, 0, 0, 0));
                continue;
            }
            // frame bytes [16q, 16q + 16) = data bytes [16q - P, 16q + 16 - P)
            uint4 v = mask16(window(lo[i][h], hi[i][h], 16 - P), q == 0 ? P : 0, total[i] - 16 * q);
            sum = sum16(v, sum);
            if (q == 0) first = v;
            else st16a(out + 16 * q, xor16n(v, mm, total[i] - 16 * q));
        }
        sum = wave_sum(sum);
        if (lane == 0) {
            const uint32_t cmd = (a.cmd & 0x1Fu) | 0xA0u, proto = a.protocol & 0xFFu;
            put_byte(first, 2, cmd);
            put_byte(first, 3, proto);
            uint32_t s2 = sum + cmd + proto;
            if (a.session) {
                const uint32_t conv = a.conv_hid[2 * row], hid = a.conv_hid[2 * row + 1];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    put_byte(first, 4 + b, conv >> (8 * b));
                    put_byte(first, 8 + b, hid >> (8 * b));
                    s2 += ((conv >> (8 * b)) & 0xFFu) + ((hid >> (8 * b)) & 0xFFu);
                }
            }
            const uint32_t c = ~((s2 >> 16) + (s2 & 0xFFFFu)) & 0xFFu;
            put_byte(first, 1, c);
            first = xor16n(first, mm, total[i]);
            put_byte(first, 0, m);
            st16a(out, first);
            a.out_len[row] = total[i];
        }
    }
    if constexpr (STAGE) {
        wave_lds_sync();
        const uint64_t nrows = min((uint64_t)ROWS, a.rows - row0);
        uint8_t* dst = a.out + row0 * a.out_pitch;
        for (int o = 16 * lane; o < (int)(nrows * a.out_pitch); o += 1024) st16(dst + o, region[o >> 4]);
    }
}

// Reverse (ProtocolUdp::RecvPacket, ProtocolBasic.cpp:152-210): status 0 ok, 1 shorter than 4
// bytes (or than the 12 with the Session prefix), 2 checksum, 3 cmd (& 0xe0 != 0xA0), 4 does
// not fit the output pitch.  The data (frame bytes [P, len), un-XORed) is written for every
// status but 1 and 4; out_len = len - P.
__global__ void __launch_bounds__(256) k_unframe_udp(FrameArgs a) {
    const uint64_t row = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (row >= a.rows) return;
    const int lane = threadIdx.x & 63;
    const int P = a.session ? 12 : 4;
    const int len = a.in_len[row];
    const uint8_t* in = a.in + row * a.in_pitch;
    uint8_t* out = a.out + row * a.out_pitch;
    if (len < P || len > (int)a.in_pitch || len - P > (int)a.out_pitch) {
        if (lane == 0) {
            a.status[row] = len < P ? 1 : 4;
            a.out_len[row] = -1;
        }
        return;
    }
    const uint4 h0 = *reinterpret_cast<const uint4*>(in);
    const uint32_t x = (get_byte(h0, 0) ^ a.gmask ^ 0x5Au) & 0xFFu;
    const uint32_t mm = x * 0x01010101u;
    const int in_chunks = (int)(a.in_pitch / 16);
    const int dlen = len - P;
    uint32_t sum = 0;  // frame bytes [2, len), un-XORed
    for (int q0 = 2 * lane; 16 * q0 < len; q0 += 128) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = q0 + h;
            if (16 * q >= len) break;
            const uint4 f = xor16(*reinterpret_cast<const uint4*>(in + 16 * q), mm);
            sum = sum16(mask16(f, 2 - 16 * q, len - 16 * q), sum);
            // data chunk q = frame bytes [16q + P, 16q + P + 16)
            if (16 * q < dlen) {
                const uint4 nx = q + 1 < in_chunks ? xor16(*reinterpret_cast<const uint4*>(in + 16 * (q + 1)), mm)
                                                   : make_uint4(0, 0, 0, 0);
                st16a(out + 16 * q, mask16(window(f, nx, P), 0, dlen - 16 * q));
            }
        }
    }
    sum = wave_sum(sum);
    if (lane == 0) {
        const uint4 f0 = xor16(h0, mm);
        const uint32_t check = get_byte(f0, 1), cmd = get_byte(f0, 2);
        const uint32_t c = ~((sum >> 16) + (sum & 0xFFFFu)) & 0xFFu;
        a.status[row] = c != check ? 2 : (cmd & 0xE0u) != 0xA0u ? 3 : 0;
        a.out_len[row] = dlen;
        if (a.info) {
            a.info[4 * row + 0] = (uint8_t)x;
            a.info[4 * row + 1] = (uint8_t)check;
            a.info[4 * row + 2] = (uint8_t)(cmd & 0x1Fu);
            a.info[4 * row + 3] = (uint8_t)get_byte(f0, 3);
        }
        if (a.session && a.conv_hid) {
            uint32_t conv = 0, hid = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                conv |= get_byte(f0, 4 + b) << (8 * b);
                hid |= get_byte(f0, 8 + b) << (8 * b);
            }
            a.conv_hid[2 * row] = conv;
            a.conv_hid[2 * row + 1] = hid;
        }
    }
}

// k_unframe_udp over ROWS rows per wave, every load issued before any use (as
// k_frame_udp_rows); rows of at most 2 048 B
template <int ROWS>
__global__ void __launch_bounds__(256) k_unframe_udp_rows(FrameArgs a) {
    const uint64_t row0 = ((uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6)) * ROWS;
    if (row0 >= a.rows) return;
    const int lane = threadIdx.x & 63;
    const int P = a.session ? 12 : 4;
    const int in_chunks = (int)(a.in_pitch / 16);
    int len[ROWS];
    bool good[ROWS];
#pragma unroll
    for (int i = 0; i < ROWS; ++i) {
        len[i] = row0 + i < a.rows ? a.in_len[row0 + i] : 0;
        good[i] = row0 + i < a.rows && len[i] >= P && len[i] <= (int)a.in_pitch && len[i] - P <= (int)a.out_pitch;
    }
    uint4 f[ROWS][2], nx[ROWS][2], h0[ROWS];
#pragma unroll
    for (int i = 0; i < ROWS; ++i) {
        const uint8_t* in = a.in + (row0 + i) * a.in_pitch;
        h0[i] = good[i] ? *reinterpret_cast<const uint4*>(in) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = 2 * lane + h;
            f[i][h] = nx[i][h] = make_uint4(0, 0, 0, 0);
            if (good[i] && 16 * q < len[i]) {
                f[i][h] = *reinterpret_cast<const uint4*>(in + 16 * q);
                if (16 * q < len[i] - P && q + 1 < in_chunks) nx[i][h] = *reinterpret_cast<const uint4*>(in + 16 * (q + 1));
            }
        }
    }
#pragma unroll
    for (int i = 0; i < ROWS; ++i) {
        const uint64_t row = row0 + i;
        if (row >= a.rows) break;
        if (!good[i]) {
            if (lane == 0) {
                a.status[row] = len[i] < P ? 1 : 4;
                a.out_len[row] = -1;
            }
            continue;
        }
        uint8_t* out = a.out + row * a.out_pitch;
        const uint32_t x = (get_byte(h0[i], 0) ^ a.gmask ^ 0x5Au) & 0xFFu;
        const uint32_t mm = x * 0x01010101u;
        const int dlen = len[i] - P;
        uint32_t sum = 0;  // frame bytes [2, len), un-XORed
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = 2 * lane + h;
            if (16 * q >= len[i]) continue;
            const uint4 fv = xor16(f[i][h], mm);
            sum = sum16(mask16(fv, 2 - 16 * q, len[i] - 16 * q), sum);
            // data chunk q = frame bytes [16q + P, 16q + P + 16)
            if (16 * q < dlen) st16a(out + 16 * q, mask16(window(fv, xor16(nx[i][h], mm), P), 0, dlen - 16 * q));
        }
        sum = wave_sum(sum);
        if (lane == 0) {
            const uint4 f0 = xor16(h0[i], mm);
            const uint32_t check = get_byte(f0, 1), cmd = get_byte(f0, 2);
            const uint32_t c = ~((sum >> 16) + (sum & 0xFFFFu)) & 0xFFu;
            a.status[row] = c != check ? 2 : (cmd & 0xE0u) != 0xA0u ? 3 : 0;
            a.out_len[row] = dlen;
            if (a.info) {
                a.info[4 * row + 0] = (uint8_t)x;
                a.info[4 * row + 1] = (uint8_t)check;
                a.info[4 * row + 2] = (uint8_t)(cmd & 0x1Fu);
                a.info[4 * row + 3] = (uint8_t)get_byte(f0, 3);
            }
            if (a.session && a.conv_hid) {
                uint32_t conv = 0, hid = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    conv |= get_byte(f0, 4 + b) << (8 * b);
                    hid |= get_byte(f0, 8 + b) << (8 * b);
                }
                a.conv_hid[2 * row] = conv;
                a.conv_hid[2 * row + 1] = hid;
            }
        }
    }
}


// qfec_gather_rows: scattered rows (datagrams in a receive ring, or bare shards with an 11-byte
// 0xEC header synthesized in front when wrap_n > 0) into the pitched batch the datagram calls
// take.  One wave per row, 16-B chunks per lane, zero padding to the pitch; rows of len <= 0
// get out_len 0 and are not written.
__global__ void __launch_bounds__(256) k_gather_rows(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                                     const int32_t* __restrict__ len, uint64_t rows, int wrap_n, int wrap_k,
                                                     uint8_t* __restrict__ out, uint64_t out_pitch,
                                                     int32_t* __restrict__ out_len) {
    const uint64_t row = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int lane = threadIdx.x & 63;
    const int n = len[row];
    const int H = wrap_n > 0 ? 11 : 0;
    if (n <= 0 || H + n > (int)out_pitch) {
        if (lane == 0) out_len[row] = n <= 0 ? 0 : -1;
        return;
    }
    const uint8_t* src = base + off[row];
    uint8_t* dst = out + row * out_pitch;
    for (int q = lane; 16 * q < (int)out_pitch; q += 64) {
        uint4 v;
        if (H && q == 0) {  // [0xEC][sent 0][src 0][n | k << 4 | ik << 8] + the shard's first 5 bytes
            v = window(make_uint4(0, 0, 0, 0), ldu16(src), 16 - H);
            const uint32_t ikn = (uint32_t)wrap_n | (uint32_t)wrap_k << 4 | (uint32_t)(row % (uint64_t)wrap_n) << 8;
            v.x = 0xECu;
            v.y = 0;
            v.z = (v.z & 0xFF000000u) | ((ikn & 0xFFFFu) << 8);
        } else {
            v = 16 * q - H < n ? ldu16(src + 16 * q - H) : make_uint4(0, 0, 0, 0);
        }
        st16a(dst + 16 * q, mask16(v, 0, H + n - 16 * q));
    }
    if (lane == 0) out_len[row] = H + n;
}

hipError_t launch_gather_rows(const uint8_t* base, const uint64_t* off, const int32_t* len, uint64_t rows, int wrap_n,
                              int wrap_k, uint8_t* out, uint64_t out_pitch, int32_t* out_len, hipStream_t s) {
    if (!rows) return hipSuccess;
    hipLaunchKernelGGL(k_gather_rows, dim3(waves_grid(rows)), dim3(256), 0, s, base, off, len, rows, wrap_n, wrap_k, out,
                       out_pitch, out_len);
    return hipGetLastError();
}

// rows whose RecvPacket verdict is not 0 are not received (the fallback of qfec_unpack_frames)
__global__ void __launch_bounds__(256) k_len_by_status(int32_t* __restrict__ len, const int32_t* __restrict__ status,
                                                       uint64_t rows) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i < rows && status[i] != 0) len[i] = 0;
}

hipError_t launch_len_by_status(int32_t* len, const int32_t* status, uint64_t rows, hipStream_t s) {
    if (!rows) return hipSuccess;
    hipLaunchKernelGGL(k_len_by_status, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, len, status, rows);
    return hipGetLastError();
}

hipError_t launch_frame_udp(const FrameArgs& a, hipStream_t s) {
    if (!a.rows) return hipSuccess;
    if (a.in_pitch <= 2048 && a.out_pitch <= 2048) {
        // two rows per wave, their loads issued first; frames built in LDS and stored flat where
        // the output pitch allows it (701 against 671 us stored directly, on the bench's 1.3 M
        // datagrams); one row per wave and four rows per wave measured slower
        // (the ABI's pitches are multiples of 16)
        hipLaunchKernelGGL((k_frame_udp_rows<2, true>), dim3(waves_grid((a.rows + 1) / 2)), dim3(256),
                           4 * 2 * a.out_pitch, s, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_frame_udp, dim3(waves_grid(a.rows)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_unframe_udp(const FrameArgs& a, hipStream_t s) {
    if (!a.rows) return hipSuccess;
    if (a.in_pitch <= 2048 && a.out_pitch <= 2048) {
        hipLaunchKernelGGL(k_unframe_udp_rows<2>, dim3(waves_grid((a.rows + 1) / 2)), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_unframe_udp, dim3(waves_grid(a.rows)), dim3(256), 0, s, a);
    return hipGetLastError();
}


}  // namespace qfec
