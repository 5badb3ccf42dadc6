// tests/zfec_host/stubs.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A CPU build of quicknet_amd/csrc/qfec_zfec.cpp (the exact NetFecCodec layer's host state
// machines) for the CPU suite: the few libqfec device entry points it calls are provided here
// by the oracle's C restatement (oracle/qfec_oracle.c), and the HIP runtime calls by host
// memory.  It lets `pytest -m "not gpu"` compare the state machines' callback sequences with
// oracle/zfec_ref.py without a GPU; the GPU tests (tests/test_gpu_zfec.py) run the same
// scripts through the real libqfec.so.  Never shipped, never loaded by the product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/qfec.h"

extern "C" {
int orc_vandermonde_parity(int k, int n, uint8_t* out);
int orc_pack_group(int k, int n, const uint8_t* rows_full, const uint8_t* payload, const long long* offs,
                   const int* sizes, uint32_t sent0, uint32_t src0, int checksum, int shard_cap, uint8_t* out,
                   long long out_pitch, int* out_len);
int orc_fec_decode(int k, int n, const uint8_t* enc_rows_full, uint8_t** pkt, int* idx, int sz);
int orc_dec_src(const uint8_t* shard, int dec_pkt_size, int checksum, int* size);
uint32_t orc_byte_sum(const uint8_t* p, long long len);
}

struct qfec_code {
    int k, m;
    std::vector<uint8_t> full;  // n x k, identity on top
};

extern "C" {

qfec_code* qfec_code_new(int flavour, int k, int m) {
    if (flavour != QFEC_VANDERMONDE || k < 1 || m < 1 || k + m > 255) return nullptr;
    qfec_code* c = new qfec_code{k, m, std::vector<uint8_t>((size_t)(k + m) * k, 0)};
    for (int i = 0; i < k; ++i) c->full[(size_t)i * k + i] = 1;
    orc_vandermonde_parity(k, k + m, c->full.data() + (size_t)k * k);
    return c;
}

void qfec_code_free(qfec_code* c) { delete c; }

int qfec_pack_datagrams(qfec_code* code, const unsigned char* payload, const long long* offs, const int* sizes,
                        const unsigned int* seq, long long groups, int checksum, unsigned char* shards,
                        long long shard_pitch, unsigned char* wire, long long wire_pitch, int* wire_len, void*) {
    (void)shards;
    const int k = code->k, n = code->k + code->m, head = checksum ? 4 : 2;
    for (long long g = 0; g < groups; ++g) {
        bool ok = true;
        for (int i = 0; i < k; ++i) ok = ok && sizes[g * k + i] >= 0 && sizes[g * k + i] <= shard_pitch - head;
        if (!ok) {
            for (int j = 0; j < n; ++j) wire_len[g * n + j] = -1;
            continue;
        }
        memset(wire + g * n * wire_pitch, 0, (size_t)(n * wire_pitch));
        orc_pack_group(k, n, code->full.data(), payload, offs + g * k, sizes + g * k, seq[2 * g], seq[2 * g + 1],
                       checksum, (int)shard_pitch, wire + g * n * wire_pitch, wire_pitch, wire_len + g * n);
    }
    return QFEC_OK;
}

// the device path's rules (qfec_wire.hip k_parse_wire / reconstruct / k_check_payloads)
int qfec_unpack_datagrams(qfec_code* code, const unsigned char* wire, long long wp, const int* wire_len,
                          long long groups, int checksum, int dec_pkt_size, unsigned char* shards, long long sp,
                          unsigned char* marks, int* rx_size, int* status, int* psize, void*) {
    (void)marks;
    const int k = code->k, n = code->k + code->m;
    std::vector<uint8_t*> pkt(k);
    std::vector<int> idx(k);
    for (long long g = 0; g < groups; ++g) {
        std::vector<int> ok(n, 0);
        for (int j = 0; j < n; ++j) {
            const uint8_t* d = wire + (g * n + j) * wp;
            uint8_t* sh = shards + (g * n + j) * sp;
            memset(sh, 0, (size_t)sp);
            const int len = wire_len[g * n + j];
            bool good = len >= 11 && len <= wp && (d[0] == 0xEC || d[0] == 0xED);
            const int hdr = good && d[0] == 0xED ? 13 : 11;
            good = good && len >= hdr;
            const unsigned ikn = good ? (unsigned)d[9] | (unsigned)d[10] << 8 : 0;
            good = good && (int)(ikn & 15) == n && (int)((ikn >> 4) & 15) == k && (int)((ikn >> 8) & 15) == j;
            good = good && len - hdr <= sp;
            if (good && hdr == 13) good = (orc_byte_sum(d + 13, len - 13) & 0xFFFF) == ((unsigned)d[11] | (unsigned)d[12] << 8);
            if (good) memcpy(sh, d + hdr, (size_t)(len - hdr));
            ok[j] = good;
            if (rx_size) rx_size[g * n + j] = good ? len - hdr : -1;
        }
        int lost = 0, v = 0;
        for (int i = 0; i < k; ++i) lost += ok[i] ? 0 : 1;
        std::vector<std::vector<uint8_t>> bufs;
        bool recovered = false;
        if (lost) {
            for (int j = 0; j < n && v < k; ++j)
                if (ok[j]) {
                    bufs.emplace_back(shards + (g * n + j) * sp, shards + (g * n + j) * sp + sp);
                    idx[v] = j;
                    ++v;
                }
            if (v == k) {
                for (int i = 0; i < k; ++i) pkt[i] = bufs[i].data();
                if (!orc_fec_decode(k, n, code->full.data(), pkt.data(), idx.data(), (int)sp)) {
                    for (int i = 0; i < k; ++i)
                        if (!ok[i]) memcpy(shards + (g * n + i) * sp, pkt[i], (size_t)sp);
                    recovered = true;
                }
            }
        }
        for (int i = 0; i < k; ++i) {
            const uint8_t* sh = shards + (g * n + i) * sp;
            int size = 0;
            int st;
            if (!ok[i] && !recovered) {
                st = -2;
                size = (int)sh[0] | (int)sh[1] << 8;
            } else {
                size = (int)sh[0] | (int)sh[1] << 8;
                st = size >= dec_pkt_size || (checksum ? 4 : 2) + size > sp ? -1
                                                                             : orc_dec_src(sh, dec_pkt_size, checksum, &size);
            }
            status[g * k + i] = st;
            psize[g * k + i] = size;
        }
    }
    return QFEC_OK;
}

// qfec_gather_rows (qfec_wire.hip k_gather_rows): rows copied into the pitched batch, an 0xEC
// header synthesized in front of bare shards (wrap_n > 0)
int qfec_gather_rows(const unsigned char* base, const unsigned long long* off, const int* len, long long rows, int wrap_n,
                     int wrap_k, unsigned char* out, long long out_pitch, int* out_len, void*) {
    const int H = wrap_n > 0 ? 11 : 0;
    for (long long r = 0; r < rows; ++r) {
        const int n = len[r];
        if (n <= 0 || H + n > out_pitch) {
            out_len[r] = n <= 0 ? 0 : -1;
            continue;
        }
        uint8_t* dst = out + r * out_pitch;
        memset(dst, 0, (size_t)out_pitch);
        if (H) {
            const unsigned ikn = (unsigned)wrap_n | (unsigned)wrap_k << 4 | (unsigned)(r % wrap_n) << 8;
            dst[0] = 0xEC;
            dst[9] = (uint8_t)(ikn & 0xFF);
            dst[10] = (uint8_t)(ikn >> 8);
        }
        memcpy(dst + H, base + off[r], (size_t)n);
        out_len[r] = H + n;
    }
    return QFEC_OK;
}

// the HIP runtime, as host memory
hipError_t hipMalloc(void** p, size_t n) {
    *p = malloc(n);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) {
    free(p);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t n, hipMemcpyKind, hipStream_t) {
    memcpy(dst, src, n);
    return hipSuccess;
}
hipError_t hipMemcpy2DAsync(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height,
                            hipMemcpyKind, hipStream_t) {
    for (size_t r = 0; r < height; ++r)
        memcpy(static_cast<uint8_t*>(dst) + r * dpitch, static_cast<const uint8_t*>(src) + r * spitch, width);
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipHostMalloc(void** p, size_t n, unsigned int) {
    *p = malloc(n);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipHostFree(void* p) {
    free(p);
    return hipSuccess;
}
// test hooks: make registration fail, and count the attempts (test_host_arena_register_failure)
int stub_register_fail = 0;
int stub_register_calls = 0;
hipError_t hipHostRegister(void*, size_t, unsigned int) {
    ++stub_register_calls;
    return stub_register_fail ? hipErrorInvalidValue : hipSuccess;
}
hipError_t hipHostUnregister(void*) { return hipSuccess; }
hipError_t hipGetLastError(void) { return hipSuccess; }
hipError_t hipGetDevice(int* d) {
    *d = 0;
    return hipSuccess;
}

}  // extern "C"
