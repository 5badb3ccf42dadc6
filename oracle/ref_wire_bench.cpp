// ref_wire_bench.cpp -- TEST INFRASTRUCTURE: the CPU baseline for the FEC datagram path.
//
// Drives the reference's own network/FecCodecBuf.cpp + system/fec.c (linked as
// oracle/_ref/libref_feccodec_ref.so, built unchanged by `make -C oracle ref`) the way
// network/NetFecCodec.cpp does for full groups:
//   send    set_fec_enc_buf + pack_fec_head per source packet, get_fec_encoded_pkt +
//           pack_fec_head per check packet            (zfec_pack_input, NetFecCodec.cpp:96-172)
//   receive unpack_fec_head per datagram, set_fec_dec_buf for the first k valid,
//           fec_decode_pkts, dec_src_pkt_info          (zfec_unpack_input, :189-371)
// on one thread, and prints payload GiB/s per direction.  It is the baseline
// tools/wire_bench.py reports beside the GPU kernels; it is never linked into libqfec.
//
//   ref_wire_bench <k> <n> <payload_bytes> <groups> <seconds>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "FecCodecBuf.h"  // the reference header, -I$(REF)/network (read in place)

extern "C" {
void *fec_new(int k, int n);
void fec_free(void *p);
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const int k = argc > 1 ? atoi(argv[1]) : 10, n = argc > 2 ? atoi(argv[2]) : 13;
    const int size = argc > 3 ? atoi(argv[3]) : 1024, groups = argc > 4 ? atoi(argv[4]) : 2000;
    const double budget = argc > 5 ? atof(argv[5]) : 5.0;
    std::vector<unsigned char> payload((size_t)groups * k * size);
    unsigned long long x = 0x5EED0001ull;
    for (auto &b : payload) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; b = (unsigned char)x; }
    FecCodecBuf S, R;
    memset(&S, 0, sizeof S);
    memset(&R, 0, sizeof R);
    init_fec_buf(S, 2048, 16);
    init_fec_buf(R, 2048, 16);
    S.is_send_checksum = true;
    void *codec = fec_new(k, n);
    std::vector<std::vector<unsigned char>> wire((size_t)n, std::vector<unsigned char>(2048 + 64));
    std::vector<int> wlen(n);
    std::vector<std::vector<unsigned char>> got((size_t)n, std::vector<unsigned char>(2048 + 64));
    std::vector<int> glen(n);
    double t_send = 0, t_recv = 0;
    long long sent_groups = 0;
    unsigned long long sink = 0;
    const double t_start = now();
    while (now() - t_start < budget) {
        for (int g = 0; g < groups; ++g) {
            // ---- send one full group
            double t0 = now();
            int en = 0, gmax = 0;
            for (int ik = 0; ik < k; ++ik) {
                const unsigned char *p = payload.data() + ((size_t)g * k + ik) * size;
                const char *shard = set_fec_enc_buf(S, ik, p, size, en);
                gmax = ik == 0 ? en : (en > gmax ? en : gmax);
                FecCodecHead h{(IUINT32)(g * n + ik), (IUINT32)(g * k + ik), (unsigned char)n, (unsigned char)k,
                               (unsigned char)ik};
                int out = 0;
                const char *d = pack_fec_head(S, h, shard, en, out);
                memcpy(wire[ik].data(), d, (size_t)out);
                wlen[ik] = out;
            }
            for (int ik = k; ik < n; ++ik) {
                const char *par = get_fec_encoded_pkt(S, codec, ik, gmax, en);
                FecCodecHead h{(IUINT32)(g * n + ik), (IUINT32)(g * k + k - 1), (unsigned char)n, (unsigned char)k,
                               (unsigned char)ik};
                int out = 0;
                const char *d = pack_fec_head(S, h, par, en, out);
                memcpy(wire[ik].data(), d, (size_t)out);
                wlen[ik] = out;
            }
            double t1 = now();
            // ---- receive with the first n - k datagrams lost (all data: worst case decode)
            reset_fec_dec_buf(R);
            int valid = 0, maxsz = 0;
            for (int ik = n - k; ik < n && valid < k; ++ik) {
                FecCodecHead h;
                int un = 0;
                const char *sh = unpack_fec_head(R, h, (const char *)wire[ik].data(), wlen[ik], un);
                if (!sh) continue;
                memcpy(got[valid].data(), sh, (size_t)un);
                glen[valid] = un;
                maxsz = un > maxsz ? un : maxsz;
                set_fec_dec_buf(R, valid, got[valid].data(), un, ik);
                ++valid;
            }
            if (valid == k) {
                fec_decode_pkts(R, codec, maxsz);
                for (int i = 0; i < k; ++i) {
                    IUINT16 psz = 0;
                    const char *pl = dec_src_pkt_info(get_fec_decoded_pkt(R, i), R, psz);
                    if (pl) sink += (unsigned char)pl[0] + psz;
                }
            }
            double t2 = now();
            t_send += t1 - t0;
            t_recv += t2 - t1;
            ++sent_groups;
        }
    }
    fec_free(codec);
    const double gib = (double)sent_groups * k * size / (1 << 30);
    printf("{\"groups\": %lld, \"k\": %d, \"n\": %d, \"payload\": %d, \"send_gibs\": %.4f, \"recv_gibs\": %.4f, "
           "\"seconds\": %.2f, \"threads\": 1, \"sink\": %llu}\n",
           sent_groups, k, n, size, gib / t_send, gib / t_recv, t_send + t_recv, sink);
    return 0;
}
