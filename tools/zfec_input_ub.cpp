// tools/zfec_input_ub.cpp -- measurement aid: cost of qfec_zfec_unpack_input per datagram (warm
// arenas) against a bare loop doing the same copy into a 16-B aligned arena plus an op record,
// so the layer's per-call overhead over the copy itself is visible.  Build: see gpu_r05h.sh.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "../include/qfec_zfec.h"

struct OpRec {
    uint8_t t;
    uint32_t off, size;
    int a, b, c;
    float f;
    uint64_t uid;
};

int main() {
    const size_t N = 153600, L = 1041, P = 1104;
    std::vector<uint8_t> src(N * P + 64);
    for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 131);
    for (size_t i = 0; i < N; ++i) {
        uint8_t* d = &src[i * P];
        d[0] = 0xED;
        d[9] = 0x3d;
        d[10] = (uint8_t)(i % 13);
    }
    qfec_zfec* z = qfec_zfec_new();
    int ss[64];
    for (int s = 0; s < 64; ++s) ss[s] = qfec_zfec_session(z, (void*)(intptr_t)(s + 1), 2048, 48, 15, 10, 13, 1, 0);
    for (int rep = 0; rep < 5; ++rep) {
        auto t0 = std::chrono::steady_clock::now();
        for (size_t i = 0; i < N; ++i) qfec_zfec_unpack_input(z, ss[(i / 12) % 64], &src[i * P], L);
        auto t1 = std::chrono::steady_clock::now();
        printf("qfec_zfec_unpack_input: %.1f ns/datagram (%.2f GB/s)\n",
               std::chrono::duration<double, std::nano>(t1 - t0).count() / N,
               N * L / std::chrono::duration<double>(t1 - t0).count() / 1e9);
        qfec_zfec_flush(z, nullptr, nullptr, nullptr);
    }
    std::vector<uint8_t> arena(N * 1120 + 64);
    std::vector<std::vector<OpRec>> ops(64);
    std::mutex mu;
    for (int rep = 0; rep < 5; ++rep) {
        for (auto& o : ops) o.clear();
        size_t used = 0;
        auto t0 = std::chrono::steady_clock::now();
        for (size_t i = 0; i < N; ++i) {
            std::lock_guard<std::mutex> lk(mu);
            const size_t o = (used + 15) & ~(size_t)15;
            memcpy(&arena[o], &src[i * P], L);
            memset(&arena[o + L], 0, 16);
            used = o + L;
            OpRec op{};
            op.off = (uint32_t)o;
            op.size = L;
            ops[(i / 12) % 64].push_back(op);
        }
        auto t1 = std::chrono::steady_clock::now();
        printf("bare copy + op record:  %.1f ns/datagram (%.2f GB/s)\n",
               std::chrono::duration<double, std::nano>(t1 - t0).count() / N,
               N * L / std::chrono::duration<double>(t1 - t0).count() / 1e9);
    }
    qfec_zfec_free(z);
    return 0;
}
