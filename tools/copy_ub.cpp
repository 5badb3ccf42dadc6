// tools/copy_ub.cpp -- measurement aid: one core copying 153 600 datagrams of 1 041 B from a
// contiguous source into a 16-B aligned arena (the qfec_zfec_unpack_input pattern), with glibc
// memcpy, `rep movsb` and an AVX2 32-B loop; destination in ordinary or 2 MiB pages.
#include <immintrin.h>
#include <string.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

static void copy_movsb(void* d, const void* s, size_t n) {
    asm volatile("rep movsb" : "+D"(d), "+S"(s), "+c"(n) : : "memory");
}
__attribute__((target("avx2"))) static void copy_avx2(uint8_t* d, const uint8_t* s, size_t n) {
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256((const __m256i*)(s + i));
        const __m256i b = _mm256_loadu_si256((const __m256i*)(s + i + 32));
        const __m256i c = _mm256_loadu_si256((const __m256i*)(s + i + 64));
        const __m256i e = _mm256_loadu_si256((const __m256i*)(s + i + 96));
        _mm256_storeu_si256((__m256i*)(d + i), a);
        _mm256_storeu_si256((__m256i*)(d + i + 32), b);
        _mm256_storeu_si256((__m256i*)(d + i + 64), c);
        _mm256_storeu_si256((__m256i*)(d + i + 96), e);
    }
    for (; i + 32 <= n; i += 32) _mm256_storeu_si256((__m256i*)(d + i), _mm256_loadu_si256((const __m256i*)(s + i)));
    if (i < n) memcpy(d + i, s + i, n - i);
}

int main() {
    const size_t N = 153600, L = 1041, P = 1041;
    std::vector<uint8_t> src(N * P + 64);
    for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 131);
    const size_t A = N * 1056 + (4u << 20);
    uint8_t* plain = (uint8_t*)aligned_alloc(4096, A);
    uint8_t* huge = (uint8_t*)mmap(nullptr, A, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    madvise(huge, A, MADV_HUGEPAGE);
    memset(plain, 0, A);
    memset(huge, 0, A);
    const char* names[3] = {"memcpy", "rep movsb", "avx2 loop"};
    for (int dst = 0; dst < 2; ++dst)
        for (int v = 0; v < 3; ++v) {
            uint8_t* arena = dst ? huge : plain;
            double best = 1e9;
            for (int rep = 0; rep < 5; ++rep) {
                auto t0 = std::chrono::steady_clock::now();
                size_t used = 0;
                for (size_t i = 0; i < N; ++i) {
                    const size_t o = (used + 15) & ~(size_t)15;
                    if (v == 0) memcpy(arena + o, &src[i * P], L);
                    else if (v == 1) copy_movsb(arena + o, &src[i * P], L);
                    else copy_avx2(arena + o, &src[i * P], L);
                    memset(arena + o + L, 0, 16);
                    used = o + L;
                }
                best = std::min(best, std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count());
            }
            printf("%-10s into %s pages: %.1f ns/datagram (%.2f GB/s)\n", names[v], dst ? "2 MiB" : "4 KiB", best / N,
                   N * L / best);
        }
    return 0;
}
