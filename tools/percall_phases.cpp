// Where the unchanged drop-in's per-call time goes (fec_encode / fec_decode on host packets,
// RS(10,3), sz 1028 -- the bench's per_call shape), timed from C++ so no ctypes cost is in it:
//   the HIP queries the call path makes (hipGetDeviceCount + hipGetDevice, and
//   hipPointerGetAttributes on a pageable pointer, which is how a host packet is told from a
//   device one), a 10 KiB memcpy into host-mapped device memory (the server's input rows), and
//   whole fec_encode / fec_decode calls under each qfec_tune per-call setting.
//   hipcc -O2 -o tools/_build/percall_phases tools/percall_phases.cpp -Lquicknet_amd -lqfec \
//         -Wl,-rpath,'$ORIGIN/../../quicknet_amd'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <vector>

#include "../include/qfec.h"
#include "../include/qfec_fec.h"

static double median_us(const std::function<void()>& f, int reps = 4000) {
    for (int i = 0; i < 200; ++i) f();
    std::vector<double> t(reps);
    for (int i = 0; i < reps; ++i) {
        const auto a = std::chrono::steady_clock::now();
        f();
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    std::sort(t.begin(), t.end());
    return t[reps / 2];
}

int main() {
    const int k = 10, n = 13, sz = 1028;
    std::vector<std::vector<unsigned char>> data(n, std::vector<unsigned char>(sz));
    for (int r = 0; r < n; ++r)
        for (int b = 0; b < sz; ++b) data[r][b] = (unsigned char)(r * 131 + b * 7 + 1);
    void* h = fec_new(k, n);
    for (int j = k; j < n; ++j) {
        unsigned char* src[16];
        for (int i = 0; i < k; ++i) src[i] = data[i].data();
        fec_encode(h, src, data[j].data(), j, sz);
    }
    int dev = 0, cnt = 0;
    printf("hipGetDeviceCount + hipGetDevice        %6.2f us\n", median_us([&] {
               (void)hipGetDeviceCount(&cnt);
               (void)hipGetDevice(&dev);
           }));
    std::vector<unsigned char> pageable(4096);
    printf("hipPointerGetAttributes (pageable)      %6.2f us\n", median_us([&] {
               hipPointerAttribute_t a;
               if (hipPointerGetAttributes(&a, pageable.data()) != hipSuccess) (void)hipGetLastError();
           }));
    unsigned char* fg = nullptr;
    if (hipExtMallocWithFlags((void**)&fg, 16 * 1040, hipDeviceMallocFinegrained) == hipSuccess) {
        std::vector<unsigned char> src(10 * 1040, 7);
        printf("memcpy 10 x 1028 B into device memory   %6.2f us\n", median_us([&] {
                   for (int r = 0; r < k; ++r) memcpy(fg + r * 1040, src.data() + r * 1040, sz);
                   __builtin_ia32_sfence();
               }));
        (void)hipFree(fg);
    }
    const int lost[3] = {3, 6, 9};
    std::vector<int> idx_t;
    for (int r = 0; r < n && (int)idx_t.size() < k; ++r)
        if (r != lost[0] && r != lost[1] && r != lost[2]) idx_t.push_back(r);
    std::vector<unsigned char> out(sz);
    // the resident server, and one launch per call (the spin / wait choice of the one-launch path
    // is automatic since round 5: spin for launches of at most 256 chunks)
    const char* settings[][2] = {{"percall_resident", "1"}, {"percall_resident", "0"}};
    for (auto& st : settings) {
        qfec_tune(st[0], atoi(st[1]));
        const double enc = median_us([&] {
            unsigned char* src[16];
            for (int i = 0; i < k; ++i) src[i] = data[i].data();
            fec_encode(h, src, out.data(), k, sz);
        });
        if (memcmp(out.data(), data[k].data(), sz)) printf("fec_encode output WRONG\n");
        std::vector<std::vector<unsigned char>> bufs(k, std::vector<unsigned char>(sz));
        bool ok = true;
        const double decu = median_us([&] {
            unsigned char* pk[16];
            int ix[16];
            for (int i = 0; i < k; ++i) {
                pk[i] = idx_t[i] < k ? data[idx_t[i]].data() : bufs[i].data();
                if (idx_t[i] >= k) memcpy(bufs[i].data(), data[idx_t[i]].data(), sz);
                ix[i] = idx_t[i];
            }
            if (fec_decode(h, pk, ix, sz)) ok = false;
        });
        // check once: the recovered rows are the lost data rows
        unsigned char* pk[16];
        int ix[16];
        for (int i = 0; i < k; ++i) {
            memcpy(bufs[i].data(), data[idx_t[i]].data(), sz);
            pk[i] = bufs[i].data();
            ix[i] = idx_t[i];
        }
        if (fec_decode(h, pk, ix, sz)) ok = false;
        for (int i = 0; i < k; ++i)
            if (memcmp(pk[i], data[i].data(), sz)) ok = false;
        printf("%-16s=%s fec_encode %6.2f us   fec_decode %6.2f us (incl. %d-B parity re-copy)  %s\n", st[0],
               st[1], enc, decu, 3 * sz, ok ? "ok" : "WRONG");
    }
    qfec_tune("percall_resident", 1);
    unsigned long long s[5];
    qfec_percall_stats(s);
    printf("server: calls %llu launches %llu relaunches %llu\n", s[0], s[1], s[2]);
    fec_free(h);
    return 0;
}
