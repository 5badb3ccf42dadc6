// Cost of a pointer-kind probe (the per-call ABIs ask whether each packet pointer is device
// memory): hipPointerGetAttributes, hipPointerGetAttribute(MEMORY_TYPE), hsa_amd_pointer_info,
// on plain malloc, hipHostMalloc and hipMalloc pointers.
//   hipcc -O2 -o /tmp/ptr_probe tools/ptr_probe.cpp -lhsa-runtime64 && /tmp/ptr_probe
#include <hip/hip_runtime.h>
#include <hsa/hsa_ext_amd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

template <class F>
static double ns_per(F f, int n = 200000) {
    for (int i = 0; i < 1000; ++i) f();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) f();
    return std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / n;
}

int main() {
    void* hm = malloc(4096);
    void* hp = nullptr;
    void* dv = nullptr;
    if (hipHostMalloc(&hp, 4096, 0) != hipSuccess || hipMalloc(&dv, 4096) != hipSuccess) return 1;
    const char* names[3] = {"malloc", "hipHostMalloc", "hipMalloc"};
    void* ps[3] = {hm, hp, dv};
    for (int i = 0; i < 3; ++i) {
        void* p = ps[i];
        const double a = ns_per([&] {
            hipPointerAttribute_t at;
            if (hipPointerGetAttributes(&at, p) != hipSuccess) (void)hipGetLastError();
        });
        const double b = ns_per([&] {
            unsigned int t = 0;
            if (hipPointerGetAttribute(&t, HIP_POINTER_ATTRIBUTE_MEMORY_TYPE, (hipDeviceptr_t)p) != hipSuccess)
                (void)hipGetLastError();
        });
        const double c = ns_per([&] {
            hsa_amd_pointer_info_t info;
            info.size = sizeof(info);
            (void)hsa_amd_pointer_info(p, &info, nullptr, nullptr, nullptr);
        });
        const double d = ns_per([&] {
            int dev = 0;
            (void)hipGetDevice(&dev);
        });
        printf("%-14s hipPointerGetAttributes %6.1f ns  hipPointerGetAttribute %6.1f ns  hsa_amd_pointer_info %6.1f ns  (hipGetDevice %5.1f ns)\n",
               names[i], a, b, c, d);
    }
    return 0;
}
