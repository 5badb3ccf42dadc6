// tools/bar_probe.hip -- per-call staging choices for fec_encode-sized work (measurement only):
// one call = host memcpy of k = 10 rows of 1040 B into the staging, one one-block launch that
// reads them and writes 3 rows into mapped pinned host memory, a spin on the completion word.
//   pinned   rows staged in mapped pinned host memory; the kernel reads them over PCIe (batched)
//   bar      rows written by the CPU straight into fine-grained DEVICE memory through its host
//            mapping (PCIe posted writes); the kernel reads HBM
//   devcopy  rows staged in pinned memory, hipMemcpyAsync H2D, then the kernel (device rows)
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/bar_probe tools/bar_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int K = 10, CH = 65, PITCH = CH * 16;

__global__ void k_rows(const uint8_t* in, uint8_t* out, uint32_t* done, uint32_t seq) {
    const int c = threadIdx.x;
    if (c < CH) {
        uint4 x[K];
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = reinterpret_cast<const uint4*>(in + (size_t)i * PITCH)[c];
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < K; ++i) { acc.x ^= x[i].x; acc.y ^= x[i].y; acc.z ^= x[i].z; acc.w ^= x[i].w; }
        for (int j = 0; j < 3; ++j) reinterpret_cast<uint4*>(out + (size_t)j * PITCH)[c] = acc;
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static void spin(volatile uint32_t* w, uint32_t seq) {
    while (__atomic_load_n(w, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
}

int main() {
    const int N = 4000;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *hw, *dw;
    CK(hipHostMalloc((void**)&hw, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&dw, hw, 0));
    *hw = 0;
    uint8_t *hp, *dp, *ho, *dout, *dd, *fg;
    CK(hipHostMalloc((void**)&hp, 1 << 16, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void**)&dp, hp, 0));
    CK(hipHostMalloc((void**)&ho, 1 << 16, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void**)&dout, ho, 0));
    CK(hipMalloc((void**)&dd, 1 << 16));
    CK(hipExtMallocWithFlags((void**)&fg, 1 << 16, hipDeviceMallocFinegrained));
    hipPointerAttribute_t at;
    CK(hipPointerGetAttributes(&at, fg));
    printf("fine-grained device block: device %p host %p type %d\n", at.devicePointer, at.hostPointer, (int)at.type);
    uint8_t* src = new uint8_t[K * PITCH];
    for (int i = 0; i < K * PITCH; ++i) src[i] = (uint8_t)(i * 7 + 1);
    uint8_t* fgh = (uint8_t*)at.hostPointer;
    uint32_t seq = 0;
    for (int rep = 0; rep < 3; ++rep) {
        double t0 = now_us();
        for (int i = 0; i < N; ++i) {
            ++seq;
            memcpy(hp, src, K * PITCH);
            hipLaunchKernelGGL(k_rows, dim3(1), dim3(128), 0, s, dp, dout, dw, seq);
            spin(hw, seq);
        }
        const double t_pin = (now_us() - t0) / N;
        t0 = now_us();
        for (int i = 0; i < N; ++i) {
            ++seq;
            memcpy(hp, src, K * PITCH);
            CK(hipMemcpyAsync(dd, hp, K * PITCH, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_rows, dim3(1), dim3(128), 0, s, dd, dout, dw, seq);
            spin(hw, seq);
        }
        const double t_dc = (now_us() - t0) / N;
        double t_bar = -1;
        if (fgh) {
            t0 = now_us();
            for (int i = 0; i < N; ++i) {
                ++seq;
                memcpy(fgh, src, K * PITCH);
                __builtin_ia32_sfence();
                hipLaunchKernelGGL(k_rows, dim3(1), dim3(128), 0, s, fg, dout, dw, seq);
                spin(hw, seq);
            }
            t_bar = (now_us() - t0) / N;
        }
        // classification of a pageable pointer (what is_device_ptr costs per call)
        t0 = now_us();
        int ndev = 0;
        for (int i = 0; i < N; ++i) {
            hipPointerAttribute_t a2;
            if (hipPointerGetAttributes(&a2, src + (i & 7)) == hipSuccess && a2.type == hipMemoryTypeDevice) ++ndev;
            else (void)hipGetLastError();
        }
        const double t_attr = (now_us() - t0) / N;
        printf("rep %d: hipPointerGetAttributes on a pageable pointer %.3f us (%d device)\n", rep, t_attr, ndev);
        CK(hipStreamSynchronize(s));
        // check the last bar call's output: XOR of the 10 rows
        bool ok = true;
        for (int b = 0; b < PITCH && fgh; ++b) {
            uint8_t x = 0;
            for (int i = 0; i < K; ++i) x ^= src[i * PITCH + b];
            ok = ok && ho[b] == x;
        }
        printf("rep %d: pinned %.2f us | devcopy %.2f us | bar %.2f us (output %s)\n", rep, t_pin, t_dc, t_bar,
               fgh ? (ok ? "ok" : "WRONG") : "n/a");
    }
    return 0;
}
