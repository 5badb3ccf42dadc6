// qfec_percall.hpp -- the per-packet ABI's (fec_encode / fec_decode, system/fec.h) low-latency
// kernel: one launch, no DMA copies.  The caller's packets are staged by the CPU into pinned,
// device-mapped host memory; the kernel reads them over PCIe, multiplies by the decode/encode
// rows (perm tables passed BY VALUE in the kernel arguments), and writes the outputs back into
// pinned memory.  Used when e * k <= kPcMaxCoef.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qfec {

constexpr int kPcMaxCoef = 160;  // e * k coefficients: 5 dwords each in the kernarg (3.2 KB)

struct PcArgs {
    const uint8_t* in;   // k rows of `pitch` bytes (pinned host, device-mapped)
    uint8_t* out;        // e rows of `pitch` bytes (pinned host, device-mapped)
    uint32_t pitch;      // multiple of 16
    uint32_t chunks;     // 16-B chunks per row to compute
    uint32_t k, e;
    // completion word in coherent pinned host memory (nullable): a one-block launch stores
    // `seq` into it after all of its output is visible to the host, so the caller can spin
    // on that word instead of waiting for the runtime's completion signal
    uint32_t* done;
    uint32_t seq;
    uint32_t tab[kPcMaxCoef * 5];  // [e][k] perm tables (5 dwords: QFEC_TAB_STRIDE's first 5)
};

hipError_t launch_percall(const PcArgs& a, hipStream_t s);

}  // namespace qfec
