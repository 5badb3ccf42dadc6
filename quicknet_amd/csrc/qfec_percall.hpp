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

// ---- the resident per-call server (tuning "percall_resident" 1, the default where the device
// memory below is host-mapped).  A launch costs ~6 us and reading the packets across PCIe
// from pinned host memory another ~3-7 us (profiles/r02zk_launch_lat.txt,
// profiles/r03k_doorbell_probe.txt), so instead one block stays resident on the device between
// calls: the CPU writes the input packets, the coefficient tables and the request number into
// device memory it can map (fine-grained, host-visible), the block -- polling that word in its
// own memory, not across PCIe -- computes the outputs into pinned host memory and stores the
// request number into a completion word there, and the CPU spins on it.  Only posted writes
// cross PCIe.  The block exits by itself after `idle_ticks` without a request (or at once
// when `stop` is set), so no grid outlives an idle caller, and the host relaunches it when
// the next request finds it gone.
constexpr int kPcMaxChunks = 256;             // 16-B columns per packet row (4 KiB)
constexpr uint32_t kPcIdleUsDefault = 1000;   // qfec_tune "percall_idle_us": 1 ms (the wall clock ticks at 100 MHz)
constexpr int kPcSrvMaxCoef = 64;             // the server serves k <= 16 and k * e <= 64 (lane c: coefficient c)
constexpr int kPcTabWords = 8 * kPcSrvMaxCoef; // coefficient c's 5 table dwords at 8 c
struct PcBell {                               // fine-grained device memory, written by the CPU
    // the request word: number (low 32 bits, 0: none yet) | k << 32 | e << 40 | (chunks - 1) << 48,
    // stored as one 8-byte write, so the block learns the shape with the request (one round trip)
    uint64_t bell;
    uint32_t stop;                            // 1: exit now
    uint32_t pad[13];
    uint32_t tab[kPcTabWords];                // [e][k] perm tables, 8 dwords apart (5 used)
};
__host__ __device__ constexpr uint64_t pc_bell(uint32_t req, uint32_t k, uint32_t e, uint32_t chunks) {
    return (uint64_t)req | ((uint64_t)k << 32) | ((uint64_t)e << 40) | ((uint64_t)(chunks - 1) << 48);
}
struct PcStatus {                             // coherent pinned host memory, written by the block
    uint32_t done;                            // the last request served
    uint32_t state;                           // (launch generation << 1) | running
    uint64_t rt;                              // QFEC_PERCALL_TRACE: wall-clock ticks (100 MHz) over ts[0..3]
    uint32_t pad[4];
    // QFEC_PERCALL_TRACE=1: shader-clock stamps (s_memtime) of the last request -- seen, inputs
    // and tables in registers, outputs issued, system fence done
    uint64_t ts[4];
};
hipError_t launch_percall_server(PcBell* bell, const uint8_t* in, uint8_t* out, PcStatus* st, uint32_t served,
                                 uint32_t gen, uint32_t flags, uint64_t idle_ticks, hipStream_t s);

}  // namespace qfec
