// qfec_internal.hpp -- shared declarations of libqfec (host runtime <-> kernels).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <vector>

namespace qfec {

// dwords per coefficient in a perm table:
//   [0..4] v_perm_b32 tables (c*{0..7}, c*{0..7}<<3, c*{0..3}<<6, packed 4 bytes/dword)
//   [5]    row flag on column 0: 1 = row starts from the output's previous bytes
//   [6]    log(c) (0xFF for c == 0), for the LDS log/exp variant
//   [7]    c itself
constexpr int QFEC_TAB_STRIDE = 8;

constexpr int QFEC_REC_NONE = -1;  // LUT: nothing erased in this group
constexpr int QFEC_REC_FAIL = -2;  // LUT: more erased data than surviving parity
constexpr int QFEC_LUT_MAX_N = 24; // n <= 24 -> 2^n-entry pattern LUT on the device

constexpr int QFEC_VARIANT_PERM_I = 0;
constexpr int QFEC_VARIANT_LDSLOG_I = 1;

// n / d for n < 2^32 via a 33-bit magic (Granlund-Montgomery, round-up form)
struct DivMagic {
    uint64_t mul;
    uint32_t shift;
    uint32_t pow2;
};

DivMagic make_div_magic(uint32_t d);

struct EncodeArgs {
    const uint8_t* data;    // [groups][k][pitch]
    uint8_t* parity;        // [groups][m][pitch]
    const uint32_t* tab;    // [m][k][QFEC_TAB_STRIDE]
    const uint8_t* gf_exp;  // LDS variant: exp[512]
    const uint8_t* gf_log;  // LDS variant: log[256]
    uint64_t work;          // groups * cols lanes (< 2^32)
    uint64_t pitch;         // bytes between rows of a group
    uint64_t dgs, pgs;      // bytes between groups: data (k*pitch when packed), parity (m*pitch)
    DivMagic cols_div;
    uint32_t cols;          // columns per row: 16-B columns (vec16) or bytes
    int k, m;
    int vec16;
    int impl;               // tuning "encode_impl"
    int lds;                // dynamic LDS bytes per block, a residency cap: -1 auto, 0 none (tuning "encode_lds")
    int block;              // threads per block: -1 auto, 64, 256 (tuning "encode_block")
};

struct ReconArgs {
    uint8_t* data;            // [groups][k][pitch]
    const uint8_t* parity;    // [groups][m][pitch]
    const uint8_t* marks;     // rs.c layout, or NULL when group_rec is given
    const int32_t* lut;       // [2^n] pattern -> record offset (dwords) / QFEC_REC_*
    const int32_t* group_rec; // explicit mode: per-group record offset / QFEC_REC_*
    const uint32_t* records;
    unsigned int* failed;
    uint64_t groups;
    uint64_t pitch;
    uint64_t dgs, pgs;        // bytes between groups: data rows, parity rows
    uint32_t cols;            // 16-B columns (vec16) or bytes per row
    int k, m;
    int surv_off, lost_off, hdr;
    int coff;                 // record word of the coefficient-table byte offsets (RecordLayout::coff)
    const uint32_t* t256;     // [256][QFEC_TAB_STRIDE] perm tables of every coefficient value (compact mode)
    int vec16;
    int impl;                 // tuning "recon_impl": -1 auto, exact-e rows on 2 16-B lanes, 3 8-B lanes,
                              // 4 12-B lanes, 8 8-B lanes with one group per block
    uint32_t wpg;             // waves per group = ceil(cols / 64) (vec16 LUT kernels)
    uint32_t cols8, wpg8;     // the same at 8-B columns: ceil(B / 8), ceil(cols8 / 64)
    uint32_t cols12, wpg12;   // the same at 12-B columns (recon_impl 4)
    int rlds;                 // reconstruct skeleton probe: LDS bytes per block, a residency cap (0 none)
};

// FEC datagram batches (qfec_wire.hip): shards[G][n][pitch], wire[G][n][wire_pitch]
struct WireArgs {
    const uint8_t* payload;   // send: concatenated payloads (16 readable bytes past the last)
    const int64_t* offsets;   // send: [G*k] payload offsets
    const int32_t* sizes;     // send: [G*k] payload sizes
    const uint32_t* seq;      // send: [G][2] sent / src index of the group's first packet
    uint8_t* shards;
    uint64_t group_stride;    // n * pitch
    uint64_t pitch;
    uint8_t* wire;
    uint64_t wire_pitch;
    int32_t* wire_len;        // [G*n] datagram lengths (receive: 0 = not received)
    uint8_t* marks;           // receive: rs.c-layout erasure marks
    int32_t* rx_size;         // receive: [G*n] shard size or -1 (may be NULL)
    int32_t* status;          // receive: [G*k] payload offset (2|4), -1 dropped, -2 lost
    int32_t* psize;           // receive: [G*k] payload size field
    uint64_t groups;
    int k, m;
    int checksum;
    int dec_pkt_size;
    int store_nt;             // fused send: bit 0 body, bit 1 head use non-temporal stores
};

hipError_t launch_build_shards(const WireArgs& a, hipStream_t s);
// fused send path for templated (k, m); *launched = false when the shape has no instance
// `part` = scratch of (lpg / 16) * ((n + 1) / 2) u32 per group, lpg ~ (pitch + 13) / 16
hipError_t launch_pack_fused(const WireArgs& a, const uint32_t* tab, uint32_t* part, hipStream_t s, bool* launched);
struct FrameArgs {
    const uint8_t* in;        // [rows][in_pitch]
    const int32_t* in_len;    // [rows]
    uint8_t* out;             // [rows][out_pitch]
    int32_t* out_len;         // [rows] (frame: framed length, -1 if it does not fit)
    const uint8_t* mask;      // frame: [rows] raw mask byte (Session::PacketOutput's _mask++)
    uint32_t* conv_hid;       // [rows][2] Session prefix (frame: in, unframe: out); may be NULL
    int32_t* status;          // unframe: [rows]
    uint8_t* info;            // unframe: [rows][4] mask, check, cmd & 0x1f, protocol; may be NULL
    uint64_t rows, in_pitch, out_pitch;
    uint32_t gmask, cmd, protocol;
    int session;              // 1: the 8-byte conv/hid prefix is part of the frame
};
hipError_t launch_frame_udp(const FrameArgs& a, hipStream_t s);
// ProtocolUdp framing inside the datagram kernels (qfec_pack_frames / qfec_unpack_frames)
struct FrameSend {
    const uint8_t* mask;       // [G*n] raw mask bytes (Session::PacketOutput's _mask++)
    const uint32_t* conv_hid;  // [G*n][2] Session prefix, or NULL (4-byte prefix)
    uint32_t gmask, cmd, protocol;
};
struct FrameRecv {
    uint32_t gmask;
    int32_t* status;           // [G*n] RecvPacket verdict (0 ok, 1 short, 2 checksum, 3 cmd, 4 too long); nullable
    uint32_t* conv_hid;        // [G*n][2] Session prefix out (session frames only); nullable
};
hipError_t launch_pack_frames(const WireArgs& a, const FrameSend& fs, int fp, const uint32_t* tab, hipStream_t s,
                              bool* launched);
hipError_t launch_unpack_frames(const WireArgs& a, const FrameRecv& fr, int fp, const int32_t* lut,
                                const uint32_t* records, uint32_t rec_hdr, hipStream_t s, bool* launched);
hipError_t launch_len_by_status(int32_t* len, const int32_t* status, uint64_t rows, hipStream_t s);
hipError_t launch_gather_rows(const uint8_t* base, const uint64_t* off, const int32_t* len, uint64_t rows, int wrap_n,
                              int wrap_k, uint8_t* out, uint64_t out_pitch, int32_t* out_len, hipStream_t s);
// the datagram receive k_rx (qfec_rx.hip) for templated (k, m); *launched = false when the shape has no instance
hipError_t launch_rx(const WireArgs& a, const int32_t* lut, const uint32_t* records, uint32_t rec_hdr, hipStream_t s,
                     bool* launched);
hipError_t launch_unframe_udp(const FrameArgs& a, hipStream_t s);
hipError_t launch_emit_wire(const WireArgs& a, hipStream_t s);
hipError_t launch_parse_wire(const WireArgs& a, hipStream_t s);
hipError_t launch_check_payloads(const WireArgs& a, hipStream_t s);

// runtime tuning knobs (qfec_tune); defaults are the measured best.  Atomic: qfec_tune may
// write a knob while launches on other threads read it (each read is one atomic load)
struct Tuning {
    std::atomic<int> recon_impl{-1};  // -1 auto (per shape); 2, 3, 4: exact-e rows on 16-, 8-, 12-B lanes; 8: 3 one group per block
    std::atomic<int> encode_impl{-1};   // -1 auto (inputs in halves for k >= 16), 0 all rows, 2 halves
    std::atomic<int> wire_fused{1};     // fused datagram send where a (k, m) instance exists (0: staged)
    std::atomic<int> wire_rx{1};        // datagram receive: 1 fused k_rx, lanes and LDS staging by pitch; 2 / 3 16-B lanes
                                        // with / without LDS staging, 4 / 5 8-B lanes likewise; 0 staged (3 launches)
    std::atomic<int> host_chunk{0};     // host-buffer paths: groups per pipelined chunk (0: by bytes)
    std::atomic<int> host_threads{0};   // host copy threads for module/rs.h on host pointers (0: usable CPUs, <= 32)
    std::atomic<int> host_zero_copy{1}; // pinned host batches: kernels read/write them directly (0: staged copies)
    std::atomic<int> host_lanes{4};     // module/rs.h on host pointers: chunk slots in flight on the device (2..8)
    std::atomic<int> host_nt{2};        // module/rs.h on host pointers: streaming stores into the slots (0 / 1 / 2 sequential rows)
    std::atomic<int> encode_block{-1};  // threads per encode block: -1 auto (64 for k = 10 all-rows), 64, 256
    std::atomic<int> encode_lds{-1};    // LDS bytes per encode block, capping waves per CU (-1 auto, 0 none)
};
Tuning& tuning();

hipError_t launch_encode(const EncodeArgs& a, int variant, hipStream_t stream);
hipError_t launch_reconstruct(const ReconArgs& a, hipStream_t stream);
hipError_t launch_synth_fill(uint8_t* p, uint64_t nbytes, uint64_t seed, hipStream_t stream);
hipError_t launch_probe_xor(const EncodeArgs& a, hipStream_t stream);
hipError_t launch_probe_recon(const ReconArgs& a, hipStream_t stream);

// ---------------------------------------------------------------- host GF(2^8) (gf256.cpp)
struct Field {
    uint8_t exp[512];  // exp[i] = 2^i, doubled (exp[i + 255] = exp[i]) + 2 pad
    uint8_t log[256];  // log[0] = 255 sentinel
    uint8_t inv[256];  // inv[0] = 0
    uint8_t mul[256][256];
};

const Field& field();

// parity rows (m x k, row-major) of the two reference matrix flavours
bool cauchy_rows(int k, int m, std::vector<uint8_t>& out);       // module/rs.c:437-440
bool vandermonde_rows(int k, int m, std::vector<uint8_t>& out);  // module/fec.c:653-707

// in-place GF inverse of a k x k matrix; false if singular
bool gf_invert(uint8_t* a, int k);
// the same with module/rs.c invert_mat's pivot order: on a singular matrix it returns false
// and leaves `a` in the partially eliminated state rs.c then decodes with (rs.c:556)
bool gf_invert_rs(uint8_t* a, int k);

// one coefficient's 8-dword perm table
void perm_entry(uint8_t c, uint32_t* out8);

// decode record of one erasure pattern (see qfec_kernels.hip, "reconstruct").
// group-order marks over n = k + m shards.  Returns e (>= 1), 0 if nothing is erased
// or -1 if under-determined; on e >= 1 fills rows (e x k), survivors (k), lost (e).
// `full` (n x k, nullable): module/rs.c's rs->m -- the sub-matrix is taken from it, data rows
// included, and inverted with rs.c's semantics (a singular one decodes with its partial state)
int decode_rows(const uint8_t* parity_rows, int k, int m, const uint8_t* marks_n,
                std::vector<uint8_t>& rows, std::vector<int>& survivors, std::vector<int>& lost,
                const uint8_t* full = nullptr);

// Record: [0] e, [1] rs.c quirk flags (bit j: row j's column-0 coefficient is zero),
// [surv_off + c] survivor shard id, [lost_off + j] erased data row,
// [coff + j*k + c] byte offset of coefficient (j, c)'s perm table in the 256-entry table
// (value * 32), then from [hdr] the tables themselves
// ([j][c][QFEC_TAB_STRIDE]).  A kernel that reads the offsets touches only the record's
// first (coff + m*k) words, so the records of every pattern stay cache-resident.
struct RecordLayout {
    int surv_off, lost_off, coff, hdr;
    size_t words(int e, int k) const { return (size_t)hdr + (size_t)e * k * QFEC_TAB_STRIDE; }
};
RecordLayout record_layout(int k, int m);
void build_record(const RecordLayout& L, int k, int e, const uint8_t* rows, const int* survivors,
                  const int* lost, bool rs_quirk, uint32_t* out);

}  // namespace qfec
