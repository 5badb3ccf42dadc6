// qfec_wire_api.cpp -- the datagram and framing entry points of include/qfec.h (qfec_pack_datagrams,
// qfec_unpack_datagrams, qfec_pack_frames, qfec_unpack_frames, qfec_frame_udp, qfec_unframe_udp,
// qfec_gather_rows): argument checks and launches of the kernels in qfec_wire.hip / qfec_rx.hip.
#include "qfec_rt.hpp"

using namespace qfec;

// ====================================================================== FEC datagram batches
namespace {

int wire_check(const qfec_code* c, long long groups, int checksum, long long pitch, long long wire_pitch,
               const void* shards, const void* wire) {
    if (!c || groups < 0 || (checksum != 0 && checksum != 1)) return QFEC_EINVAL;
    if (c->k + c->m > 15 || c->k < 1) {
        set_error("FEC datagrams carry 4-bit n and k (network/FecCodecBuf.cpp:290-299): n = %d > 15", c->k + c->m);
        return QFEC_EUNSUP;
    }
    if (pitch < 16 || pitch % 16 || wire_pitch % 16 || wire_pitch < (long long)round_up((size_t)pitch + 13, 16) ||
        ((uintptr_t)shards | (uintptr_t)wire) % 16) {
        set_error("datagram batch: shard pitch and wire pitch must be multiples of 16, wire >= shard + 13, 16-B aligned");
        return QFEC_EINVAL;
    }
    return QFEC_OK;
}

// frame rows: a 16-B multiple pitch that holds prefix + 13 + shard pitch
int frame_check(const qfec_code* c, long long groups, int checksum, long long pitch, long long frame_pitch, int fp,
                const void* shards, const void* frames) {
    const int rc = wire_check(c, groups, checksum, pitch, (long long)round_up((size_t)pitch + 13, 16), shards, frames);
    if (rc) return rc;
    if (frame_pitch % 16 || frame_pitch < pitch + 13 + fp) {
        set_error("frames: frame pitch must be a multiple of 16 and >= prefix (%d) + 13 + shard pitch", fp);
        return QFEC_EINVAL;
    }
    return QFEC_OK;
}

}  // namespace

extern "C" {

int qfec_pack_datagrams(qfec_code* code, const unsigned char* d_payload, const long long* d_offsets,
                        const int* d_sizes, const unsigned int* d_seq, long long groups, int checksum,
                        unsigned char* d_shards, long long shard_pitch, unsigned char* d_wire, long long wire_pitch,
                        int* d_wire_len, void* stream) {
    int rc = wire_check(code, groups, checksum, shard_pitch, wire_pitch, d_shards, d_wire);
    if (rc) return rc;
    if (groups == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    if ((rc = current_ctx(&ctx))) return rc;
    uint32_t* tab = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_enc(code, ctx->device, &tab);
    }
    if (rc) return rc;
    const int k = code->k, m = code->m, n = k + m;
    hipStream_t s = (hipStream_t)stream;
    WireArgs a{};
    a.payload = d_payload;
    a.offsets = (const int64_t*)d_offsets;
    a.sizes = d_sizes;
    a.seq = d_seq;
    a.shards = d_shards;
    a.pitch = (uint64_t)shard_pitch;
    a.group_stride = (uint64_t)n * shard_pitch;
    a.wire = d_wire;
    a.wire_pitch = (uint64_t)wire_pitch;
    a.wire_len = d_wire_len;
    a.groups = (uint64_t)groups;
    a.k = k;
    a.m = m;
    a.checksum = checksum;
    a.store_nt = 3;  // non-temporal datagram stores, body and head
    if (tuning().wire_fused) {
        bool launched = false;
        // the fused path never materialises shards; their buffer holds its partial sums
        // ((wire_pitch + 63) / 256 + 2) * 8 u32 per group  <<  n * pitch bytes
        hipError_t e = launch_pack_fused(a, tab, reinterpret_cast<uint32_t*>(d_shards), s, &launched);
        if (e != hipSuccess) return hip_fail(e, "pack_fused launch");
        if (launched) return QFEC_OK;
    }
    hipError_t e = launch_build_shards(a, s);
    if (e != hipSuccess) return hip_fail(e, "build_shards launch");
    // check shards: fec_encode(.., groupMax) over the k data shards (FecCodecBuf.cpp:151);
    // bytes past a group's groupMax are zero in every data shard, hence in the parity.
    if (m > 0 && (rc = run_encode(*ctx, code, tab, m, d_shards, d_shards + (size_t)k * shard_pitch, groups,
                                  (int)shard_pitch, shard_pitch, s, (long long)a.group_stride, (long long)a.group_stride)))
        return rc;
    e = launch_emit_wire(a, s);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "emit_wire launch");
}

int qfec_unpack_datagrams(qfec_code* code, const unsigned char* d_wire, long long wire_pitch, const int* d_wire_len,
                          long long groups, int checksum, int dec_pkt_size, unsigned char* d_shards,
                          long long shard_pitch, unsigned char* d_marks, int* d_rx_size, int* d_status, int* d_psize,
                          void* stream) {
    int rc = wire_check(code, groups, checksum, shard_pitch, wire_pitch, d_shards, d_wire);
    if (rc) return rc;
    if (groups == 0) return QFEC_OK;
    if (!d_marks || !d_status || !d_psize || !d_wire_len) return QFEC_EINVAL;
    DevCtx* ctx = nullptr;
    if ((rc = current_ctx(&ctx))) return rc;
    DevTables* d = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_lut(code, ctx->device, &d);
    }
    if (rc) return rc;
    const int k = code->k, m = code->m, n = k + m;
    hipStream_t s = (hipStream_t)stream;
    WireArgs a{};
    a.shards = d_shards;
    a.pitch = (uint64_t)shard_pitch;
    a.group_stride = (uint64_t)n * shard_pitch;
    a.wire = const_cast<uint8_t*>(d_wire);
    a.wire_pitch = (uint64_t)wire_pitch;
    a.wire_len = const_cast<int32_t*>(d_wire_len);
    a.marks = d_marks;
    a.rx_size = d_rx_size;
    a.status = d_status;
    a.psize = d_psize;
    a.groups = (uint64_t)groups;
    a.k = k;
    a.m = m;
    a.checksum = checksum;
    a.dec_pkt_size = dec_pkt_size;
    if (tuning().wire_rx && d->d_lut) {
        bool launched = false;
        const hipError_t ef =
            launch_rx(a, d->d_lut, d->d_rec, (uint32_t)record_layout(k, m).hdr, s, &launched);
        if (ef != hipSuccess) return hip_fail(ef, "datagram receive launch");
        if (launched) return QFEC_OK;
    }
    hipError_t e = launch_parse_wire(a, s);
    if (e != hipSuccess) return hip_fail(e, "parse_wire launch");
    // decode the missing data shards from the first k valid ones in group order
    // (network/NetFecCodec.cpp:504-528 == module/rs.c:620-629)
    if ((rc = run_reconstruct(*ctx, code, d->d_lut, nullptr, d->d_rec, d_shards, d_shards + (size_t)k * shard_pitch,
                              d_marks, groups, (int)shard_pitch, shard_pitch, nullptr, s, (long long)a.group_stride,
                              (long long)a.group_stride)))
        return rc;
    e = launch_check_payloads(a, s);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "check_payloads launch");
}


// ---- datagrams straight to / from ProtocolUdp frames (one pass where a kernel instance exists)
int qfec_pack_frames(qfec_code* code, const unsigned char* d_payload, const long long* d_offsets, const int* d_sizes,
                     const unsigned int* d_seq, long long groups, int checksum, unsigned char* d_shards,
                     long long shard_pitch, const unsigned char* d_mask, const unsigned int* d_conv_hid, int gmask,
                     int cmd, int protocol, unsigned char* d_frames, long long frame_pitch, int* d_frame_len,
                     void* stream) {
    const int fp = d_conv_hid ? 12 : 4;
    int rc = frame_check(code, groups, checksum, shard_pitch, frame_pitch, fp, d_shards, d_frames);
    if (rc) return rc;
    if (!d_mask || !d_frame_len) return QFEC_EINVAL;
    if (groups == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    if ((rc = current_ctx(&ctx))) return rc;
    uint32_t* tab = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_enc(code, ctx->device, &tab);
    }
    if (rc) return rc;
    const int k = code->k, m = code->m, n = k + m;
    hipStream_t s = (hipStream_t)stream;
    if (tuning().wire_fused) {
        WireArgs a{};
        a.payload = d_payload;
        a.offsets = (const int64_t*)d_offsets;
        a.sizes = d_sizes;
        a.seq = d_seq;
        a.pitch = (uint64_t)shard_pitch;
        a.group_stride = (uint64_t)n * shard_pitch;
        a.wire = d_frames;
        a.wire_pitch = (uint64_t)frame_pitch;
        a.wire_len = d_frame_len;
        a.groups = (uint64_t)groups;
        a.k = k;
        a.m = m;
        a.checksum = checksum;
        a.store_nt = 3;  // non-temporal datagram stores, body and head
        FrameSend fs{d_mask, d_conv_hid, (uint32_t)gmask & 0xFFu, (uint32_t)cmd, (uint32_t)protocol};
        bool launched = false;
        const hipError_t e = launch_pack_frames(a, fs, fp, tab, s, &launched);
        if (e != hipSuccess) return hip_fail(e, "pack_frames launch");
        if (launched) return QFEC_OK;
    }
    // two passes: datagrams into stream-ordered scratch, then qfec_frame_udp over them
    const long long wp = (long long)round_up((size_t)shard_pitch + 13, 16);
    const size_t rows = (size_t)groups * n, wbytes = rows * (size_t)wp;
    uint8_t* scratch = nullptr;
    if (hipMallocAsync((void**)&scratch, wbytes + rows * 4, s) != hipSuccess)
        return hip_fail(hipGetLastError(), "pack_frames scratch");
    int* wlen = reinterpret_cast<int*>(scratch + wbytes);
    rc = qfec_pack_datagrams(code, d_payload, d_offsets, d_sizes, d_seq, groups, checksum, d_shards, shard_pitch,
                             scratch, wp, wlen, stream);
    if (!rc)
        rc = qfec_frame_udp(scratch, wp, wlen, (long long)rows, d_mask, d_conv_hid, gmask, cmd, protocol, d_frames,
                            frame_pitch, d_frame_len, stream);
    (void)hipFreeAsync(scratch, s);
    return rc;
}

int qfec_unpack_frames(qfec_code* code, const unsigned char* d_frames, long long frame_pitch, const int* d_frame_len,
                       long long groups, int gmask, int session, int checksum, int dec_pkt_size,
                       unsigned char* d_shards, long long shard_pitch, unsigned char* d_marks, int* d_rx_size,
                       int* d_status, int* d_psize, int* d_frame_status, unsigned int* d_conv_hid, void* stream) {
    if (session != 0 && session != 1) return QFEC_EINVAL;
    const int fp = session ? 12 : 4;
    int rc = frame_check(code, groups, checksum, shard_pitch, frame_pitch, fp, d_shards, d_frames);
    if (rc) return rc;
    if (groups == 0) return QFEC_OK;
    if (!d_marks || !d_status || !d_psize || !d_frame_len) return QFEC_EINVAL;
    DevCtx* ctx = nullptr;
    if ((rc = current_ctx(&ctx))) return rc;
    DevTables* d = nullptr;
    {
        std::lock_guard<std::mutex> lk(code->mu);
        rc = ensure_lut(code, ctx->device, &d);
    }
    if (rc) return rc;
    const int k = code->k, m = code->m, n = k + m;
    hipStream_t s = (hipStream_t)stream;
    if (tuning().wire_rx && d->d_lut) {
        WireArgs a{};
        a.shards = d_shards;
        a.pitch = (uint64_t)shard_pitch;
        a.group_stride = (uint64_t)n * shard_pitch;
        a.wire = const_cast<uint8_t*>(d_frames);
        a.wire_pitch = (uint64_t)frame_pitch;
        a.wire_len = const_cast<int32_t*>(d_frame_len);
        a.marks = d_marks;
        a.rx_size = d_rx_size;
        a.status = d_status;
        a.psize = d_psize;
        a.groups = (uint64_t)groups;
        a.k = k;
        a.m = m;
        a.checksum = checksum;
        a.dec_pkt_size = dec_pkt_size;
        FrameRecv fr{(uint32_t)gmask & 0xFFu, d_frame_status, session ? d_conv_hid : nullptr};
        bool launched = false;
        const hipError_t e = launch_unpack_frames(a, fr, fp, d->d_lut, d->d_rec, (uint32_t)record_layout(k, m).hdr, s,
                                                  &launched);
        if (e != hipSuccess) return hip_fail(e, "unpack_frames launch");
        if (launched) return QFEC_OK;
    }
    // two passes: qfec_unframe_udp into stream-ordered scratch (rows RecvPacket rejects count as
    // not received), then qfec_unpack_datagrams
    const long long wp = (long long)round_up((size_t)frame_pitch, 16);
    const size_t rows = (size_t)groups * n, wbytes = rows * (size_t)wp;
    uint8_t* scratch = nullptr;
    if (hipMallocAsync((void**)&scratch, wbytes + rows * 8, s) != hipSuccess)
        return hip_fail(hipGetLastError(), "unpack_frames scratch");
    int* wlen = reinterpret_cast<int*>(scratch + wbytes);
    int* fst = d_frame_status ? d_frame_status : wlen + rows;
    rc = qfec_unframe_udp(d_frames, frame_pitch, d_frame_len, (long long)rows, gmask, session, scratch, wp, wlen, fst,
                          nullptr, session ? d_conv_hid : nullptr, stream);
    if (!rc) {
        const hipError_t e = launch_len_by_status(wlen, fst, rows, s);
        if (e != hipSuccess) rc = hip_fail(e, "len_by_status launch");
    }
    if (!rc)
        rc = qfec_unpack_datagrams(code, scratch, wp, wlen, groups, checksum, dec_pkt_size, d_shards, shard_pitch,
                                   d_marks, d_rx_size, d_status, d_psize, stream);
    (void)hipFreeAsync(scratch, s);
    return rc;
}

int qfec_gather_rows(const unsigned char* d_base, const unsigned long long* d_off, const int* d_len, long long rows,
                     int wrap_n, int wrap_k, unsigned char* d_out, long long out_pitch, int* d_out_len, void* stream) {
    if (rows < 0 || (rows && (!d_base || !d_off || !d_len || !d_out || !d_out_len)) || out_pitch < 16 || out_pitch % 16 ||
        (uintptr_t)d_out % 16 || wrap_n < 0 || wrap_n > 15 || (wrap_n && (wrap_k < 1 || wrap_k >= wrap_n))) {
        set_error("gather_rows: out_pitch a multiple of 16, 16-B aligned output, 0 < wrap_k < wrap_n <= 15");
        return QFEC_EINVAL;
    }
    if (rows == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    const int rc = current_ctx(&ctx);
    if (rc) return rc;
    const hipError_t e = launch_gather_rows(d_base, (const uint64_t*)d_off, d_len, (uint64_t)rows, wrap_n, wrap_k, d_out,
                                            (uint64_t)out_pitch, d_out_len, (hipStream_t)stream);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "gather_rows launch");
}

int qfec_frame_udp(const unsigned char* d_in, long long in_pitch, const int* d_len, long long rows,
                   const unsigned char* d_mask, const unsigned int* d_conv_hid, int gmask, int cmd, int protocol,
                   unsigned char* d_out, long long out_pitch, int* d_out_len, void* stream) {
    if (rows < 0 || !d_len || !d_mask || !d_out_len || in_pitch < 16 || out_pitch < 16 || in_pitch % 16 ||
        out_pitch % 16 || ((uintptr_t)d_in | (uintptr_t)d_out) % 16) {
        set_error("frame_udp: pitches must be multiples of 16 and rows 16-B aligned");
        return QFEC_EINVAL;
    }
    if (rows == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    FrameArgs a{};
    a.in = d_in;
    a.in_len = d_len;
    a.out = d_out;
    a.out_len = d_out_len;
    a.mask = d_mask;
    a.conv_hid = const_cast<uint32_t*>(d_conv_hid);
    a.rows = (uint64_t)rows;
    a.in_pitch = (uint64_t)in_pitch;
    a.out_pitch = (uint64_t)out_pitch;
    a.gmask = (uint32_t)gmask & 0xFFu;
    a.cmd = (uint32_t)cmd;
    a.protocol = (uint32_t)protocol;
    a.session = d_conv_hid != nullptr;
    const hipError_t e = launch_frame_udp(a, (hipStream_t)stream);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "frame_udp launch");
}

int qfec_unframe_udp(const unsigned char* d_in, long long in_pitch, const int* d_len, long long rows, int gmask,
                     int session, unsigned char* d_out, long long out_pitch, int* d_out_len, int* d_status,
                     unsigned char* d_info, unsigned int* d_conv_hid, void* stream) {
    if (rows < 0 || !d_len || !d_out_len || !d_status || (session != 0 && session != 1) || in_pitch < 16 ||
        out_pitch < 16 || in_pitch % 16 || out_pitch % 16 || ((uintptr_t)d_in | (uintptr_t)d_out) % 16) {
        set_error("unframe_udp: pitches must be multiples of 16 and rows 16-B aligned");
        return QFEC_EINVAL;
    }
    if (rows == 0) return QFEC_OK;
    DevCtx* ctx = nullptr;
    int rc = current_ctx(&ctx);
    if (rc) return rc;
    FrameArgs a{};
    a.in = d_in;
    a.in_len = d_len;
    a.out = d_out;
    a.out_len = d_out_len;
    a.conv_hid = d_conv_hid;
    a.status = d_status;
    a.info = d_info;
    a.rows = (uint64_t)rows;
    a.in_pitch = (uint64_t)in_pitch;
    a.out_pitch = (uint64_t)out_pitch;
    a.gmask = (uint32_t)gmask & 0xFFu;
    a.session = session;
    const hipError_t e = launch_unframe_udp(a, (hipStream_t)stream);
    return e == hipSuccess ? QFEC_OK : hip_fail(e, "unframe_udp launch");
}

}  // extern "C"

