/*
 * qfec.h -- batched, device-resident GF(2^8) Reed-Solomon API of libqfec.so (MI355X).
 *
 * This is the GPU boundary the reference does not have: the reference codecs work one
 * group (module/rs.c:574-643) or one packet (system/fec.c:714-862) at a time on the CPU.
 * Here many independent (k+m)-shard groups are encoded or reconstructed by one kernel
 * launch over device buffers, on the caller's HIP stream, with no host synchronisation.
 * The per-packet / per-call C ABIs (qfec_fec.h, qfec_rs.h) are built on top of it.
 *
 * Device layout (one contiguous region per role; `pitch` bytes between shard starts):
 *   data   [groups][k][pitch]   shard bytes [0, block_size) of each row are the payload
 *   parity [groups][m][pitch]
 *   marks  [groups*k data marks][groups*m parity marks]  (module/rs.c:609-612 layout;
 *          non-zero = erased)
 * With pitch == block_size, data followed by parity is exactly module/rs.c's shard order.
 * Bytes in [block_size, round_up(block_size, 16)) of a row may be read and written when
 * pitch allows (fast path); they are scratch.
 *
 * Arithmetic is bit-exact with module/rs.c (QFEC_CAUCHY) and module/fec.c / system/fec.c
 * (QFEC_VANDERMONDE), including rs.c's column-0 zero-coefficient behaviour when a code is
 * built with rs_stale_quirk = 1 (the default for QFEC_CAUCHY).
 *
 * All functions are thread-safe.  The device context of the calling thread's current HIP
 * device is created lazily, once.  `stream` is a hipStream_t passed as void* (NULL = the
 * null stream).  Return values: 0 or a negative QFEC_E* code.
 */
#ifndef QFEC_H
#define QFEC_H

#ifdef __cplusplus
extern "C" {
#endif

#define QFEC_CAUCHY 0      /* module/rs.c:437-440 parity rows (reed_solomon_new)   */
#define QFEC_VANDERMONDE 1 /* module/fec.c:653-707 parity rows (fec_new)          */

#define QFEC_OK 0
#define QFEC_EINVAL (-1)   /* bad argument / shape                                   */
#define QFEC_ENODEV (-2)   /* no HIP device                                          */
#define QFEC_EHIP (-3)     /* a HIP runtime call failed                              */
#define QFEC_ENOMEM (-4)   /* allocation failed                                      */
#define QFEC_EUNSUP (-5)   /* shape not supported by this entry point                */

#define QFEC_VARIANT_PERM 0    /* register byte-permute GF tables (v_perm_b32), default */
#define QFEC_VARIANT_LDSLOG 1  /* log/exp tables staged in LDS                          */

typedef struct qfec_code qfec_code;

/* A code over k data and m parity shards with the given parity-row flavour.
 * QFEC_CAUCHY: 1 <= k, 1 <= m, k + m <= 255 (rs.c:404).  QFEC_VANDERMONDE: 1 <= k,
 * 0 <= m, k + m <= 256 (fec.c:664).  NULL on error. */
qfec_code *qfec_code_new(int flavour, int k, int m);
/* A code over explicit m x k parity rows (row-major). */
qfec_code *qfec_code_from_rows(int k, int m, const unsigned char *parity_rows, int rs_stale_quirk);
void qfec_code_free(qfec_code *code);
int qfec_code_rows(const qfec_code *code, unsigned char *out_rows /* m*k */);
int qfec_code_shape(const qfec_code *code, int *k, int *m);

/* parity[g] = P x data[g] for every group g.  block_size >= 1, pitch >= block_size. */
int qfec_encode(qfec_code *code, const unsigned char *d_data, unsigned char *d_parity,
                long long groups, int block_size, long long pitch, void *stream);

/* qfec_encode on HOST buffers (the network path starts and ends in host memory).  Pinned
 * buffers the device can address (hipHostMalloc'd, or registered mapped) are read and written
 * in place by one launch over PCIe ("zero copy"); pageable ones run in ~32 MiB chunks over two
 * internal streams, staged through pinned memory, H2D -> encode -> D2H of one chunk overlapping
 * the staging of the next.  Returns after the parity is in h_parity.  Layouts as qfec_encode. */
int qfec_encode_host(qfec_code *code, const unsigned char *h_data, unsigned char *h_parity,
                     long long groups, int block_size, long long pitch);

/* qfec_reconstruct on HOST buffers: h_data is rewritten in place, h_marks is in the rs.c
 * layout over all `groups` (G*k data marks, then G*m parity marks); *failed (may be NULL) =
 * groups left under-determined.  k + m <= 24.  Pinned data and parity are worked on in place
 * (zero copy: the survivors are read and only the erased rows written, over PCIe; the marks are
 * staged); otherwise chunked and staged like qfec_encode_host. */
int qfec_reconstruct_host(qfec_code *code, unsigned char *h_data, const unsigned char *h_parity,
                          const unsigned char *h_marks, long long groups, int block_size, long long pitch,
                          long long *failed);

/* ---- host streaming pipe (BASELINE config 5: mixed (k,m) batches host -> device -> host) ----
 * A pipe owns `nstreams` slots per device (HIP stream + event + `slot_bytes` of device
 * staging), over the listed devices (devices = NULL / ndev = 0: every visible device;
 * a device may be listed more than once).  qfec_pipe_encode / qfec_pipe_reconstruct split a
 * batch into pieces that fit a slot and spread over all slots; each piece takes the next
 * slot round-robin (devices interleaved), waits for that slot's previous piece, and queues
 * its kernel on the pinned buffers in place (zero copy; only the piece's marks are staged)
 * -- or, with qfec_tune("host_zero_copy", 0) or a device that cannot address the buffers,
 * H2D -> kernel -> D2H through the slot's staging -- so the pieces overlap each other.  They return once the pieces are queued.  Host buffers must be
 * PINNED (hipHostMalloc'd or hipHostRegister'ed; DMA'd directly) and must not be touched
 * until qfec_pipe_wait returns.  Layouts as qfec_encode / qfec_reconstruct_host (marks in
 * the rs.c layout over the batch's `groups`).  Any number of codes may share a pipe.
 * qfec_pipe_wait: every queued piece has finished; *failed (may be NULL) = under-determined
 * groups since the previous wait.  On an error return the pipe has been drained. */
typedef struct qfec_pipe qfec_pipe;
qfec_pipe *qfec_pipe_new(const int *devices, int ndev, int nstreams, long long slot_bytes);
void qfec_pipe_free(qfec_pipe *pipe);
int qfec_pipe_encode(qfec_pipe *pipe, qfec_code *code, const unsigned char *h_data, unsigned char *h_parity,
                     long long groups, int block_size, long long pitch);
int qfec_pipe_reconstruct(qfec_pipe *pipe, qfec_code *code, unsigned char *h_data, const unsigned char *h_parity,
                          const unsigned char *h_marks, long long groups, int block_size, long long pitch);
int qfec_pipe_wait(qfec_pipe *pipe, long long *failed);
int qfec_pipe_slots(const qfec_pipe *pipe);

/* Rewrite every erased data shard from k survivors: the surviving data shards in
 * ascending order, then the first e surviving parity shards in ascending order
 * (module/rs.c:620-629; the same set network/NetFecCodec.cpp:504-528 hands to
 * fec_decode).  Groups with no erased data are untouched; groups with more erased data
 * than surviving parity are untouched and counted into *d_failed (device counter,
 * may be NULL; accumulated, not reset).  k + m <= 24: asynchronous on `stream`, erasure
 * pattern -> decode matrix through a device LUT.  k + m > 24: the marks are read back
 * (k + m bytes per group), decode records are built per distinct pattern on the host,
 * and the call returns after the kernel has run on `stream`. */
int qfec_reconstruct(qfec_code *code, unsigned char *d_data, const unsigned char *d_parity,
                     const unsigned char *d_marks, long long groups, int block_size,
                     long long pitch, unsigned int *d_failed, void *stream);

/* Build the per-erasure-pattern decode tables of `code` on the current device now
 * (otherwise done on the first qfec_reconstruct). */
int qfec_prepare_reconstruct(qfec_code *code);

/* Host-side decode-matrix query for one group (group-order marks[n]).  Writes e <= m
 * rows of k coefficients over the survivors listed in survivors[k] (shard ids 0..n-1).
 * Returns e, 0 when nothing is erased, or -1 when under-determined.  CPU only. */
int qfec_decode_rows(const qfec_code *code, const unsigned char *marks_n,
                     unsigned char *rows_out, int *survivors_out, int *erased_out);

/* The qfec_code behind a handle of the per-call ABIs, so a caller holding fec_new() /
 * reed_solomon_new() handles (e.g. network/FecCodec.cpp's codec list) can batch groups
 * through qfec_encode / qfec_reconstruct with the very same matrix. */
struct _reed_solomon;
qfec_code *qfec_fec_code(void *fec_handle);
qfec_code *qfec_rs_code(struct _reed_solomon *rs);
/* The n x k systematic matrix of a fec_new() handle (identity on top). */
int qfec_fec_matrix(void *fec_handle, unsigned char *out_full);

/* ---- FEC datagram batches: the network layer's shard + wire format ----
 * Send, for `groups` full groups of k packets (zfec_pack_input, network/NetFecCodec.cpp:96-172):
 *   shard (g, i)    = [size u16][cksum16(payload) u16 if checksum][payload], zero-filled
 *                     (set_fec_enc_buf, network/FecCodecBuf.cpp:66-103)
 *   check shards    = fec_encode(.., groupMax) (get_fec_encoded_pkt, FecCodecBuf.cpp:137-156)
 *   datagram (g, j) = [0xEC|0xED][sent u32][src u32][n | k<<4 | ik<<8 u16][cksum16 if 0xED][shard]
 *                     (pack_fec_head, FecCodecBuf.cpp:274-328); sent = seq[g][0] + j,
 *                     src = seq[g][1] + min(j, k - 1)
 * Receive reverses it: unpack_fec_head (:334-411; a failed shard checksum drops the
 * datagram), reconstruct of the missing data shards from the first k valid ones, and
 * dec_src_pkt_info (:109-133): status[g*k+i] = payload offset in the shard row (2 or 4),
 * -1 dropped (size >= dec_pkt_size or checksum mismatch), -2 lost (group unrecoverable);
 * psize = the payload size field.
 * Layout: d_shards [G][n][shard_pitch], d_wire [G][n][wire_pitch] (16-B aligned, pitches
 * multiples of 16, wire_pitch >= shard_pitch + 13), d_wire_len [G*n] (0 = not received),
 * d_marks [G*n] rs.c-layout scratch, d_rx_size [G*n] (nullable).  n = k + m <= 15 (the
 * header's 4-bit fields).  d_payload must stay readable 16 bytes past its last byte. */
int qfec_pack_datagrams(qfec_code *code, const unsigned char *d_payload, const long long *d_offsets,
                        const int *d_sizes, const unsigned int *d_seq, long long groups, int checksum,
                        unsigned char *d_shards, long long shard_pitch, unsigned char *d_wire,
                        long long wire_pitch, int *d_wire_len, void *stream);
int qfec_unpack_datagrams(qfec_code *code, const unsigned char *d_wire, long long wire_pitch,
                          const int *d_wire_len, long long groups, int checksum, int dec_pkt_size,
                          unsigned char *d_shards, long long shard_pitch, unsigned char *d_marks,
                          int *d_rx_size, int *d_status, int *d_psize, void *stream);

/* ---- ProtocolUdp framing of datagram batches ----
 * The byte stage below FEC.  Row r of d_out = Session::PacketOutput + ProtocolUdp::SendPacket
 * (network/SessionDesc.cpp:69-77, network/ProtocolBasic.cpp:111-150) applied to d_in row r:
 *   [mask][c][(cmd & 0x1f) | 0xA0][protocol]([conv u32 LE][hid u32 LE])[d_in[r][0, len)]
 * with bytes 1.. XORed by mask ^ gmask ^ 0x5a, mask = d_mask[r] (the session's _mask++),
 * c = CheckSum(bytes 2..) & 0xff, CheckSum(x) = ~(fold16(byte sum)) (ProtocolBasic.cpp:56-87).
 * The 8-byte Session prefix is present iff d_conv_hid ([rows][2] conv, hid) is non-NULL.
 * d_out_len[r] = framed length, or -1 when it does not fit out_pitch.  Bytes of a row past its
 * frame, up to out_pitch, are zero, and a row with d_out_len -1 is all zero (every path).
 * qfec_unframe_udp reverses it (ProtocolUdp::RecvPacket, ProtocolBasic.cpp:152-210):
 * d_status[r] = 0 ok, 1 short, 2 bad checksum, 3 bad cmd, 4 too long; d_out row = the data,
 * d_out_len = len - 4 (- 8 with session = 1); d_info [rows][4] = xor mask, c, cmd & 0x1f,
 * protocol (nullable); d_conv_hid receives the Session prefix when session = 1 (nullable; its
 * entries are meaningful only for rows whose d_status is 0).
 * Pitches multiples of 16, rows 16-B aligned. */
int qfec_frame_udp(const unsigned char *d_in, long long in_pitch, const int *d_len, long long rows,
                   const unsigned char *d_mask, const unsigned int *d_conv_hid, int gmask, int cmd, int protocol,
                   unsigned char *d_out, long long out_pitch, int *d_out_len, void *stream);
int qfec_unframe_udp(const unsigned char *d_in, long long in_pitch, const int *d_len, long long rows, int gmask,
                     int session, unsigned char *d_out, long long out_pitch, int *d_out_len, int *d_status,
                     unsigned char *d_info, unsigned int *d_conv_hid, void *stream);

/* ---- FEC datagrams straight to / from ProtocolUdp frames (SURVEY 8(f) ranks 2-4 fused) ----
 * qfec_pack_frames = qfec_pack_datagrams followed by qfec_frame_udp on every datagram, with
 * cmd / protocol as Session::TransmissionOutput sets them for FEC data (QUICKNET_CMD_DATA,
 * QUICKNET_PROTOCOL_FEC, network/SessionDesc.cpp:513-519): frame row (g, j) of d_frames =
 * [mask][c][(cmd & 0x1f) | 0xA0][protocol]([conv][hid])[datagram (g, j)], bytes 1.. XORed with
 * d_mask[g*n+j] ^ gmask ^ 0x5a; d_frame_len[g*n+j] = framed length (-1 for a void group).
 * The Session prefix is present iff d_conv_hid ([G*n][2]) is non-NULL.  Bytes of a row past its
 * frame, up to frame_pitch, are zero.  One pass (no datagram buffer in HBM) with checksums on, a
 * templated (k, m) and frame_pitch = 1088 or 576 equal to the 64-B multiple above prefix + 13 +
 * shard_pitch (1 KiB / 512-B payloads); other cases run the two calls over stream-ordered scratch.
 * d_shards is scratch as in qfec_pack_datagrams.
 * qfec_unpack_frames = qfec_unframe_udp (ProtocolUdp::RecvPacket, ProtocolBasic.cpp:155-199) of
 * every row, rows RecvPacket rejects counting as not received, then qfec_unpack_datagrams over
 * the datagrams inside: the same d_marks / d_rx_size / d_status / d_psize / d_shards as that
 * call.  d_frame_status [G*n] (nullable) = RecvPacket's verdict per row (0 ok, 1 short,
 * 2 checksum, 3 cmd, 4 too long, as qfec_unframe_udp; a row with both a bad checksum and a bad
 * cmd is 2, RecvPacket's order); d_conv_hid receives the Session prefix when session = 1
 * (nullable): its entries are meaningful only for rows whose d_frame_status is 0, the others are
 * unspecified.  One pass for the templated (k, m). */
int qfec_pack_frames(qfec_code *code, const unsigned char *d_payload, const long long *d_offsets,
                     const int *d_sizes, const unsigned int *d_seq, long long groups, int checksum,
                     unsigned char *d_shards, long long shard_pitch, const unsigned char *d_mask,
                     const unsigned int *d_conv_hid, int gmask, int cmd, int protocol, unsigned char *d_frames,
                     long long frame_pitch, int *d_frame_len, void *stream);
int qfec_unpack_frames(qfec_code *code, const unsigned char *d_frames, long long frame_pitch,
                       const int *d_frame_len, long long groups, int gmask, int session, int checksum,
                       int dec_pkt_size, unsigned char *d_shards, long long shard_pitch, unsigned char *d_marks,
                       int *d_rx_size, int *d_status, int *d_psize, int *d_frame_status,
                       unsigned int *d_conv_hid, void *stream);

/* Gather scattered rows (e.g. datagrams where a receive ring put them) into the pitched batch the
 * calls above take: row r of d_out = the d_len[r] bytes at d_base + d_off[r], zero-padded to
 * out_pitch, d_out_len[r] = d_len[r]; rows with d_len <= 0 get 0 and are not written, rows that
 * do not fit get -1.  wrap_n > 0: the rows are bare shards (row r = shard ik = r % wrap_n of a
 * group) and each gets the 11-byte header a 0xEC datagram of it carries ([0xEC][sent 0][src 0]
 * [wrap_n | wrap_k << 4 | ik << 8]), so qfec_unpack_datagrams decodes groups of chosen shards
 * (fec_decode_pkts, network/FecCodecBuf.cpp:181-232).  Sources stay readable 16 bytes past
 * their last byte. */
int qfec_gather_rows(const unsigned char *d_base, const unsigned long long *d_off, const int *d_len, long long rows,
                     int wrap_n, int wrap_k, unsigned char *d_out, long long out_pitch, int *d_out_len, void *stream);

/* Fill nbytes of device memory with the synthetic stream of quicknet_amd/synth.py. */
int qfec_synth_fill(unsigned char *d_ptr, long long nbytes, unsigned long long seed, void *stream);

/* module/rs.h on host shard pointers (reed_solomon_encode / reed_solomon_reconstruct with every shard
 * in host memory) pipelines its chunks over two slots on the calling thread's current device.
 * qfec_rs_host_devices spreads them over two slots per entry of `devices` instead -- each GPU has
 * its own PCIe link, and a device may be listed more than once (more chunks in flight on it); n = 0
 * goes back to the current device.  Outputs are identical either way.  Not to be called while a
 * module/rs.h call is running on another thread (it waits for it).  qfec_rs_host_devices_get
 * copies up to `cap` entries of the list and returns its length (0: the current device). */
int qfec_rs_host_devices(const int *devices, int n);
int qfec_rs_host_devices_get(int *devices, int cap);

/* Calibration probe, NOT a codec: streams the encode's traffic (k rows in, m rows out,
 * XOR only).  Its time is the memory-side ceiling the GF kernels are compared with. */
int qfec_probe_stream(const unsigned char *d_data, unsigned char *d_parity, long long groups, int k, int m,
                      int block_size, long long pitch, void *stream);

/* Calibration probe, NOT a codec: the reconstruct's memory skeleton for RS(10,3) and RS(16,4) --
 * the same mapping, marks reads, survivor rows and erased-row writes as the auto reconstruct body,
 * XOR in place of the decode (the erased rows receive garbage; no other byte is written).
 * lds_cap: LDS bytes per block (0 none), a residency cap.  QFEC_EUNSUP for other shapes. */
int qfec_probe_reconstruct(unsigned char *d_data, const unsigned char *d_parity, const unsigned char *d_marks,
                           long long groups, int k, int m, int block_size, long long pitch, int lds_cap,
                           void *stream);

/* Knobs.  Integration settings: host chunking, host copy threads, zero copy, the per-call
 * server's footprint.  Plus one A/B switch per kernel family (tools/ab.py, tools/wire_ab.py)
 * and one test hook.  Defaults are the measured best; outputs are identical either way.
 *   "host_zero_copy"   1 pinned host batches worked on in place | 0 staged copies (module/rs.h on host
 *                      pointers: the reconstruct only; its encode always stages through the device,
 *                      measured faster for a freshly gathered slot)
 *   "host_lanes"       4 (default) | 2 .. 8: module/rs.h on host pointers, chunk slots in flight on the
 *                      current device; qfec_rs_host_devices spreads them over listed devices instead
 *   "host_nt"          2 (default) | 1 | 0: module/rs.h on host pointers, streaming (non-temporal) stores
 *                      when gathering caller rows into a slot: 2 for rows that start where the previous
 *                      row ended, 1 for every row, 0 never
 *   "host_chunk"       groups per staged host chunk (0: by bytes: ~32 MiB for qfec_*_host, ~16 MiB of
 *                      caller shards for module/rs.h on host pointers)
 *   "host_threads"     host threads that gather / scatter module/rs.h host shard pointers (0: the
 *                      CPUs this process may use -- affinity and cgroup quota -- at most 32)
 *   "percall_resident" 1 fec_encode / fec_decode of packets up to 4 KiB with k <= 16 and k * e <= 64
 *                      go to a resident one-block server that polls a request word in device memory
 *                      and exits by itself after percall_idle_us without a request | 0 one launch per
 *                      call (setting 0 stops the servers)
 *   "percall_idle_us"  how long the resident server's block stays on the device after its last
 *                      request, 0 .. 1 000 000 us (default 1 000); 0 = it exits right after each
 *                      call (every call then pays a launch).  A hipDeviceSynchronize issued while it
 *                      is resident waits for it: at most this long after the last call.
 *   "percall_timeout_us" how long a call spins for the server before it stops the block and waits
 *                      for it (the block serves the pending request first), or, if the request was
 *                      never taken, runs it through one launch (default 2 000 000)
 *   "percall_stop_us"  how long that wait for the stopped block may last (default 2 000 000).  A
 *                      block still not done then (every CU held by other persistent kernels) is
 *                      abandoned: the call fails -- fec_encode prints to stderr and leaves dst as it
 *                      was, fec_decode returns 1 (module/fec.c's own failure shapes, fec.c:730-732,
 *                      833-836) -- and the device takes the one-launch path until percall_resident
 *                      is set to 1 again (the abandoned block's buffers stay allocated)
 *   "percall_fast"     1 per-packet calls on host packets through the server / one launch on mapped
 *                      pinned staging | 0 the staged DMA path (the one device-pointer packets take)
 *   "encode_lds"       -1 auto | 0 none | N: bytes of LDS each encode block allocates (and does not
 *                      use), of the CU's 160 KiB: a cap on the encode's resident waves per CU.  Auto
 *                      caps device-resident launches of >= 8 192 256-thread blocks at 16 waves per CU,
 *                      24 for the two-half inputs on rows <= 1 KiB, and runs 6 <= k <= 10 with m <= 3
 *                      (all rows in registers, rows >= 1 KiB with 128-B-aligned pitch, strides and
 *                      bases, >= 2^21 lanes) as one-wave blocks held
 *                      at 10 per CU (fewer concurrent row streams move more bytes per second through
 *                      HBM); k <= 2
 *                      and encodes of host memory are never capped.  The XOR probe follows the same
 *                      rule for its k (on one-wave blocks at 6 per CU, where its stream runs best)
 *   "encode_block"     -1 auto (64 where the rule above says so, else 256) | 64 | 256: threads per
 *                      encode block
 * A/B, one per kernel family:
 *   "encode_impl"      -1 auto (2 for k >= 16, else 0) | 0 all rows | 2 all rows, the inputs loaded in
 *                      two halves (fewer registers, more waves per SIMD)
 *   "recon_impl"       -1 auto | exact-e rows on 2 16-B lanes | 3 8-B lanes | 4 12-B lanes | 8 = 3 with
 *                      one group per block (auto picks it for 3 where a group is <= 4 waves)
 *   "wire_fused"       1 fused datagram send where a (k, m) instance exists | 0 staged build -> encode -> emit
 *   "wire_rx"          1 fused datagram receive (k_rx, one wave per group), lanes and LDS staging by
 *                      pitch | 2 / 3 16-B lanes with / without the K rows staged in LDS | 4 / 5 8-B
 *                      lanes likewise | 0 staged parse -> reconstruct -> check (3 launches)
 *   "percall_group"    1 fec_encode of a parity index computes the group's n - k rows in one request
 *                      and serves the group's other indices from a per-handle copy while src[], sz and
 *                      every input byte are unchanged | 0 one request per index
 * Test hook:
 *   "percall_fault"    1 requests are never handed to a server, so every call takes the timeout
 *                      branch | 2 the same, and the stopped server counts as not done within
 *                      percall_stop_us (the abandon branch) */
int qfec_tune(const char *key, int value);
/* The current value of a knob of qfec_tune (*value); QFEC_EINVAL for an unknown key. */
int qfec_tune_get(const char *key, int *value);

/* The resident per-call server of the current device (qfec_tune "percall_resident"): out[0] calls
 * it served, out[1] launches, out[2] relaunches because it had exited (idle) just before a request
 * arrived, out[3] 1 while its block may still be running (it exits 1 ms after the last request),
 * out[4] 1 set up | -1 unavailable on this device (device memory not CPU-mapped) | 0 not yet used.
 * Returns QFEC_OK, or an error without a device. */
int qfec_percall_stats(unsigned long long out[5]);
/* The same counters and more, as many as `n` asks for (returns how many were written, or an error):
 * [0..4] as qfec_percall_stats, [5] requests the server did not serve within percall_timeout_us
 * (each then waited for the stopped server, or ran through one launch), [6] / [7] fec_encode calls
 * served from / computing the group cache (all handles), [8] the current percall_idle_us, [9] servers
 * abandoned after percall_stop_us (qfec_percall_stats out[4] is then -2). */
int qfec_percall_counters(unsigned long long *out, int n);

int qfec_set_kernel_variant(int variant);
int qfec_get_kernel_variant(void);
int qfec_device_count(void);
const char *qfec_strerror(int err);
const char *qfec_last_error(void);
const char *qfec_version(void);

#ifdef __cplusplus
}
#endif

#endif /* QFEC_H */
