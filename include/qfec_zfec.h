/* qfec_zfec.h -- network/NetFecCodec.cpp's FEC layer, exact, with its byte work batched on the
 * MI355X (the reference interface is NetFecCodec.h:82-156 + FecTransmission).
 *
 * One session = one NetFecCodecLayer set up as FecTransmission::Init does it
 * (FecTransmission.cpp:240-257): init_zfec_layer(max_pkt_size, buf_items, kmax), the candidate
 * codec list (2,4) (3,5) (5,8) (4,6) (3,4) (4,5) (5,6) (7,8), set_zfec_kn(k, n), enable_zfec,
 * enable_sorted_zfec.  CreateFecTransmission's defaults are 2048, 48, 10, (4, 5), enabled, unsorted.
 *
 * Calls are QUEUED per session in call order (pack input, unpack input, and the configuration
 * calls, which take effect between the queued packets exactly where they were made);
 * qfec_zfec_flush runs every session's queue through the reference's state machines
 *   zfec_pack_input    (NetFecCodec.cpp:68-175)   numbering, groups, dynamic k/n (:51-65, :167-170)
 *   zfec_unpack_input  (NetFecCodec.cpp:189-371)  the 48-slot window (update_fec_dec_buf :540-554),
 *                      unsorted immediate delivery (:256-265), sorted delivery with its expected
 *                      index and 2n skip-ahead (:266-293), flush_avail_pkts (:407-443), decode of
 *                      the first k valid packets (add_packet_fec_buf :485-535), bUsed bookkeeping
 * on the host (bookkeeping only), while every byte of work -- shard build, checksums, headers,
 * check packets, datagram and payload checksum verdicts, decoding -- runs in batched device
 * launches (qfec_pack_datagrams / qfec_unpack_datagrams) over all sessions' packets of the flush.
 * The callbacks then receive exactly what the reference's PackOutput / UnpackOutput would have,
 * per session in the same order, with the same bytes and source indices.
 *
 * Differences, documented:
 *   - outputs leave at the flush, not inside the input call (a batching layer);
 *   - a (k, n) change in the middle of a send group (set_zfec_kn between two packets of one
 *     group; the reference then numbers the rest of the group with the new n) takes effect at
 *     the group's end;
 *   - k > kmax: the reference's set_fec_enc_buf / set_fec_dec_buf silently drop rows ik >= kmax
 *     (FecCodecBuf.cpp:66-78, :162-169) and then encode / decode with stale buffers; such (k, n)
 *     are refused here (set_kn returns -3);
 *   - the receive side uses the reference's rules for which packets decode and in what order,
 *     reading them from its own copy of the window; a decode whose inputs include a row ik >= kmax
 *     (undefined in the reference) is skipped.
 * Thread-safe per context (one mutex); callbacks run on the flushing thread.
 */
#ifndef QFEC_ZFEC_H
#define QFEC_ZFEC_H

#include "qfec_net.h" /* qfec_pack_output_fn, qfec_unpack_output_fn */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qfec_zfec qfec_zfec;

qfec_zfec *qfec_zfec_new(void);
void qfec_zfec_free(qfec_zfec *z);

/* A session (FecTransmission::Init).  Returns its id (>= 0) or < 0. */
int qfec_zfec_session(qfec_zfec *z, void *peer, int max_pkt_size, int buf_items, int kmax, int k, int n,
                      int enabled, int is_sorted);

/* Queued configuration calls (NetFecCodec.cpp / FecTransmission::Option) */
int qfec_zfec_set_kn(qfec_zfec *z, int s, int k, int n, int add_new); /* set_zfec_kn :591-611 */
int qfec_zfec_enable(qfec_zfec *z, int s, int on);                    /* enable_zfec :375-378 */
int qfec_zfec_sorted(qfec_zfec *z, int s, int on);                    /* enable_sorted_zfec :752-755 */
int qfec_zfec_dynkn(qfec_zfec *z, int s, int on);                     /* enable_zfec_dynkn :385-388 */
int qfec_zfec_lost_rate(qfec_zfec *z, int s, float lost_rate);        /* set_transimision_state :182-186 */

/* Queued inputs: zfec_pack_input (a payload to send) and zfec_unpack_input (a datagram received) */
int qfec_zfec_pack_input(qfec_zfec *z, int s, const void *data, unsigned int size);
int qfec_zfec_unpack_input(qfec_zfec *z, int s, const void *datagram, unsigned int size);

/* Run every queue; returns the number of callbacks made (datagrams + deliveries), or < 0. */
int qfec_zfec_flush(qfec_zfec *z, qfec_pack_output_fn pack_out, qfec_unpack_output_fn unpack_out, void *stream);

/* [0] fec_src_count, [1] fec_restore_count (NetFecCodec.h), [2] i_sent_pkt, [3] i_recv_pkt,
 * [4] i_expected_packet, [5] current k, [6] current n, [7] decodes skipped as undefined */
int qfec_zfec_stats(const qfec_zfec *z, int s, long long *out8);

#ifdef __cplusplus
}
#endif

#endif /* QFEC_ZFEC_H */
