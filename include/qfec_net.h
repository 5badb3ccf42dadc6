/* qfec_net.h -- batched NetFecCodec layer over libqfec.
 *
 * The reference runs the FEC layer one packet at a time per session:
 *   zfec_pack_input   (network/NetFecCodec.cpp:68-175)  send: shard, header, and at the
 *                     k-th packet of a group fec_encode of the n - k check packets;
 *   zfec_unpack_input (network/NetFecCodec.cpp:189-371) receive: header, dec buffer,
 *                     fec_decode_pkts once k valid datagrams of a group are in.
 * This layer keeps the same per-session numbering (i_sent_pkt / i_sent_src_pkt, init 0 as in
 * init_zfec_layer, :613-626) and the same wire bytes, but defers the byte work: complete
 * groups of ALL sessions are packed by one qfec_pack_datagrams launch per flush, and
 * received groups of all sessions are unpacked by one qfec_unpack_datagrams launch.
 *
 * Differences from the per-packet layer, by design:
 *   - a session's datagrams leave at the flush after its group completes (the reference
 *     sends each source datagram at once and the check datagrams at the k-th);
 *   - received packets are delivered per group, in source order (the reference's default
 *     is_sorted mode), at the flush that processes the group;
 *   - the handle sends with one (k, n); it receives groups of any (k, n) with n <= 15, each
 *     decoded with the code its headers name (the reference looks the codec up per header,
 *     NetFecCodec.cpp:301, but only decodes the (k, n) pairs registered with it);
 *   - datagrams arriving for a group already processed are dropped (counted).
 * Non-FEC datagrams (tag other than 0xEC / 0xED, or shorter than 11 bytes: FEC off at the
 * sender) are handed over minus their tag byte with source index 0, as zfec_unpack_input
 * does (:200-209), at the next flush_unpack before the groups.
 * Output callbacks have the reference's signatures (NetFecCodec.h:72-73).  Thread-safe per
 * handle (an internal mutex); callbacks run on the flushing thread. */
#ifndef QFEC_NET_H
#define QFEC_NET_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qfec_net qfec_net;

/* zfec.PackOutput(outpeer, packet, size) */
typedef int (*qfec_pack_output_fn)(void *peer, const char *packet, unsigned int size);
/* zfec.UnpackOutput(peer, packet, size, i_src_pkt) */
typedef int (*qfec_unpack_output_fn)(void *peer, const char *packet, unsigned int size, unsigned int i_src_pkt);

/* k source packets + (n - k) check packets per group, n <= 15 (the header's 4-bit fields);
 * payloads up to max_pkt_size bytes; checksum 1 = 0xED datagrams with payload and datagram
 * checksums (init_zfec_layer's default is_send_checksum = true), 0 = 0xEC. */
qfec_net *qfec_net_new(int k, int n, int max_pkt_size, int checksum);
void qfec_net_free(qfec_net *net);

/* A session = one NetFecCodecLayer's FEC state; peer is handed back to the callbacks. */
int qfec_net_session(qfec_net *net, void *peer);

/* enable_zfec (NetFecCodec.cpp:375-378, FecTransmission.cpp:72-77); sessions start enabled.
 * With FEC off, qfec_net_pack_input queues [0x13][payload] (pack_fec_off_tag,
 * FecCodecBuf.cpp:237-269), sent at the next flush before the session's groups, and the
 * session's FEC numbering does not advance (NetFecCodec.cpp:75-94). */
int qfec_net_enable(qfec_net *net, int session, int on);

/* zfec_pack_input: queue one payload of session s.  Returns 0, or < 0 (size > max_pkt_size,
 * bad session).  The session's group is packed at the next flush once it holds k packets. */
int qfec_net_pack_input(qfec_net *net, int session, const void *data, unsigned int size);

/* One device launch for every complete group of every session; then out(peer, datagram,
 * len) for each datagram, session by session, in sent order.  Returns the number of
 * datagrams emitted, or < 0. */
int qfec_net_flush_pack(qfec_net *net, qfec_pack_output_fn out, void *stream);

/* zfec_unpack_input: file one received datagram of session s under its group (sent index -
 * ik).  Returns 1 queued, 0 dropped (not an FEC datagram of this code, or late), < 0 error. */
int qfec_net_unpack_input(qfec_net *net, int session, const char *datagram, unsigned int size);

/* One device launch over the queued groups: with all = 0 those holding at least k
 * datagrams, with all = 1 every queued group.  Then out(peer, payload, size, i_src_pkt) for
 * each source packet received or recovered with a good checksum, group by group in source
 * order.  Returns the number of packets delivered, or < 0. */
int qfec_net_flush_unpack(qfec_net *net, qfec_unpack_output_fn out, int all, void *stream);

/* counters: [0] groups packed, [1] datagrams emitted, [2] groups unpacked, [3] packets
 * delivered, [4] packets recovered (delivered from lost datagrams), [5] groups that could
 * not be decoded, [6] datagrams dropped as foreign, [7] datagrams dropped as late */
int qfec_net_stats(const qfec_net *net, long long *out8);

#ifdef __cplusplus
}
#endif

#endif /* QFEC_NET_H */
