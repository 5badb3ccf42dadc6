/*
 * qfec_fec.h -- drop-in for the reference's per-packet systematic-Vandermonde codec.
 *
 * Replaces system/fec.h:233-246 (== module/fec.h) of skywind3000/QuickNet, the codec the
 * network stack links (network/FecCodec.cpp:5,84,133; network/FecCodecBuf.cpp:13,151,204),
 * with the same C ABI, exported by libqfec.so.  The GF(2^8) multiply-accumulate runs in
 * HIP kernels on an MI355X; packet buffers may be host or device memory.
 *
 * Semantics kept bit-exact with system/fec.c:
 *   - fec_new(k, n): parity rows = V_bottom * V_top^-1 of the Vandermonde matrix on the
 *     points 0, 1, a, a^2 ...; NULL (and a message on stderr) for k > 256, n > 256 or
 *     k > n                                                         (fec.c:653-707)
 *   - fec_encode(): index < k copies src[index]; k <= index < n writes one parity packet
 *     of sz bytes; any other index writes nothing                     (fec.c:714-733)
 *   - fec_decode(): shuffles data packets into their own slots, permuting pkt[] and
 *     index[] in place; recovered data i lands in slot i (a slot that held a parity
 *     packet, whose index value is kept); returns 1 on a shuffle conflict, an index >= n
 *     or a singular matrix, else 0                                    (fec.c:738-862)
 *   - a negative index (undefined behaviour in the reference) is rejected with 1.
 *
 * Device footprint: host packets of up to 4 KiB (k <= 16, k * rows <= 64) are served by a
 * resident one-block kernel on the library's own stream.  After the last call that block stays
 * on the device for at most percall_idle_us (qfec_tune, default 1 ms) and then exits by itself,
 * so a hipDeviceSynchronize() issued right after a call may wait up to that long;
 * qfec_tune("percall_idle_us", 0) makes it exit after every call.
 * fec_encode of a parity index computes the group's n - k rows at once and serves the group's
 * other indices from a per-handle copy while src[], sz and every input byte are unchanged.
 *
 * Device failure: a call whose request the resident block has not served within
 * percall_timeout_us (default 2 s; e.g. other kernels hold every CU) stops the block and waits
 * for it at most percall_stop_us more (default 2 s).  If the block still has not run then, the
 * call gives up: fec_encode prints "[qfec] fec_encode: ..." to stderr and leaves dst as it was (as
 * the reference does for an invalid index), fec_decode returns 1 (as for a singular matrix).  The
 * same two outcomes report any other device error.  Neither call blocks longer than about
 * percall_timeout_us + percall_stop_us in the server path (tests/test_gpu_host.py::
 * test_percall_abandon_branch).
 */
#ifndef QFEC_FEC_H
#define QFEC_FEC_H

#ifdef __cplusplus
extern "C" {
#endif

/* fec.h:237 */
void *fec_new(int k, int n);
/* fec.h:238 */
void fec_free(void *p);
/* fec.h:240 -- u_char in the reference; same ABI */
void fec_encode(void *code, unsigned char **src, unsigned char *dst, int index, int sz);
/* fec.h:241 */
int fec_decode(void *code, unsigned char **pkt, int *index, int sz);

#ifdef __cplusplus
}
#endif

#endif /* QFEC_FEC_H */
