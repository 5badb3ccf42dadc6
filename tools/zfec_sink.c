/* tools/zfec_sink.c -- C callbacks for tools/zfec_rate.py (measurement aid, not the product).
 * sink_pack collects the datagrams a send flush hands to PackOutput (as a socket layer would
 * copy them out); sink_unpack counts the deliveries of a receive flush and sums their bytes,
 * so the rate tool checks every payload arrived without a Python call per packet. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static unsigned char *buf;
static size_t cap, used;
static uint32_t *offs, *lens;
static intptr_t *peers;
static size_t n, ncap;
static unsigned long long ndeliv, dbytes, dsum;

/* sum of the payload's little-endian 64-bit words (the last one zero-padded): order-free, so the
 * rate tool compares the total with the one of the payloads it sent */
static unsigned long long fold(const unsigned char *q, unsigned int size) {
    unsigned long long s = 0, w;
    unsigned int i = 0;
    for (; i + 8 <= size; i += 8) {
        memcpy(&w, q + i, 8);
        s += w;
    }
    if (i < size) {
        w = 0;
        memcpy(&w, q + i, size - i);
        s += w;
    }
    return s;
}


/* forwarding mode (sink_forward): the send flush's datagrams go straight into a receiving
 * context's qfec_zfec_unpack_input, session s -> rx session rx_of[s], dropping `ndrop` of
 * every n consecutive datagrams of a session (positions g, g+1, .. mod n of its g-th group) */
typedef int (*unpack_input_fn)(void *z, int s, const void *d, unsigned int size);
static void *fwd_z;
static unpack_input_fn fwd_fn;
static int *fwd_rx, fwd_n, fwd_ndrop;
static unsigned long long *fwd_cnt;

void sink_forward(void *z, void *fn, const int *rx_of, int nsess, int n, int ndrop) {
    fwd_z = z;
    fwd_fn = (unpack_input_fn)fn;
    free(fwd_rx);
    free(fwd_cnt);
    fwd_rx = malloc(sizeof(int) * (size_t)nsess);
    fwd_cnt = calloc((size_t)nsess, sizeof(unsigned long long));
    memcpy(fwd_rx, rx_of, sizeof(int) * (size_t)nsess);
    fwd_n = n;
    fwd_ndrop = ndrop;
}

int sink_pack_forward(void *peer, const char *p, unsigned int size) {
    const int s = (int)(intptr_t)peer - 1;
    const unsigned long long c = fwd_cnt[s]++;
    const int j = (int)(c % (unsigned long long)fwd_n), g = (int)(c / (unsigned long long)fwd_n);
    for (int t = 0; t < fwd_ndrop; ++t)
        if ((g + t) % fwd_n == j) return 0;
    ++n;
    return fwd_fn(fwd_z, fwd_rx[s], p, size);
}

/* sampled deliveries, for a byte check of the payloads against what was sent: every
 * `samp_every`-th delivery's peer, source index, size and bytes (up to SAMP_MAX of them) */
#define SAMP_MAX 4096
#define SAMP_BYTES 2048
static unsigned samp_every = 61, nsamp;
static int samp_peer[SAMP_MAX];
static unsigned samp_src[SAMP_MAX], samp_size[SAMP_MAX];
static unsigned char samp_buf[SAMP_MAX][SAMP_BYTES];

/* receive side without a copy: fold the payload where the layer hands it over */
static unsigned samp_left;  /* deliveries until the next sample (a countdown: no division per call) */
int sink_unpack_fold(void *peer, const char *p, unsigned int size, unsigned int src) {
    if (samp_every && samp_left-- == 0 && nsamp < SAMP_MAX) {
        samp_left = samp_every - 1;
        samp_peer[nsamp] = (int)(intptr_t)peer;
        samp_src[nsamp] = src;
        samp_size[nsamp] = size;
        memcpy(samp_buf[nsamp], p, size < SAMP_BYTES ? size : SAMP_BYTES);
        ++nsamp;
    }
    ndeliv++;
    dbytes += size;
    dsum += fold((const unsigned char *)p, size);
    return 0;
}

unsigned sink_nsamp(void) { return nsamp; }
const int *sink_samp_peer(void) { return samp_peer; }
const unsigned *sink_samp_src(void) { return samp_src; }
const unsigned *sink_samp_size(void) { return samp_size; }
const unsigned char *sink_samp_buf(void) { return &samp_buf[0][0]; }

/* end-to-end drivers: the per-packet input calls an application makes, as C loops, so their
 * cost is timed with the flushes.
 * sink_pack_inputs: sender session sess[i] gets `packets` payloads, the p-th being payload
 * (i * 7 + p + rep) % npay of the `npay` payloads of `size` bytes at pay; returns 0 or the first
 * failing call's code.  *sum = the fold of everything sent. */
typedef int (*pack_input_fn)(void *z, int s, const void *d, unsigned int size);
int sink_pack_inputs(void *z, void *fn, const int *sess, int nsess, int packets, const unsigned char *pay, int npay,
                     int size, int rep, unsigned long long *sum, const unsigned long long *pay_fold) {
    pack_input_fn f = (pack_input_fn)fn;
    unsigned long long s = 0;
    for (int i = 0; i < nsess; ++i)
        for (int p = 0; p < packets; ++p) {
            const int j = (i * 7 + p + rep) % npay;
            const int rc = f(z, sess[i], pay + (size_t)j * (size_t)size, (unsigned)size);
            if (rc < 0) return rc;
            s += pay_fold[j];
        }
    *sum = s;
    return 0;
}

/* sink_unpack_inputs: the datagrams sink_pack collected go to a receiving context's
 * unpack_input, session peer - 1 -> rx_of[peer - 1], dropping `ndrop` of every n consecutive
 * datagrams of a session the way sink_pack_forward does; returns the number handed over or a
 * negative code */
long long sink_unpack_inputs(void *z, void *fn, const int *rx_of, int nsess, int nn, int ndrop) {
    unpack_input_fn f = (unpack_input_fn)fn;
    /* per session: position j in its current group of nn and that group's index g mod nn, kept
     * incrementally (the same drops as sink_pack_forward, without a division per datagram) */
    int *pos = calloc((size_t)nsess * 2, sizeof(int));
    long long kept = 0;
    for (size_t i = 0; i < n; ++i) {
        const int s = (int)peers[i] - 1;
        const int j = pos[2 * s], gm = pos[2 * s + 1];
        if (++pos[2 * s] == nn) {
            pos[2 * s] = 0;
            pos[2 * s + 1] = gm + 1 == nn ? 0 : gm + 1;
        }
        int drop = 0;
        for (int t = 0; t < ndrop; ++t) {
            const int x = gm + t;
            if ((x >= nn ? x - nn : x) == j) drop = 1;
        }
        if (drop) continue;
        const int rc = f(z, rx_of[s], buf + offs[i], lens[i]);
        if (rc < 0) {
            free(pos);
            return rc;
        }
        ++kept;
    }
    free(pos);
    return kept;
}

int sink_pack(void *peer, const char *p, unsigned int size) {
    if (used + size > cap) {
        size_t c = (used + size) * 2 + (1 << 20);
        unsigned char *nb = realloc(buf, c);
        if (!nb) return -1;
        buf = nb;
        cap = c;
    }
    if (n == ncap) {
        size_t c = ncap * 2 + 4096;
        uint32_t *no = realloc(offs, c * 4), *nl;
        if (!no) return -1;
        offs = no;
        nl = realloc(lens, c * 4);
        if (!nl) return -1;
        lens = nl;
        intptr_t *np = realloc(peers, c * sizeof(intptr_t));
        if (!np) return -1;
        peers = np;
        ncap = c;
    }
    memcpy(buf + used, p, size);
    offs[n] = (uint32_t)used;
    lens[n] = size;
    peers[n] = (intptr_t)peer;
    used += size;
    ++n;
    return 0;
}

/* the application's copy of a delivered payload (a ring it consumes from) */
static unsigned char app[1 << 22];
static size_t app_pos;

int sink_unpack(void *peer, const char *p, unsigned int size, unsigned int src) {
    (void)peer;
    (void)src;
    if (app_pos + size > sizeof(app)) app_pos = 0;
    memcpy(app + app_pos, p, size);
    app_pos += size;
    ndeliv++;
    dbytes += size;
    dsum += fold(app + app_pos - size, size);
    return 0;
}

unsigned long long sink_fold(const unsigned char *q, unsigned int size) { return fold(q, size); }

void sink_reset(void) { used = n = 0; ndeliv = dbytes = dsum = 0; nsamp = 0; samp_left = 0; }
size_t sink_count(void) { return n; }
const unsigned char *sink_buf(void) { return buf; }
const uint32_t *sink_offs(void) { return offs; }
const uint32_t *sink_lens(void) { return lens; }
const intptr_t *sink_peers(void) { return peers; }
unsigned long long sink_ndeliv(void) { return ndeliv; }
unsigned long long sink_dbytes(void) { return dbytes; }
unsigned long long sink_dsum(void) { return dsum; }
