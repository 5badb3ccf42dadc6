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

/* receive side without a copy: fold the payload where the layer hands it over */
int sink_unpack_fold(void *peer, const char *p, unsigned int size, unsigned int src) {
    (void)peer;
    (void)src;
    ndeliv++;
    dbytes += size;
    dsum += fold((const unsigned char *)p, size);
    return 0;
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

void sink_reset(void) { used = n = 0; ndeliv = dbytes = dsum = 0; }
size_t sink_count(void) { return n; }
const unsigned char *sink_buf(void) { return buf; }
const uint32_t *sink_offs(void) { return offs; }
const uint32_t *sink_lens(void) { return lens; }
const intptr_t *sink_peers(void) { return peers; }
unsigned long long sink_ndeliv(void) { return ndeliv; }
unsigned long long sink_dbytes(void) { return dbytes; }
unsigned long long sink_dsum(void) { return dsum; }
