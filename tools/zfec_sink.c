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
