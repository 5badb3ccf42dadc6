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

int sink_unpack(void *peer, const char *p, unsigned int size, unsigned int src) {
    (void)peer;
    (void)src;
    const unsigned char *q = (const unsigned char *)p;
    unsigned long long s = 0;
    for (unsigned int i = 0; i < size; ++i) s += q[i];
    ndeliv++;
    dbytes += size;
    dsum += s;
    return 0;
}

void sink_reset(void) { used = n = 0; ndeliv = dbytes = dsum = 0; }
size_t sink_count(void) { return n; }
const unsigned char *sink_buf(void) { return buf; }
const uint32_t *sink_offs(void) { return offs; }
const uint32_t *sink_lens(void) { return lens; }
const intptr_t *sink_peers(void) { return peers; }
unsigned long long sink_ndeliv(void) { return ndeliv; }
unsigned long long sink_dbytes(void) { return dbytes; }
unsigned long long sink_dsum(void) { return dsum; }
