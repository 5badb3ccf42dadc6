// gf256.cpp -- host-side GF(2^8) arithmetic for libqfec: field tables, the two reference
// parity-matrix flavours, GF Gauss-Jordan inversion, decode-matrix selection and the
// perm-table / decode-record encodings the kernels consume.
//
// The field is built independently of the reference's table generator (carry-less
// multiply reduced by 0x11D, then exp/log from the generator 2); tests check it against
// the reference's tables (module/rs.c:157-216, module/fec.c:255-316) through the golden
// matrices.
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "qfec_internal.hpp"

namespace qfec {

namespace {

uint8_t clmul_reduce(uint8_t a, uint8_t b) {
    unsigned acc = 0, x = a;
    for (int i = 0; i < 8; ++i)
        if (b & (1u << i)) acc ^= x << i;
    for (int bit = 14; bit >= 8; --bit)
        if (acc & (1u << bit)) acc ^= 0x11Du << (bit - 8);
    return (uint8_t)acc;
}

Field g_field;
std::once_flag g_field_once;

void build_field() {
    Field& f = g_field;
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b) f.mul[a][b] = clmul_reduce((uint8_t)a, (uint8_t)b);
    uint8_t x = 1;
    memset(f.log, 0, sizeof(f.log));
    for (int i = 0; i < 255; ++i) {
        f.exp[i] = x;
        f.exp[i + 255] = x;
        f.log[x] = (uint8_t)i;
        x = f.mul[x][2];
    }
    f.exp[510] = f.exp[511] = 0;
    f.log[0] = 255;
    f.inv[0] = 0;
    for (int a = 1; a < 256; ++a) f.inv[a] = f.exp[(255 - f.log[a]) % 255];
}

}  // namespace

Tuning& tuning() {
    static Tuning t;
    return t;
}

const Field& field() {
    std::call_once(g_field_once, build_field);
    return g_field;
}

DivMagic make_div_magic(uint32_t d) {
    DivMagic m{};
    if (d == 0) d = 1;
    if ((d & (d - 1)) == 0) {
        m.pow2 = 1;
        m.shift = 0;
        while ((1u << m.shift) < d) ++m.shift;
        m.mul = 1;
        return m;
    }
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;  // l = ceil(log2 d)
    m.pow2 = 0;
    m.shift = l;
    // floor(2^(32+l) / d) + 1 : exact quotient for every n < 2^32
    m.mul = (uint64_t)(((unsigned __int128)1 << (32 + l)) / d) + 1;
    return m;
}

bool gf_invert(uint8_t* a, int k) {
    const Field& f = field();
    // augmented Gauss-Jordan with partial pivoting; the inverse is unique, so the
    // pivot order has no effect on the result.
    std::vector<uint8_t> aug((size_t)k * 2 * k, 0);
    const int w = 2 * k;
    for (int r = 0; r < k; ++r) {
        memcpy(&aug[(size_t)r * w], a + (size_t)r * k, (size_t)k);
        aug[(size_t)r * w + k + r] = 1;
    }
    for (int c = 0; c < k; ++c) {
        int p = c;
        while (p < k && aug[(size_t)p * w + c] == 0) ++p;
        if (p == k) return false;
        if (p != c)
            for (int j = 0; j < w; ++j) std::swap(aug[(size_t)p * w + j], aug[(size_t)c * w + j]);
        uint8_t* pr = &aug[(size_t)c * w];
        const uint8_t s = f.inv[pr[c]];
        for (int j = 0; j < w; ++j) pr[j] = f.mul[s][pr[j]];
        for (int r = 0; r < k; ++r) {
            if (r == c) continue;
            uint8_t* rr = &aug[(size_t)r * w];
            const uint8_t q = rr[c];
            if (!q) continue;
            const uint8_t* mq = f.mul[q];
            for (int j = 0; j < w; ++j) rr[j] ^= mq[pr[j]];
        }
    }
    for (int r = 0; r < k; ++r) memcpy(a + (size_t)r * k, &aug[(size_t)r * w + k], (size_t)k);
    return true;
}

bool gf_invert_rs(uint8_t* a, int k) {
    // module/rs.c:224-344 (invert_mat): in-place Gauss-Jordan whose pivot for step s is the
    // diagonal a[s][s] when column s is unused and non-zero, else the first non-zero entry
    // of an unused column in a row-major scan of the rows not yet pivoted.  The pivot row is
    // swapped into row `col`, scaled so the pivot reads 1/p, and eliminated from every other
    // row (skipped when it already is a unit row); the column swaps are undone at the end.
    // rs.c ignores the result (rs.c:556), so on failure the caller uses `a` exactly as the
    // elimination left it: rows swapped and reduced up to the failing step, no column swaps.
    const Field& f = field();
    std::vector<uint8_t> used((size_t)k, 0);
    std::vector<int> sw_row((size_t)k, -1), sw_col((size_t)k, -1);
    auto row = [&](int r) { return a + (size_t)r * k; };
    for (int s = 0; s < k; ++s) {
        int pr = -1, pc = -1;
        if (!used[s] && row(s)[s]) {
            pr = pc = s;
        } else {
            for (int r = 0; r < k && pc < 0; ++r) {
                if (used[r]) continue;
                for (int c = 0; c < k; ++c)
                    if (!used[c] && row(r)[c]) { pr = r; pc = c; break; }
            }
            if (pc < 0) return false;  // "pivot not found"
        }
        used[pc] = 1;
        if (pr != pc) std::swap_ranges(row(pr), row(pr) + k, row(pc));
        sw_row[s] = pr;
        sw_col[s] = pc;
        uint8_t* p = row(pc);
        if (p[pc] != 1) {
            const uint8_t* sc = f.mul[f.inv[p[pc]]];
            p[pc] = 1;
            for (int c = 0; c < k; ++c) p[c] = sc[p[c]];
        }
        bool unit = true;
        for (int c = 0; c < k && unit; ++c) unit = p[c] == (c == pc);
        if (unit) continue;
        for (int r = 0; r < k; ++r) {
            if (r == pc) continue;
            uint8_t* q = row(r);
            const uint8_t x = q[pc];
            q[pc] = 0;
            if (!x) continue;
            const uint8_t* mx = f.mul[x];
            for (int c = 0; c < k; ++c) q[c] ^= mx[p[c]];
        }
    }
    for (int s = k - 1; s >= 0; --s)
        if (sw_row[s] != sw_col[s])
            for (int r = 0; r < k; ++r) std::swap(row(r)[sw_row[s]], row(r)[sw_col[s]]);
    return true;
}

bool cauchy_rows(int k, int m, std::vector<uint8_t>& out) {
    // module/rs.c:404 shape check, :437-440 rows
    if (k <= 0 || m <= 0 || k + m > 255) return false;
    const Field& f = field();
    out.assign((size_t)m * k, 0);
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < k; ++i) out[(size_t)j * k + i] = f.inv[(m + i) ^ j];
    return true;
}

bool vandermonde_rows(int k, int m, std::vector<uint8_t>& out) {
    // module/fec.c:664 shape check; :678-699 construction.  Evaluation points 0, 1, a,
    // a^2, ...; the systematic matrix is V * V_top^-1, whose bottom rows are the parity.
    const int n = k + m;
    if (k <= 0 || m < 0 || k > 256 || n > 256) return false;
    const Field& f = field();
    std::vector<uint8_t> v((size_t)n * k, 0);
    v[0] = 1;
    for (int r = 1; r < n; ++r)
        for (int c = 0; c < k; ++c) v[(size_t)r * k + c] = f.exp[((r - 1) * c) % 255];
    std::vector<uint8_t> top(v.begin(), v.begin() + (size_t)k * k);
    if (!gf_invert(top.data(), k)) return false;
    out.assign((size_t)m * k, 0);
    for (int r = 0; r < m; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t acc = 0;
            const uint8_t* row = &v[(size_t)(k + r) * k];
            for (int i = 0; i < k; ++i) acc ^= f.mul[row[i]][top[(size_t)i * k + c]];
            out[(size_t)r * k + c] = acc;
        }
    return true;
}

static inline uint32_t pack4(uint8_t a, uint8_t b, uint8_t c, uint8_t d) {
    return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24);
}

void perm_entry(uint8_t c, uint32_t* o) {
    const Field& f = field();
    const uint8_t* mc = f.mul[c];
    o[0] = pack4(mc[0], mc[1], mc[2], mc[3]);
    o[1] = pack4(mc[4], mc[5], mc[6], mc[7]);
    o[2] = pack4(mc[0], mc[8], mc[16], mc[24]);
    o[3] = pack4(mc[32], mc[40], mc[48], mc[56]);
    o[4] = pack4(mc[0], mc[64], mc[128], mc[192]);
    o[5] = 0;
    o[6] = c ? f.log[c] : 0xFFu;
    o[7] = c;
}

int decode_rows(const uint8_t* P, int k, int m, const uint8_t* marks, std::vector<uint8_t>& rows,
                std::vector<int>& survivors, std::vector<int>& lost, const uint8_t* full) {
    lost.clear();
    survivors.clear();
    for (int i = 0; i < k; ++i) {
        if (marks[i]) lost.push_back(i);
        else survivors.push_back(i);
    }
    const int e = (int)lost.size();
    if (e == 0) return 0;
    // module/rs.c:620-629: the first e parity rows that are not erased, ascending
    for (int j = 0; j < m && (int)survivors.size() < k; ++j)
        if (!marks[k + j]) survivors.push_back(k + j);
    if ((int)survivors.size() < k) return -1;
    std::vector<uint8_t> d((size_t)k * k, 0);
    if (full) {
        // module/rs.c:528-556: every row of the sub-matrix comes from the handle's n x k
        // matrix `rs->m` (data rows included), and invert_mat's failure is ignored
        for (int r = 0; r < k; ++r) memcpy(&d[(size_t)r * k], full + (size_t)survivors[r] * k, (size_t)k);
        (void)gf_invert_rs(d.data(), k);
    } else {
        for (int r = 0; r < k; ++r) {
            const int s = survivors[r];
            if (s < k) d[(size_t)r * k + s] = 1;
            else memcpy(&d[(size_t)r * k], P + (size_t)(s - k) * k, (size_t)k);
        }
        if (!gf_invert(d.data(), k)) return -1;  // cannot happen for the MDS flavours
    }
    rows.assign((size_t)e * k, 0);
    for (int j = 0; j < e; ++j) memcpy(&rows[(size_t)j * k], &d[(size_t)lost[j] * k], (size_t)k);
    return e;
}

RecordLayout record_layout(int k, int m) {
    RecordLayout L;
    L.surv_off = 4;
    L.lost_off = 4 + k;
    L.coff = (4 + k + m + 7) & ~7;
    L.hdr = (L.coff + m * k + 7) & ~7;
    return L;
}

void build_record(const RecordLayout& L, int k, int e, const uint8_t* rows, const int* survivors,
                  const int* lost, bool rs_quirk, uint32_t* out) {
    memset(out, 0, L.words(e, k) * sizeof(uint32_t));
    out[0] = (uint32_t)e;
    for (int c = 0; c < k; ++c) out[L.surv_off + c] = (uint32_t)survivors[c];
    for (int j = 0; j < e; ++j) out[L.lost_off + j] = (uint32_t)lost[j];
    for (int j = 0; j < e; ++j)
        for (int c = 0; c < k; ++c) {
            uint32_t* t = out + L.hdr + ((size_t)j * k + c) * QFEC_TAB_STRIDE;
            perm_entry(rows[(size_t)j * k + c], t);
            out[L.coff + j * k + c] = (uint32_t)rows[(size_t)j * k + c] * (QFEC_TAB_STRIDE * 4);
        }
    // module/rs.c:116-117: a zero column-0 coefficient leaves the output's bytes in place
    // (flag in the row's first table; word 1 holds the same flags as a bit per row)
    if (rs_quirk)
        for (int j = 0; j < e; ++j)
            if (rows[(size_t)j * k] == 0) {
                out[L.hdr + ((size_t)j * k) * QFEC_TAB_STRIDE + 5] = 1;
                // word 1 covers rows 0..31: its readers (the specialised kernels, the LUT's seed
                // bit) only see codes with n <= QFEC_LUT_MAX_N; wider rows rely on the table flag
                if (j < 32) out[1] |= 1u << j;
            }
}

}  // namespace qfec
