/*
 * qfec_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * A plain-C, scalar restatement of the two GF(2^8) Reed-Solomon erasure codecs that
 * skywind3000/QuickNet carries, written from a reading of the reference sources:
 *
 *   - module/rs.c   : Cauchy parity matrix, batched encode / reconstruct over groups
 *   - module/fec.c  : Rizzo's systematic-Vandermonde codec, per-packet encode / decode
 *                     (system/fec.c is byte-identical and is what network/ links)
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library (liboracle.so), and only to check or time against. The product path lives in
 * quicknet_amd/csrc and never links or calls anything here.
 *
 * Parity of this restatement is pinned by the tests/golden vectors, which oracle/gen_golden.py
 * produced by running the reference itself (compiled by oracle/Makefile into
 * oracle/_ref/ from /root/reference/module/{rs,fec}.c).
 *
 * Every function cites the reference lines it follows.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint8_t u8;

/* ------------------------------------------------------------------ field tables */
/* rs.c:52 GF_PP "101110001" == fec.c:136 allPp[8]: 1 + x^2 + x^3 + x^4 + x^8 (0x11D). */
static u8 t_exp[2 * 255];
static int t_log[256];
static u8 t_inv[256];
static u8 t_mul[256][256];
static int t_ready = 0;

/* generate_gf(): rs.c:157-216, fec.c:255-316 */
static void build_field(void)
{
    const char *poly = "101110001";
    u8 bit = 1;
    int i;
    t_exp[8] = 0;
    for (i = 0; i < 8; ++i, bit = (u8)(bit << 1)) {
        t_exp[i] = bit;
        t_log[bit] = i;
        if (poly[i] == '1')
            t_exp[8] ^= bit;
    }
    t_log[t_exp[8]] = 8;
    for (i = 9; i < 255; ++i) {
        u8 prev = t_exp[i - 1];
        t_exp[i] = (prev & 0x80) ? (u8)(t_exp[8] ^ (u8)((prev ^ 0x80) << 1)) : (u8)(prev << 1);
        t_log[t_exp[i]] = i;
    }
    t_log[0] = 255;
    for (i = 0; i < 255; ++i)
        t_exp[i + 255] = t_exp[i];
    t_inv[0] = 0;
    t_inv[1] = 1;
    for (i = 2; i < 256; ++i)
        t_inv[i] = t_exp[255 - t_log[i]];
}

/* init_mul_table(): rs.c:144-152 (flat) / fec.c:197-207 (2-D); row and column 0 forced to 0 */
static void build_mul(void)
{
    int a, b;
    for (a = 0; a < 256; ++a)
        for (b = 0; b < 256; ++b)
            t_mul[a][b] = t_exp[(t_log[a] + t_log[b]) % 255];
    for (a = 0; a < 256; ++a)
        t_mul[0][a] = t_mul[a][0] = 0;
}

void orc_init(void)
{
    if (t_ready)
        return;
    build_field();
    build_mul();
    t_ready = 1;
}

u8 orc_mul(u8 a, u8 b) { orc_init(); return t_mul[a][b]; }
u8 orc_inv(u8 a) { orc_init(); return t_inv[a]; }
u8 orc_exp(int i) { orc_init(); return t_exp[i]; }
int orc_log(u8 a) { orc_init(); return t_log[a]; }

/* ------------------------------------------------------------------ linear algebra */

/* Gauss-Jordan with the Numerical-Recipes pivot search (diagonal first, then a
 * row-major scan over unused rows/columns), row swaps while eliminating and
 * column un-swaps at the end.  invert_mat(): rs.c:224-344 == fec.c:418-542.
 * Returns 0 on success, 1 if singular. */
int orc_invert(u8 *a, int k)
{
    int *col_of = (int *)malloc(sizeof(int) * (size_t)k);
    int *row_of = (int *)malloc(sizeof(int) * (size_t)k);
    int *used = (int *)calloc((size_t)k, sizeof(int));
    u8 *unit = (u8 *)calloc((size_t)k, 1);
    int step, rc = 1;

    orc_init();
    for (step = 0; step < k; ++step) {
        int pr = -1, pc = -1, r, c;
        u8 *prow, f;
        if (used[step] != 1 && a[step * k + step] != 0) {
            pr = pc = step;
        } else {
            for (r = 0; r < k && pr < 0; ++r) {
                if (used[r] == 1)
                    continue;
                for (c = 0; c < k; ++c) {
                    if (used[c] == 0) {
                        if (a[r * k + c] != 0) { pr = r; pc = c; break; }
                    } else if (used[c] > 1) {
                        goto out; /* "singular matrix" */
                    }
                }
            }
            if (pc < 0)
                goto out; /* "pivot not found" */
        }
        used[pc] += 1;
        if (pr != pc)
            for (c = 0; c < k; ++c) { u8 t = a[pr * k + c]; a[pr * k + c] = a[pc * k + c]; a[pc * k + c] = t; }
        row_of[step] = pr;
        col_of[step] = pc;
        prow = a + pc * k;
        f = prow[pc];
        if (f == 0)
            goto out; /* "singular matrix 2" */
        if (f != 1) {
            f = t_inv[f];
            prow[pc] = 1;
            for (c = 0; c < k; ++c)
                prow[c] = t_mul[f][prow[c]];
        }
        unit[pc] = 1;
        if (memcmp(prow, unit, (size_t)k) != 0) {
            for (r = 0; r < k; ++r) {
                u8 *row = a + r * k;
                if (r == pc)
                    continue;
                f = row[pc];
                row[pc] = 0;
                if (f)
                    for (c = 0; c < k; ++c)
                        row[c] ^= t_mul[f][prow[c]];
            }
        }
        unit[pc] = 0;
    }
    for (step = k - 1; step >= 0; --step) {
        int x = row_of[step], y = col_of[step], r;
        if (x < 0 || x >= k || y < 0 || y >= k || x == y)
            continue;
        for (r = 0; r < k; ++r) { u8 t = a[r * k + x]; a[r * k + x] = a[r * k + y]; a[r * k + y] = t; }
    }
    rc = 0;
out:
    free(col_of); free(row_of); free(used); free(unit);
    return rc;
}

/* ------------------------------------------------------------------ matrix builders */

/* reed_solomon_new(): rs.c:387-476.  The identity top is untouched by the inversion and
 * product the reference performs (rs.c:416-435); the parity rows are the Cauchy rows
 * P[j][i] = inverse[(m + i) XOR j] (rs.c:437-440).  Writes m*k bytes.
 * Returns 0, or the reference's errno 1 for bad shapes (rs.c:404). */
int orc_cauchy_parity(int k, int m, u8 *out)
{
    int i, j;
    orc_init();
    if (k + m > 255 || k <= 0 || m <= 0)
        return 1;
    for (j = 0; j < m; ++j)
        for (i = 0; i < k; ++i)
            out[j * k + i] = t_inv[(m + i) ^ j];
    return 0;
}

/* invert_vdm(): fec.c:556-610.  In-place inverse of a k x k Vandermonde matrix whose
 * second column holds the evaluation points p_i (p_0 = 0 for the special first row). */
static void invert_vandermonde(u8 *v, int k)
{
    u8 *coef, *syn, *pts;
    int i, j, row, col;
    if (k == 1)
        return;
    coef = (u8 *)calloc((size_t)k, 1);
    syn = (u8 *)calloc((size_t)k, 1);
    pts = (u8 *)calloc((size_t)k, 1);
    for (i = 0; i < k; ++i)
        pts[i] = v[i * k + 1];
    /* coefficients of P(x) = prod (x - p_i), leading 1 implicit */
    coef[k - 1] = pts[0];
    for (i = 1; i < k; ++i) {
        for (j = k - i; j < k - 1; ++j)
            coef[j] ^= t_mul[pts[i]][coef[j + 1]];
        coef[k - 1] ^= pts[i];
    }
    for (row = 0; row < k; ++row) {
        u8 x = pts[row], t = 1;
        syn[k - 1] = 1;
        for (i = k - 2; i >= 0; --i) {
            syn[i] = (u8)(coef[i + 1] ^ t_mul[x][syn[i + 1]]);
            t = (u8)(t_mul[x][t] ^ syn[i]);
        }
        for (col = 0; col < k; ++col)
            v[col * k + row] = t_mul[t_inv[t]][syn[col]];
    }
    free(coef); free(syn); free(pts);
}

/* fec_new(): fec.c:653-707.  Writes the (n-k) x k parity rows of the systematic matrix.
 * Returns 0, or 1 for the reference's rejected shapes (fec.c:664). */
int orc_vandermonde_parity(int k, int n, u8 *out)
{
    u8 *v;
    int r, c, i;
    orc_init();
    if (k > 256 || n > 256 || k > n || k <= 0)
        return 1;
    v = (u8 *)calloc((size_t)n * (size_t)k, 1);
    v[0] = 1; /* row 0 = point 0: [1, 0, ..., 0] */
    for (r = 1; r < n; ++r)
        for (c = 0; c < k; ++c)
            v[r * k + c] = t_exp[((r - 1) * c) % 255];
    invert_vandermonde(v, k);
    /* parity = bottom (n-k) rows x inverse(top) (fec.c:375-389, :693) */
    for (r = 0; r < n - k; ++r)
        for (c = 0; c < k; ++c) {
            u8 acc = 0;
            for (i = 0; i < k; ++i)
                acc ^= t_mul[v[(k + r) * k + i]][v[i * k + c]];
            out[r * k + c] = acc;
        }
    free(v);
    return 0;
}

/* ------------------------------------------------------------------ rs.c codec */

/* code_some_shards(): rs.c:364-378, with mul()/addmul() (rs.c:96-118).
 * Column 0 is a plain multiply; a zero coefficient there leaves dst as it was
 * (the reference's memset of 0 bytes, rs.c:116-117). */
static void rs_apply(const u8 *rows, u8 *const *in, u8 *const *out, int k, int nout, int len)
{
    int c, r, b;
    for (c = 0; c < k; ++c) {
        const u8 *src = in[c];
        for (r = 0; r < nout; ++r) {
            u8 f = rows[r * k + c];
            u8 *dst = out[r];
            if (f == 0)
                continue;
            if (c == 0)
                for (b = 0; b < len; ++b) dst[b] = t_mul[f][src[b]];
            else
                for (b = 0; b < len; ++b) dst[b] ^= t_mul[f][src[b]];
        }
    }
}

/* reed_solomon_encode(): rs.c:574-588.  shards[0 .. G*k-1] are all data shards
 * (group-major), shards[G*k .. G*n-1] all parity shards. */
int orc_rs_encode(int k, int m, const u8 *parity_rows, u8 **shards, int nr_shards, int len)
{
    int groups = nr_shards / (k + m), g;
    orc_init();
    for (g = 0; g < groups; ++g)
        rs_apply(parity_rows, shards + (size_t)g * k, shards + (size_t)groups * k + (size_t)g * m, k, m, len);
    return 0;
}


/* reed_solomon_decode() (rs.c:500-565) for one group.  `lost` are the erased data
 * indices (sorted here, rs.c:512-526), `fixp` the chosen parity buffers, `fixr` their
 * parity-row numbers, all of length e. */
static int rs_decode_group(int k, const u8 *parity_rows, const u8 *full, u8 **data, u8 **fixp,
                           const int *fixr, int *lost, int e, int len)
{
    u8 *mat = (u8 *)malloc((size_t)k * (size_t)k);
    u8 **in = (u8 **)malloc(sizeof(u8 *) * (size_t)k);
    u8 **out = (u8 **)malloc(sizeof(u8 *) * (size_t)(e > 0 ? e : 1));
    int i, j, rows = 0, x = 0;
    for (i = 0; i < e; ++i)
        for (j = i + 1; j < e; ++j)
            if (lost[i] > lost[j]) { int t = lost[i]; lost[i] = lost[j]; lost[j] = t; }
    /* surviving data rows in ascending order (rs.c:528-542): row i of rs->m when `full` is
     * given (the n x k matrix the handle carries), else the unit row */
    for (i = 0; i < k; ++i) {
        if (x < e && lost[x] == i) { ++x; continue; }
        if (full) {
            memcpy(mat + rows * k, full + (size_t)i * k, (size_t)k);
        } else {
            memset(mat + rows * k, 0, (size_t)k);
            mat[rows * k + i] = 1;
        }
        in[rows++] = data[i];
    }
    /* then the chosen parity rows (rs.c:544-551): rs->m row k + fixr[i] */
    for (i = 0; i < e && rows < k; ++i) {
        memcpy(mat + rows * k, full ? full + (size_t)(k + fixr[i]) * k : parity_rows + fixr[i] * k, (size_t)k);
        in[rows++] = fixp[i];
    }
    if (rows < k) { free(mat); free(in); free(out); return -1; }
    orc_invert(mat, k); /* return value ignored, as in rs.c:556 */
    for (i = 0; i < e; ++i) {
        out[i] = data[lost[i]];
        memmove(mat + i * k, mat + lost[i] * k, (size_t)k);
    }
    rs_apply(mat, in, out, k, e, len);
    free(mat); free(in); free(out);
    return 0;
}

/* reed_solomon_reconstruct(): rs.c:598-643.  marks[0 .. G*k-1] mark data shards,
 * marks[G*k .. G*n-1] parity shards.  Per group the first e non-erased parity rows
 * (ascending) are used (rs.c:620-629); parity is never regenerated.  Returns -1 if
 * any group had fewer usable parity rows than erased data shards. */
static int rs_reconstruct(int k, int m, const u8 *parity_rows, const u8 *full, u8 **shards,
                          const u8 *marks, int nr_shards, int len)
{
    int groups = nr_shards / (k + m), g, i, err = 0;
    int *lost = (int *)malloc(sizeof(int) * (size_t)k);
    int *fixr = (int *)malloc(sizeof(int) * (size_t)m);
    u8 **fixp = (u8 **)malloc(sizeof(u8 *) * (size_t)m);
    orc_init();
    for (g = 0; g < groups; ++g) {
        u8 **data = shards + (size_t)g * k;
        u8 **par = shards + (size_t)groups * k + (size_t)g * m;
        const u8 *dm = marks + (size_t)g * k;
        const u8 *pm = marks + (size_t)groups * k + (size_t)g * m;
        int e = 0, p = 0;
        for (i = 0; i < k; ++i)
            if (dm[i]) lost[e++] = i;
        if (e == 0)
            continue;
        for (i = 0; i < m && p < e; ++i)
            if (!pm[i]) { fixr[p] = i; fixp[p] = par[i]; ++p; }
        if (p == e)
            rs_decode_group(k, parity_rows, full, data, fixp, fixr, lost, e, len);
        else
            err = -1;
    }
    free(lost); free(fixr); free(fixp);
    return err;
}

int orc_rs_reconstruct(int k, int m, const u8 *parity_rows, u8 **shards, const u8 *marks,
                       int nr_shards, int len)
{
    return rs_reconstruct(k, m, parity_rows, NULL, shards, marks, nr_shards, len);
}

/* The same with the handle's whole n x k matrix rs->m, as rs.c reads it (rs.c:505, 536-548):
 * a caller may have edited it (data rows included), and a sub-matrix that is singular then
 * decodes with invert_mat's partial state (its return value is ignored, rs.c:556). */
int orc_rs_reconstruct_full(int k, int m, const u8 *full, u8 **shards, const u8 *marks,
                            int nr_shards, int len)
{
    return rs_reconstruct(k, m, NULL, full, shards, marks, nr_shards, len);
}

/* ------------------------------------------------------------------ fec.c codec */

/* fec_encode(): fec.c:714-733 with addmul1 (fec.c:333-369).  rows = the full n x k
 * systematic matrix.  index < k copies; k <= index < n computes one parity packet;
 * any other index leaves dst untouched (the reference prints an error). */
void orc_fec_encode(int k, int n, const u8 *enc_rows_full, u8 *const *src, u8 *dst, int index, int sz)
{
    int i, b;
    orc_init();
    if (index < 0)
        return; /* reference behaviour undefined (reads enc_matrix[negative]); treated as invalid */
    if (index < k) {
        memcpy(dst, src[index], (size_t)sz);
    } else if (index < n) {
        const u8 *row = enc_rows_full + (size_t)index * k;
        memset(dst, 0, (size_t)sz);
        for (i = 0; i < k; ++i) {
            u8 f = row[i];
            if (!f) continue;
            for (b = 0; b < sz; ++b)
                dst[b] ^= t_mul[f][src[i][b]];
        }
    }
}

/* shuffle(): fec.c:738-771.  Returns 1 on a conflict. */
static int fec_shuffle(u8 **pkt, int *idx, int k)
{
    int i = 0;
    while (i < k) {
        int c = idx[i];
        if (c >= k || c == i) { ++i; continue; }
        if (c < 0)
            return 1; /* undefined in the reference (reads idx[-1]); rejected here */
        if (idx[c] == c)
            return 1;
        idx[i] = idx[c]; idx[c] = c;
        { u8 *t = pkt[i]; pkt[i] = pkt[c]; pkt[c] = t; }
    }
    return 0;
}

/* fec_decode(): fec.c:821-862 with build_decode_matrix (fec.c:778-808).
 * pkt[] and idx[] are permuted in place; recovered data lands in the slots that held
 * parity packets (which keep their parity index).  Returns 0, or 1 on error. */
int orc_fec_decode(int k, int n, const u8 *enc_rows_full, u8 **pkt, int *idx, int sz)
{
    u8 *mat, **fresh;
    int r, c, b;
    orc_init();
    if (k <= 0)
        return 1;
    if (fec_shuffle(pkt, idx, k))
        return 1;
    mat = (u8 *)malloc((size_t)k * (size_t)k);
    for (r = 0; r < k; ++r) {
        if (idx[r] < k) {
            memset(mat + r * k, 0, (size_t)k);
            mat[r * k + r] = 1;
        } else if (idx[r] < n) {
            memcpy(mat + r * k, enc_rows_full + (size_t)idx[r] * k, (size_t)k);
        } else {
            free(mat);
            return 1;
        }
    }
    if (orc_invert(mat, k)) {
        free(mat);
        return 1;
    }
    fresh = (u8 **)calloc((size_t)k, sizeof(u8 *));
    for (r = 0; r < k; ++r) {
        if (idx[r] < k) continue;
        fresh[r] = (u8 *)calloc((size_t)(sz > 0 ? sz : 1), 1);
        for (c = 0; c < k; ++c) {
            u8 f = mat[r * k + c];
            if (!f) continue;
            for (b = 0; b < sz; ++b)
                fresh[r][b] ^= t_mul[f][pkt[c][b]];
        }
    }
    for (r = 0; r < k; ++r) {
        if (!fresh[r]) continue;
        memcpy(pkt[r], fresh[r], (size_t)sz);
        free(fresh[r]);
    }
    free(fresh);
    free(mat);
    return 0;
}

/* ------------------------------------------------------------------ contiguous batch helpers
 * data[G][k][pitch], parity[G][m][pitch], marks[G*k data | G*m parity] -- the layout of the
 * product's batched device API.  Thin loops over the functions above. */

int orc_rs_encode_contig(int k, int m, const u8 *parity_rows, u8 *data, u8 *parity,
                         long long groups, int len, long long pitch)
{
    long long g;
    int i;
    u8 **in = (u8 **)malloc(sizeof(u8 *) * (size_t)k);
    u8 **out = (u8 **)malloc(sizeof(u8 *) * (size_t)m);
    orc_init();
    for (g = 0; g < groups; ++g) {
        for (i = 0; i < k; ++i) in[i] = data + (g * k + i) * pitch;
        for (i = 0; i < m; ++i) out[i] = parity + (g * m + i) * pitch;
        rs_apply(parity_rows, in, out, k, m, len);
    }
    free(in); free(out);
    return 0;
}

/* fec_encode() for every parity index of every group: parity[g][j] = row k+j. */
int orc_fec_encode_contig(int k, int m, const u8 *parity_rows, u8 *data, u8 *parity,
                          long long groups, int len, long long pitch)
{
    long long g;
    int i, j, b;
    orc_init();
    for (g = 0; g < groups; ++g)
        for (j = 0; j < m; ++j) {
            u8 *dst = parity + (g * m + j) * pitch;
            memset(dst, 0, (size_t)len);
            for (i = 0; i < k; ++i) {
                u8 f = parity_rows[j * k + i];
                const u8 *src = data + (g * k + i) * pitch;
                if (!f) continue;
                for (b = 0; b < len; ++b) dst[b] ^= t_mul[f][src[b]];
            }
        }
    return 0;
}

int orc_rs_reconstruct_contig(int k, int m, const u8 *parity_rows, u8 *data, u8 *parity,
                              const u8 *marks, long long groups, int len, long long pitch)
{
    long long g, n = k + m;
    int i, rc;
    u8 **sh = (u8 **)malloc(sizeof(u8 *) * (size_t)(groups * n));
    for (g = 0; g < groups; ++g) {
        for (i = 0; i < k; ++i) sh[g * k + i] = data + (g * k + i) * pitch;
        for (i = 0; i < m; ++i) sh[groups * k + g * m + i] = parity + (g * m + i) * pitch;
    }
    rc = orc_rs_reconstruct(k, m, parity_rows, sh, marks, (int)(groups * n), len);
    free(sh);
    return rc;
}

int orc_rs_reconstruct_full_contig(int k, int m, const u8 *full, u8 *data, u8 *parity,
                                   const u8 *marks, long long groups, int len, long long pitch)
{
    long long g, n = k + m;
    int i, rc;
    u8 **sh = (u8 **)malloc(sizeof(u8 *) * (size_t)(groups * n));
    for (g = 0; g < groups; ++g) {
        for (i = 0; i < k; ++i) sh[g * k + i] = data + (g * k + i) * pitch;
        for (i = 0; i < m; ++i) sh[groups * k + g * m + i] = parity + (g * m + i) * pitch;
    }
    rc = orc_rs_reconstruct_full(k, m, full, sh, marks, (int)(groups * n), len);
    free(sh);
    return rc;
}

/* The NetFecCodec receive order (network/NetFecCodec.cpp:504-528): per group the first
 * k valid shards in group order (data 0..k-1, then parity k..n-1) go to fec_decode()
 * (network/FecCodecBuf.cpp:204), and recovered data i is read back from slot i
 * (FecCodecBuf.cpp:211-224).  Writes recovered data into the erased data shards, like
 * the rs.c reconstruct.  Returns the number of groups that were not decodable. */
long long orc_fec_reconstruct_contig(int k, int m, const u8 *parity_rows, u8 *data, u8 *parity,
                                     const u8 *marks, long long groups, int len, long long pitch)
{
    int n = k + m, i, v;
    long long g, bad = 0;
    u8 *full = (u8 *)calloc((size_t)n * (size_t)k, 1);
    u8 **slot = (u8 **)malloc(sizeof(u8 *) * (size_t)k);
    u8 **bufs = (u8 **)malloc(sizeof(u8 *) * (size_t)k);
    int *idx = (int *)malloc(sizeof(int) * (size_t)k);
    orc_init();
    for (i = 0; i < k; ++i) full[i * k + i] = 1;
    memcpy(full + (size_t)k * k, parity_rows, (size_t)m * k);
    for (i = 0; i < k; ++i) bufs[i] = (u8 *)malloc((size_t)(len > 0 ? len : 1));
    for (g = 0; g < groups; ++g) {
        const u8 *dm = marks + g * k, *pm = marks + groups * k + g * m;
        int lost = 0, haspar = 0;
        for (i = 0; i < k; ++i) lost += dm[i] ? 1 : 0;
        if (!lost) continue;
        v = 0;
        for (i = 0; i < n && v < k; ++i) {
            int erased = i < k ? dm[i] : pm[i - k];
            const u8 *src = i < k ? data + (g * k + i) * pitch : parity + (g * m + (i - k)) * pitch;
            if (erased) continue;
            memcpy(bufs[v], src, (size_t)len);
            slot[v] = bufs[v];
            idx[v] = i;
            if (i >= k) haspar = 1;
            ++v;
        }
        if (v < k || !haspar || orc_fec_decode(k, n, full, slot, idx, len)) { ++bad; continue; }
        for (i = 0; i < k; ++i)
            if (dm[i]) memcpy(data + (g * k + i) * pitch, slot[i], (size_t)len);
    }
    for (i = 0; i < k; ++i) free(bufs[i]);
    free(full); free(slot); free(bufs); free(idx);
    return bad;
}

/* ------------------------------------------------------------------ shard checksum */
/* icrypt_checksum() (system/imemdata.h:1697-1703): u32 byte sum; FEC keeps the low 16
 * bits (network/FecCodecBuf.cpp:29-61). */
uint32_t orc_byte_sum(const u8 *p, long long len)
{
    uint32_t s = 0;
    long long i;
    for (i = 0; i < len; ++i) s += p[i];
    return s;
}

/* ------------------------------------------------------------------ FEC wire marshalling
 * network/FecCodecBuf.cpp: the shard format the network layer feeds the codec, and the
 * 11-byte (+2 checksum) FEC header on every datagram.  All integers little-endian
 * (iencode16u_lsb / iencode32u_lsb, system/imemdata.h:805-870). */

static void put16(u8 *p, unsigned v) { p[0] = (u8)v; p[1] = (u8)(v >> 8); }
static void put32(u8 *p, uint32_t v) { p[0] = (u8)v; p[1] = (u8)(v >> 8); p[2] = (u8)(v >> 16); p[3] = (u8)(v >> 24); }
static unsigned get16(const u8 *p) { return (unsigned)p[0] | ((unsigned)p[1] << 8); }
static uint32_t get32(const u8 *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }

/* set_fec_enc_buf() (FecCodecBuf.cpp:66-103): shard = [size][cksum16(payload) if checksum]
 * [payload], zero-filled to cap bytes.  Returns en_size = size + 2 or + 4. */
int orc_build_shard(const u8 *payload, int size, int checksum, u8 *shard, int cap)
{
    int head = checksum ? 4 : 2;
    memset(shard, 0, (size_t)cap);
    put16(shard, (unsigned)size);
    if (checksum)
        put16(shard + 2, orc_byte_sum(payload, size) & 0xFFFF);
    memcpy(shard + head, payload, (size_t)size);
    return size + head;
}

/* pack_fec_head() (FecCodecBuf.cpp:274-328): [tag 0xEC | 0xED][sent u32][src u32]
 * [ikn u16 = n | k << 4 | ik << 8][cksum16(buf) if checksum][buf].  Returns the length. */
int orc_pack_head(uint32_t sent, uint32_t src, int n, int k, int ik, int checksum, const u8 *buf, int len, u8 *out)
{
    int off = 0;
    unsigned ikn = ((unsigned)n | ((unsigned)k << 4) | ((unsigned)ik << 8)) & 0xFFFF;
    out[off++] = checksum ? 0xED : 0xEC;
    put32(out + off, sent); off += 4;
    put32(out + off, src); off += 4;
    put16(out + off, ikn); off += 2;
    if (checksum) { put16(out + off, orc_byte_sum(buf, len) & 0xFFFF); off += 2; }
    memcpy(out + off, buf, (size_t)len);
    return off + len;
}

/* unpack_fec_head() (FecCodecBuf.cpp:334-411).  Returns 1 for an FEC datagram (fields and
 * the shard bytes [0, *shard_len) written out), 0 for a non-FEC datagram (tag not EC/ED, or
 * shorter than 11 bytes: payload = dgram + 1), -1 when the shard checksum fails (the
 * network layer drops the datagram, NetFecCodec.cpp:210-213).  is_checksum receives
 * whether the tag carried a checksum (it also governs dec_src_pkt_info's check). */
int orc_unpack_head(const u8 *d, int len, uint32_t *sent, uint32_t *src, int *n, int *k, int *ik,
                    int *is_checksum, u8 *shard, int *shard_len)
{
    unsigned ikn;
    int off = 11;
    if (len < 1 || (d[0] != 0xEC && d[0] != 0xED) || len < 11)
        return 0;
    *is_checksum = d[0] == 0xED;
    *sent = get32(d + 1);
    *src = get32(d + 5);
    ikn = get16(d + 9);
    *n = (int)(ikn & 0xF);
    *k = (int)((ikn >> 4) & 0xF);
    *ik = (int)((ikn >> 8) & 0xF);
    if (*is_checksum) {
        /* rm_checksum (FecCodecBuf.cpp:42-61) over the bytes after the checksum */
        unsigned want = get16(d + off);
        if ((orc_byte_sum(d + off + 2, len - off - 2) & 0xFFFF) != want)
            return -1;
        off += 2;
    }
    *shard_len = len - off;
    memcpy(shard, d + off, (size_t)(len - off));
    return 1;
}

/* dec_src_pkt_info() (FecCodecBuf.cpp:109-133): returns the payload offset in the shard (2
 * or 4) and its size, or -1 for a size >= dec_pkt_size or a checksum mismatch. */
int orc_dec_src(const u8 *shard, int dec_pkt_size, int checksum, int *size)
{
    unsigned sz = get16(shard);
    *size = (int)sz;
    if ((int)sz >= dec_pkt_size)
        return -1;
    if (checksum) {
        if ((orc_byte_sum(shard + 4, sz) & 0xFFFF) != get16(shard + 2))
            return -1;
        return 4;
    }
    return 2;
}

/* One full group through the send path of zfec_pack_input (NetFecCodec.cpp:96-172):
 * k source datagrams (sent0 + i, src0 + i), then n - k check datagrams (sent0 + k + j,
 * src0 + k - 1) whose shards are fec_encode(.., k + j, groupMax).  rows_full is the n x k
 * fec.c matrix.  out: n datagrams at stride out_pitch, lengths in out_len.  Returns groupMax. */
int orc_pack_group(int k, int n, const u8 *rows_full, const u8 *payload, const long long *offs, const int *sizes,
                   uint32_t sent0, uint32_t src0, int checksum, int shard_cap, u8 *out, long long out_pitch,
                   int *out_len)
{
    u8 *shards = (u8 *)calloc((size_t)k * (size_t)shard_cap, 1);
    u8 **src = (u8 **)malloc(sizeof(u8 *) * (size_t)k);
    u8 *par = (u8 *)calloc((size_t)shard_cap, 1);
    int i, j, gmax = 0;
    orc_init();
    for (i = 0; i < k; ++i) {
        int en = orc_build_shard(payload + offs[i], sizes[i], checksum, shards + (size_t)i * shard_cap, shard_cap);
        src[i] = shards + (size_t)i * shard_cap;
        gmax = i == 0 ? en : (en > gmax ? en : gmax);
        out_len[i] = orc_pack_head(sent0 + (uint32_t)i, src0 + (uint32_t)i, n, k, i, checksum, src[i], en,
                                   out + (size_t)i * out_pitch);
    }
    for (j = k; j < n; ++j) {
        orc_fec_encode(k, n, rows_full, src, par, j, gmax);
        out_len[j] = orc_pack_head(sent0 + (uint32_t)j, src0 + (uint32_t)k - 1, n, k, j, checksum, par, gmax,
                                   out + (size_t)j * out_pitch);
    }
    free(shards); free(src); free(par);
    return gmax;
}

/* ---------------------------------------------------------------- ProtocolUdp framing
 * Restated from network/ProtocolBasic.cpp (which does not build here: ../system/option.h is
 * absent from the reference tree), so this part of the oracle is PARITY UNPINNED: no
 * reference output exists to check it against.
 *   CheckSum2 / CheckSum (ProtocolBasic.cpp:65-87): s = byte sum; ~((s >> 16) + (s & 0xffff))
 *   SendPacket (:111-150): push protocol, push (cmd & 0x1f) | 0xA0, push CheckSum & 0xff,
 *                           XOR everything with mask ^ gmask ^ 0x5a, push mask
 *   Session::PacketOutput (SessionDesc.cpp:69-77): push hid, push conv (u32 LE) first. */
static uint32_t udp_checksum(const u8 *p, int n)
{
    uint32_t s = 0;
    int i;
    for (i = 0; i < n; ++i) s += p[i];
    s = (s >> 16) + (s & 0xffffu);
    return ~s;
}

/* returns the framed length; out holds at least len + 12 bytes */
int orc_frame_udp(const u8 *data, int len, int mask, int gmask, int cmd, int protocol, int session, uint32_t conv,
                  uint32_t hid, u8 *out)
{
    int P = session ? 12 : 4, i;
    u8 x = (u8)((mask ^ gmask ^ 0x5a) & 0xff);
    out[2] = (u8)((cmd & 0x1f) | 0xa0);
    out[3] = (u8)protocol;
    if (session) {
        for (i = 0; i < 4; ++i) {
            out[4 + i] = (u8)(conv >> (8 * i));
            out[8 + i] = (u8)(hid >> (8 * i));
        }
    }
    memcpy(out + P, data, (size_t)len);
    out[1] = (u8)(udp_checksum(out + 2, P - 2 + len) & 0xff);
    for (i = 1; i < P + len; ++i) out[i] ^= x;
    out[0] = (u8)mask;
    return P + len;
}

/* RecvPacket (:152-210).  Returns 0 ok, 1 short, 2 checksum, 3 cmd; the un-XORed frame goes
 * to work (len bytes); info = xor mask, check, cmd & 0x1f, protocol */
int orc_unframe_udp(const u8 *frame, int len, int gmask, int session, u8 *work, u8 *info)
{
    int P = session ? 12 : 4, i;
    u8 x;
    uint32_t c;
    if (len < P) return 1;
    x = (u8)((frame[0] ^ gmask ^ 0x5a) & 0xff);
    work[0] = frame[0];
    for (i = 1; i < len; ++i) work[i] = frame[i] ^ x;
    c = udp_checksum(work + 2, len - 2) & 0xff;
    info[0] = x;
    info[1] = work[1];
    info[2] = (u8)(work[2] & 0x1f);
    info[3] = work[3];
    if (c != work[1]) return 2;
    if ((work[2] & 0xe0) != 0xa0) return 3;
    return 0;
}
