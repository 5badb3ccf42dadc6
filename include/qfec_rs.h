/*
 * qfec_rs.h -- drop-in for the reference's batched Cauchy Reed-Solomon codec.
 *
 * Replaces module/rs.h:1-58 of skywind3000/QuickNet (implementation module/rs.c) with the
 * same C ABI, exported by libqfec.so.  Arithmetic runs in HIP kernels on an MI355X
 * (quicknet_amd/csrc/qfec_kernels.hip); shard pointers may be host or device memory.
 *
 * Semantics kept bit-exact with module/rs.c:
 *   - parity rows P[j][i] = inverse[(m + i) ^ j]                  (rs.c:437-440)
 *   - shards[0 .. G*k-1] are all data shards (group-major), shards[G*k .. G*n-1] all
 *     parity shards; marks[] uses the same layout                 (rs.c:578-586, :609-612)
 *   - reconstruct uses, per group, the surviving data shards in ascending order and the
 *     first e non-erased parity rows in ascending order; parity is never regenerated,
 *     returns -1 when any group is under-determined                (rs.c:598-643)
 *   - a zero coefficient in column 0 leaves the output's previous bytes in place
 *     (mul() memsets 0 bytes, rs.c:116-117)
 *   - the public matrices may be edited between calls and are re-read on every call, each
 *     where rs.c reads it: encode multiplies by `parity` (rs.c:583); reconstruct builds its
 *     k x k sub-matrix from the rows of `m` (data rows included, rs.c:505, 536-548), so the
 *     two are independent copies, as in rs.c (:431-442).  A sub-matrix that an edit made
 *     singular is decoded with invert_mat's partially eliminated state and does not change
 *     the return value: rs.c ignores invert_mat's result (rs.c:556)
 *   - reed_solomon_new() errors: 1 bad shape, 2..5 allocation     (rs.c:404-476)
 */
#ifndef QFEC_RS_H
#define QFEC_RS_H

/* use small value to save memory (rs.h:5) */
#define DATA_SHARDS_MAX 255

/* rs.h:7-13 -- public layout kept; the library allocates a larger private object whose
 * first member is this struct. */
typedef struct _reed_solomon {
    int data_shards;
    int parity_shards;
    int shards;
    unsigned char *m;      /* n x k: identity on top, parity rows below (reconstruct reads it) */
    unsigned char *parity; /* m x k parity rows (encode reads it)                             */
} reed_solomon;

#ifdef __cplusplus
extern "C" {
#endif

/* rs.h:22 / rs.c:382 -- builds the field tables; the device context is created lazily on
 * the first encode/reconstruct, once, thread-safely. */
void reed_solomon_init(void);

/* rs.h:24 / rs.c:387 */
reed_solomon *reed_solomon_new(int data_shards, int parity_shards);

/* rs.h:25 / rs.c:478 */
void reed_solomon_release(reed_solomon *rs);

/* rs.h:34 / rs.c:574 -- G = nr_shards / (k + m) groups of block_size bytes. Returns 0 on
 * success, as rs.c always does.  A device failure (no HIP device, a failed launch or copy)
 * returns the negative QFEC_E* code of include/qfec.h instead -- a deviation: rs.c has no
 * device that can fail -- and is also reported on stderr and by qfec_last_error().
 * shards[] may mix host and device pointers; each pointer is classified on its own. */
int reed_solomon_encode(reed_solomon *rs, unsigned char **shards, int nr_shards, int block_size);

/* rs.h:44 / rs.c:598 -- erased data shards are rewritten in place. Returns 0, or -1 if
 * any group had more erased data shards than surviving parity shards (such groups are left
 * untouched, as in rs.c), or a negative QFEC_E* code (< -1) on a device failure. */
int reed_solomon_reconstruct(reed_solomon *rs, unsigned char **shards, unsigned char *marks,
                             int nr_shards, int block_size);

/* rs.h:49 / rs.c:649 */
int reed_solomon_error(void);

#ifdef __cplusplus
}
#endif

#endif /* QFEC_RS_H */
