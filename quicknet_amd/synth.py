"""Synthetic shard payloads, reproducible on host and device.

Counter-based splitmix64: 64-bit word j of a stream seeded with ``seed`` is
``splitmix64(seed + (j + 1) * GOLDEN)``, emitted little-endian.  The device mirror is
``qfec_synth_fill`` in ``csrc/qfec_kernels.hip``; tests check the two agree byte for
byte.  Uniform bytes hit GF zero (1/256) often enough to exercise the zero paths.

The seeds used for the BASELINE.json configs are the ones SURVEY.md section 8(d) names
(0x5EED0001 .. 0x5EED0004).
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)

SEED_CPU_ENCODE = 0x5EED0001
SEED_ENCODE = 0x5EED0002
SEED_DECODE = 0x5EED0003
SEED_RS16 = 0x5EED0004


def splitmix_words(seed: int, nwords: int, start: int = 0) -> np.ndarray:
    j = np.arange(start + 1, start + nwords + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + j * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        z = z ^ (z >> np.uint64(31))
    return z


def synth_bytes(seed: int, nbytes: int) -> np.ndarray:
    """``nbytes`` uniform bytes of stream ``seed`` (uint8 array)."""
    nwords = (nbytes + 7) // 8
    w = splitmix_words(seed, nwords).astype("<u8")
    return w.view(np.uint8)[:nbytes].copy()


def erasure_marks(seed: int, groups: int, n: int, erasures: int) -> np.ndarray:
    """Per group, exactly ``erasures`` distinct positions out of ``n`` marked (uint8 [G, n],
    group order data 0..k-1 then parity).  Drawn uniformly from the stream ``seed`` by a
    partial Fisher-Yates shuffle over positions."""
    g = np.arange(groups)
    pos = np.tile(np.arange(n, dtype=np.int64), (groups, 1))
    words = splitmix_words(seed, groups * erasures).reshape(groups, erasures) if erasures else None
    for t in range(erasures):
        r = (words[:, t] % np.uint64(n - t)).astype(np.int64) + t
        a = pos[g, t].copy()
        pos[g, t] = pos[g, r]
        pos[g, r] = a
    marks = np.zeros((groups, n), dtype=np.uint8)
    if erasures:
        np.put_along_axis(marks, pos[:, :erasures], 1, axis=1)
    return marks


def marks_to_rs_layout(marks_gn: np.ndarray, k: int) -> np.ndarray:
    """[G, n] group-order marks -> module/rs.c layout: G*k data marks, then G*m parity marks
    (rs.c:609-612)."""
    return np.concatenate([marks_gn[:, :k].reshape(-1), marks_gn[:, k:].reshape(-1)])
