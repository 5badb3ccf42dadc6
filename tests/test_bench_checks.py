"""bench.py's checker for BASELINE config 5 (host_to_host_mixed): sampled groups of the pipe's
output are re-derived with the reference's own module/rs.c (oracle/_ref; the C restatement when
_ref is absent), so the line's `verified` is not a self-comparison.  CPU only."""
import numpy as np

import bench


def _samples(orc, rng):
    out = []
    for k, m, B in ((4, 2, 1024), (10, 3, 1024), (16, 4, 1400)):
        G = 6
        d = rng.integers(0, 256, (G, k, B), dtype=np.uint8)
        p = np.zeros((G, m, B), np.uint8)
        orc.rs_encode(orc.cauchy(k, m), d, p, B)
        md, mp = np.zeros((G, k), np.uint8), np.zeros((G, m), np.uint8)
        for g in range(G):
            for x in rng.choice(k + m, m, replace=False):
                if x < k:
                    md[g, x] = 1
                else:
                    mp[g, x - k] = 1
        out.append(dict(k=k, m=m, B=B, idx=np.arange(G), data=d, parity=p, marks_data=md, marks_parity=mp,
                        restored=d.copy()))
    return out


def test_host_sample_checker(oracle):
    bench._load()
    s = _samples(oracle, np.random.default_rng(5))
    r = bench.cpu_check_host_sample(s)
    assert r["match"] and r["groups_checked"] == 18 and r["mismatched_groups"] == 0
    s[1]["restored"][2, 1, 7] ^= 0x10   # a wrong restored row
    s[2]["parity"][4, 3, 1399] ^= 1     # a wrong parity byte
    r = bench.cpu_check_host_sample(s)
    assert not r["match"] and r["mismatched_groups"] == 2
