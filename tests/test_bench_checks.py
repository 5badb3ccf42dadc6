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


def test_config4_traffic_scaled_per_rank(tmp_path):
    """At N > 1 a rank's share of config 4 has no PMC entry of its own: the whole batch's entry
    (taken at N = 1) is scaled by the rank's share of the groups and says so; a rank whose group
    count has its own entry takes it as is; a stale or missing whole-batch entry gives none."""
    import json
    h = bench.kernel_sources_hash()
    path = tmp_path / "traffic.json"
    full = {"kernel_sources_sha256": h, "run": "rX", "encode_bytes_per_launch": 7.0e9,
            "reconstruct_bytes_per_launch": 6.8e9}
    path.write_text(json.dumps({"rs16_4_b1400_g250000_e4": full,
                                "rs16_4_b1400_g125000_e4": dict(full, encode_bytes_per_launch=3.6e9)}))
    tr, src = bench.config4_traffic(str(path), 16, 4, 1400, 250000, 250000, 4)
    assert tr["encode_bytes_per_launch"] == 7.0e9 and not src.startswith("scaled")
    tr, src = bench.config4_traffic(str(path), 16, 4, 1400, 125000, 250000, 4)
    assert tr["encode_bytes_per_launch"] == 3.6e9 and not src.startswith("scaled")
    tr, src = bench.config4_traffic(str(path), 16, 4, 1400, 31250, 250000, 4)
    assert abs(tr["encode_bytes_per_launch"] - 7.0e9 / 8) < 1 and abs(tr["reconstruct_bytes_per_launch"] - 6.8e9 / 8) < 1
    assert src.startswith("scaled by 31250/250000 groups from")
    path.write_text(json.dumps({"rs16_4_b1400_g250000_e4": dict(full, kernel_sources_sha256="stale")}))
    tr, src = bench.config4_traffic(str(path), 16, 4, 1400, 31250, 250000, 4)
    assert tr is None and src == "no entry for this workload"
