#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 PMC counters (MI355X_MICROARCH.md, HBM section).

Two separate counter passes over the same bench workload (FETCH_SIZE and WRITE_SIZE do not
fit one pass on gfx950), each its own `rocprofv3 --pmc` run with no tracing domains.
Corrections per the guide: FETCH_SIZE reads exactly half the bytes of a wide coalesced
streaming read on gfx950, so reads = 2 * FETCH_SIZE; WRITE_SIZE is exact for 16-B/lane
streaming stores.  Both counters are in KiB.  The XOR probe kernel (known bytes) is
profiled in the same run as a calibration check.

Writes profiles/traffic.json (read by bench.py as roofline.traffic) and the raw CSVs to
the output directory.  Run on the GPU box:
    python tools/pmc_traffic.py --out gpurun_out/pmc
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"encode": "k_encode_perm<{k}, {m},", "reconstruct": "k_reconstruct_perm<{k}, {m},", "probe": "k_probe_xor"}
# --workload wire: bench.py's `wire` leg (tools/side_legs.py), RS(10,13) 1 KiB payloads
WIRE_KERNELS = {"pack": "k_pack_wave64<10, 3, 1, 0, 1, 16, 0>", "unpack": "k_rx<10, 3, 4, false, true>",
                "pack_frames": "k_pack_wave64<10, 3, 1, 4, 1, 16, 0>", "unpack_frames": "k_rx<10, 3, 4, true, true>"}


def run_pass(counter, out, bench_args, k, m, kernels=KERNELS, script="bench.py"):
    d = os.path.abspath(os.path.join(out, counter.lower()))
    os.makedirs(d, exist_ok=True)
    extra = ["--no-cpu"] if script == "bench.py" else []
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", counter.lower(), "--",
           sys.executable, os.path.join(ROOT, script)] + extra + bench_args
    env = dict(os.environ, TMPDIR="/tmp")
    with open(os.path.join(d, "run.log"), "w") as log:
        subprocess.run(cmd, check=True, stdout=log, stderr=subprocess.STDOUT, env=env, cwd="/tmp", timeout=600)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise RuntimeError(f"no counter_collection.csv under {d}")
    per = {k: [] for k in kernels}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                for key, pat in kernels.items():
                    if pat.format(k=k, m=m) in name:
                        per[key].append(float(row["Counter_Value"]))
    return per


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    p.add_argument("--json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--m", type=int, default=3)
    p.add_argument("--block", type=int, default=1024)
    p.add_argument("--groups", type=int, default=100_000)
    p.add_argument("--erasures", type=int, default=3, help="erasures per group (bench.py --erasures); key suffix _eN "
                                                           "when not 3 (config 4: 4, read by bench.py's config4 field)")
    p.add_argument("--tag", default="PMC run", help="which run produced the numbers (recorded in the JSON)")
    p.add_argument("--workload", choices=["headline", "wire", "config4"], default="headline",
                   help="headline: bench.py's timed step; config4: its RS(16,4) config 4 leg alone (key "
                        "rs16_4_b1400_g<G>_e4, read by the line's config4 field); wire: the datagram leg")
    p.add_argument("--csv-home", default=None,
                   help="where the counter CSVs are kept in the repository (default profiles/<tag>/pmc): recorded "
                        "in the JSON so the bench line names tracked files whether or not they travel to the box")
    a = p.parse_args()
    if a.workload == "wire":
        return wire_main(a)
    if a.workload == "config4":
        return config4_main(a)
    bench_args = ["--steps", "5", "--warmup", "1", "--k", str(a.k), "--m", str(a.m), "--block", str(a.block),
                  "--groups", str(a.groups), "--erasures", str(a.erasures), "--no-side", "--no-config4", "--no-host"]
    fetch = run_pass("FETCH_SIZE", a.out, bench_args, a.k, a.m)
    write = run_pass("WRITE_SIZE", a.out, bench_args, a.k, a.m)
    k, m, B, G = a.k, a.m, a.block, a.groups
    probe_alg_read, probe_alg_write = k * B * G, m * B * G
    res = {}
    for key in KERNELS:
        if not fetch[key] or not write[key]:
            continue
        f = sum(fetch[key]) / len(fetch[key])
        w = sum(write[key]) / len(write[key])
        res[key] = {"fetch_kib_raw": f, "write_kib_raw": w, "read_bytes": 2 * f * 1024, "write_bytes": w * 1024,
                    "bytes_per_launch": 2 * f * 1024 + w * 1024, "launches": len(fetch[key])}
    if "probe" in res:
        res["probe"]["algorithmic_read"] = probe_alg_read
        res["probe"]["algorithmic_write"] = probe_alg_write
    key = f"rs{k}_{m}_b{B}_g{G}" + (f"_e{a.erasures}" if a.erasures != 3 else "")
    doc = {}
    if os.path.exists(a.json):
        with open(a.json) as fh:
            doc = json.load(fh)
    sys.path.insert(0, ROOT)
    from bench import kernel_sources_hash
    doc[key] = {
        "kernel_sources_sha256": kernel_sources_hash(),  # bench.py ignores the entry once the kernels change
        "run": a.tag,
        "encode_bytes_per_launch": res.get("encode", {}).get("bytes_per_launch"),
        "reconstruct_bytes_per_launch": res.get("reconstruct", {}).get("bytes_per_launch"),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; bytes = 2*FETCH_SIZE*1024 "
                  "+ WRITE_SIZE*1024 (gfx950 corrections, MI355X_MICROARCH.md HBM section)",
        "raw": res,
        "csv": a.csv_home or f"profiles/{a.tag}/pmc",
    }
    os.makedirs(os.path.dirname(a.json), exist_ok=True)
    with open(a.json, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc[key], indent=1))


def config4_main(a):
    """PMC bytes per launch of bench.py's config 4 leg (RS(16,4) 1400 B, 4 erasures, --config4-groups
    groups on one rank): its encode (inputs in halves) and reconstruct (8-B lanes, one group per block)."""
    G = a.groups
    kernels = {"encode": "k_encode_perm_halves<16, 4,", "reconstruct": "k_reconstruct_perm<16, 4, 8>"}
    args = ["--config4-only", "--config4-groups", str(G), "--steps", "5", "--warmup", "1"]
    fetch = run_pass("FETCH_SIZE", a.out, args, 16, 4, kernels)
    write = run_pass("WRITE_SIZE", a.out, args, 16, 4, kernels)
    res = {}
    for key in kernels:
        if not fetch[key] or not write[key]:
            print(f"no PMC rows for {kernels[key]}", file=sys.stderr)
            return 1
        f = sum(fetch[key]) / len(fetch[key])
        w = sum(write[key]) / len(write[key])
        res[key] = {"fetch_kib_raw": f, "write_kib_raw": w, "read_bytes": 2 * f * 1024, "write_bytes": w * 1024,
                    "bytes_per_launch": 2 * f * 1024 + w * 1024, "launches": len(fetch[key])}
    doc = {}
    if os.path.exists(a.json):
        with open(a.json) as fh:
            doc = json.load(fh)
    sys.path.insert(0, ROOT)
    from bench import kernel_sources_hash
    key = f"rs16_4_b1400_g{G}_e4"
    doc[key] = {"kernel_sources_sha256": kernel_sources_hash(), "run": a.tag,
                "encode_bytes_per_launch": res["encode"]["bytes_per_launch"],
                "reconstruct_bytes_per_launch": res["reconstruct"]["bytes_per_launch"],
                "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py "
                          "--config4-only; bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 corrections)",
                "raw": res, "csv": a.csv_home or f"profiles/{a.tag}/pmc"}
    with open(a.json, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc[key], indent=1))


def wire_main(a):
    """PMC bytes per launch of the datagram and one-pass frame kernels of bench.py's `wire` leg."""
    args = ["--steps", "20", "--warmup", "2"]
    fetch = run_pass("FETCH_SIZE", a.out, args, 10, 3, WIRE_KERNELS, "tools/side_legs.py")
    write = run_pass("WRITE_SIZE", a.out, args, 10, 3, WIRE_KERNELS, "tools/side_legs.py")
    res = {}
    for key in WIRE_KERNELS:
        if not fetch[key] or not write[key]:
            continue
        f = sum(fetch[key]) / len(fetch[key])
        w = sum(write[key]) / len(write[key])
        res[key] = {"fetch_kib_raw": f, "write_kib_raw": w, "read_bytes": 2 * f * 1024, "write_bytes": w * 1024,
                    "bytes_per_launch": 2 * f * 1024 + w * 1024, "launches": len(fetch[key])}
    missing = [k2 for k2 in WIRE_KERNELS if k2 not in res]
    if missing:  # a kernel renamed (template arguments) without this table following
        print(f"no PMC rows for {missing}: kernel names {[WIRE_KERNELS[k2] for k2 in missing]} not found", file=sys.stderr)
        return 1
    doc = {}
    if os.path.exists(a.json):
        with open(a.json) as fh:
            doc = json.load(fh)
    sys.path.insert(0, ROOT)
    from bench import WIRE_KERNEL_SOURCES, kernel_sources_hash
    key = "wire_rs10_13_s1024_g100000"
    doc[key] = {"kernel_sources_sha256": kernel_sources_hash(WIRE_KERNEL_SOURCES), "run": a.tag,
                "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over tools/side_legs.py; "
                          "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 corrections)",
                "raw": res, "csv": a.csv_home or f"profiles/{a.tag}/pmc"}
    for k2, v in res.items():
        doc[key][k2] = v["bytes_per_launch"]
    with open(a.json, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc[key], indent=1))


if __name__ == "__main__":
    sys.exit(main())
