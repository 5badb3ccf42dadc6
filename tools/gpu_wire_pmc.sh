#!/bin/bash
# HBM bytes per launch of the datagram kernels: separate --pmc passes (FETCH_SIZE,
# WRITE_SIZE) over tools/wire_bench.py; bytes = 2 * FETCH_SIZE + WRITE_SIZE KiB (gfx950).
#   gpurun --timeout 600 -- bash tools/gpu_wire_pmc.sh tag
set -o pipefail
OUT=gpurun_out/${1:-wire_pmc}; R=$GRAFT_REPO_ROOT; mkdir -p $OUT; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/$OUT/$c -o run -- \
     python3 $R/tools/wire_bench.py --cpu-seconds 0 > $R/$OUT/$c.json 2> $R/$OUT/$c.err) || { tail -20 $OUT/$c.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0][-40:]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        if "qfec" in k:
            kib = sum(v) / len(v)
            mult = 2 if c == "FETCH_SIZE" else 1
            print(f"{c:10s} {k:42s} launches {len(v):3d}  {kib * 1024 * mult / 1e6:10.1f} MB per launch")
PY
