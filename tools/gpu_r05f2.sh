#!/bin/bash
# round 5 closing pass on the final sources (kernel sources as r05y, whose PMC traffic the line
# carries): GPU suite, smoke, the bench line, rocprof of the bench step
set -o pipefail
TAG=${1:-r05final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
echo "== pytest -m gpu" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 2; }
tail -1 $OUT/pytest_gpu.log
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
echo "== bench" && timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 4; }
echo "== rocprofv3 kernel trace (bench step + config 4)" && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $R/$OUT/prof -o trace -- python3 $R/bench.py --no-cpu --no-host --no-side > $R/$OUT/bench_prof.json 2> $R/$OUT/prof.err) || { tail -20 $OUT/prof.err; exit 5; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
python3 - <<PY
import json
d=json.loads(open("$OUT/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["roofline"]["frac"], d["roofline"]["traffic_source"])
print("config4", d["config4"]["rank0_encode_frac"], d["config4"]["rank0_reconstruct_frac"])
print("wire", d["wire"]["pack_frac"], d["wire"]["unpack_frac"], d["wire"]["framed"]["pack_frames_frac"], d["wire"]["framed"]["unpack_frames_frac"])
print("rs_abi_host", d["rs_abi_host"]["value"], d["rs_abi_host"]["vs_cpu_threads"], d["rs_abi_host"]["verified"])
print("zfec", d["zfec"]["send_e2e_gibs"], d["zfec"]["recv_e2e_gibs"], d["zfec"]["verified"])
PY
echo done
