#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Usage (from the repo root, in this container):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
(rocminfo 2>/dev/null | grep -m1 -E "Name:\s+gfx" ; lscpu | grep -E "Model name|^CPU\(s\)") > $OUT/host.txt
echo "== pytest -m gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
echo "== bench" && timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 4; }
cat $OUT/bench.json
echo "== rocprofv3 kernel trace" && cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $GRAFT_REPO_ROOT/$OUT/prof -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $GRAFT_REPO_ROOT/$OUT/bench_prof.json 2> $GRAFT_REPO_ROOT/$OUT/prof.err || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof.err; exit 5; }
cd $GRAFT_REPO_ROOT
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | head -20
echo done
