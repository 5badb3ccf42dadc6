#!/bin/bash
# Quick GPU iteration: parity tests, bench (no CPU baseline), optional extra command.
#   gpurun --timeout 900 -- bash tools/gpu_quick.sh tag ["extra command"]
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 4; }
cat $OUT/bench.json
if [ -n "$2" ]; then
  echo "== extra: $2"
  timeout -k 10 600 bash -c "$2" > $OUT/extra.log 2>&1; rc=$?
  cat $OUT/extra.log | tail -60
  exit $rc
fi
