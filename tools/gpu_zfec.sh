#!/bin/bash
# The exact NetFecCodec layer: its GPU tests and its rate with C callbacks.
#   gpurun --timeout 900 -- bash tools/gpu_zfec.sh TAG
set -o pipefail
TAG=${1:-zfec}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest zfec"
timeout -k 10 400 python -u -m pytest tests/test_gpu_zfec.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 2; }
tail -2 $OUT/pytest.log
echo "== rate"
QFEC_ZFEC_TIMING=1 timeout -k 10 300 python tools/zfec_rate.py > $OUT/rate.txt 2>&1 || { tail -40 $OUT/rate.txt; exit 3; }
cat $OUT/rate.txt
timeout -k 10 300 python tools/zfec_rate.py --sorted 1 --reps 2 > $OUT/rate_sorted.txt 2>&1 || { tail -40 $OUT/rate_sorted.txt; exit 4; }
cat $OUT/rate_sorted.txt

