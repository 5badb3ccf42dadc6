#!/bin/bash
# round 5: zfec receive after request dedup and parallel scratch teardown; prefetch distance with phase times
set -o pipefail
OUT=gpurun_out/${1:-r05j}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 300 python -u -m pytest tests/test_gpu_zfec.py -x -q --timeout 120 --timeout-method thread
for a in 3 6 10; do
  QFEC_ZFEC_AHEAD=$a QFEC_ZFEC_TIMING=1 step zfec_ta$a 200 python tools/zfec_rate.py --reps 3
done
for a in 3 6 10 3 6 10; do
  QFEC_ZFEC_AHEAD=$a step zfec_a$a 200 python tools/zfec_rate.py --reps 4
  grep -h "end to end" $OUT/zfec_a$a.log | tail -3 | cut -c1-200 >> $OUT/ahead_summary.txt
done
for a in 3 6 10; do echo "== $a"; grep -h "rep 5\|zfec flush" $OUT/zfec_ta$a.log | tail -18; done
cat $OUT/ahead_summary.txt
