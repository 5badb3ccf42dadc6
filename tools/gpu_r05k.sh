#!/bin/bash
# round 5: full GPU suite; zfec receive with the early arena copies (phase times, then plain reps)
set -o pipefail
OUT=gpurun_out/${1:-r05k}; mkdir -p $OUT
source tools/gpu_step.sh
step full_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
QFEC_ZFEC_TIMING=1 step zfec_timing 200 python tools/zfec_rate.py --reps 3
for i in 1 2 3; do
  step zfec_plain$i 200 python tools/zfec_rate.py --reps 4
done
grep -h "rep 5\|zfec flush" $OUT/zfec_timing.log | tail -18
grep -h "end to end" $OUT/zfec_plain*.log | cut -c1-200
