#!/bin/bash
# round 5: zfec receive after the false-sharing fix and per-session dedup; callback prefetch distance A/B
set -o pipefail
OUT=gpurun_out/${1:-r05i}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 300 python -u -m pytest tests/test_gpu_zfec.py -x -q --timeout 120 --timeout-method thread
QFEC_ZFEC_TIMING=1 step zfec_timing 200 python tools/zfec_rate.py --reps 3
for a in 3 0 6 10; do
  QFEC_ZFEC_AHEAD=$a step zfec_a$a 200 python tools/zfec_rate.py --reps 4
done
QFEC_ZFEC_RX_THREADS=12 step zfec_t12 200 python tools/zfec_rate.py --reps 4
grep -h "rep \|zfec flush" $OUT/zfec_timing.log | tail -18
for f in a3 a0 a6 a10 t12; do echo "== $f"; grep -h "end to end" $OUT/zfec_$f.log | cut -c1-200; done
