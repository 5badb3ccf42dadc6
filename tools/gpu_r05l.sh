#!/bin/bash
# round 5: zfec receive, early arena copies A/B (0 off, 1 on, 2 lagging one step), interleaved
set -o pipefail
OUT=gpurun_out/${1:-r05l}; mkdir -p $OUT
source tools/gpu_step.sh
for i in 1 2 3; do
  for e in 0 1 2; do
    QFEC_ZFEC_EARLY=$e step zfec_e${e}_$i 200 python tools/zfec_rate.py --reps 4
    grep -h "end to end" $OUT/zfec_e${e}_$i.log | tail -3 | sed "s/^/e$e /" | cut -c1-190 >> $OUT/summary.txt
  done
done
sort $OUT/summary.txt
