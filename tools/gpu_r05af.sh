#!/bin/bash
# round 5: rs.h host pipeline, zero copy (kernels read the pinned slot over PCIe) against staged
# (DMA engine H2D / D2H through the slot's device buffer), alternating processes
set -o pipefail
OUT=gpurun_out/${1:-r05af}; mkdir -p $OUT
source tools/gpu_step.sh
export QFEC_RS_TRACE=1
for i in 1 2 3; do
  for z in 1 0; do
    step rs_zc${z}_$i 200 python tools/rs_abi_rate.py --reps 3 --zero-copy $z
    python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/rs_zc${z}_$i.log') if l.startswith('{')][-1]
print('zc$z', d['value'], d['encode_gibs'], d['reconstruct_gibs'], d['verified'])" | tee -a $OUT/summary.txt
  done
done
grep -h "\[qfec\]" $OUT/rs_zc0_3.log | tail -2 | cut -c1-200
grep -h "\[qfec\]" $OUT/rs_zc1_3.log | tail -2 | cut -c1-200
