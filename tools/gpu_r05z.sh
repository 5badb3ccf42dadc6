#!/bin/bash
# round 5: rs.h host pipeline with 2 MiB-page registered slots (QFEC_RS_THP=1) against
# hipHostMalloc slots, alternating processes; the rs host tests in the new mode
set -o pipefail
OUT=gpurun_out/${1:-r05z}; mkdir -p $OUT
source tools/gpu_step.sh
QFEC_RS_THP=1 step tests_thp 300 python -u -m pytest tests/test_gpu_rs_host.py tests/test_gpu_zfec.py -x -q --timeout 120 --timeout-method thread
export QFEC_RS_TRACE=1
for i in 1 2 3; do
  for t in 0 1; do
    QFEC_RS_THP=$t step rs_t${t}_$i 200 python tools/rs_abi_rate.py --reps 3
    python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/rs_t${t}_$i.log') if l.startswith('{')][-1]
print('thp$t', d['value'], d['encode_gibs'], d['reconstruct_gibs'], d['verified'])" | tee -a $OUT/summary.txt
  done
done
grep -h "\[qfec\]" $OUT/rs_t1_3.log | tail -2 | cut -c1-200
grep -h "\[qfec\]" $OUT/rs_t0_3.log | tail -2 | cut -c1-200
