#!/bin/bash
# round 5: rs.h host pipeline with the encode staged (reconstruct in place): tests and rate
set -o pipefail
OUT=gpurun_out/${1:-r05ag}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 400 python -u -m pytest tests/test_gpu_rs_host.py -x -q --timeout 120 --timeout-method thread
export QFEC_RS_TRACE=1
for i in 1 2 3; do
  step rs_$i 200 python tools/rs_abi_rate.py --reps 3
  python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/rs_$i.log') if l.startswith('{')][-1]
print('staged-encode', d['value'], d['encode_gibs'], d['reconstruct_gibs'], d['verified'])" | tee -a $OUT/summary.txt
done
grep -h "\[qfec\]" $OUT/rs_3.log | tail -2 | cut -c1-200
