#!/bin/bash
# round 5: rs.h host pipeline, streaming-store gather (default) against memcpy (QFEC_RS_NT=0),
# alternating processes, with the per-call trace
set -o pipefail
OUT=gpurun_out/${1:-r05o}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 300 python -u -m pytest tests/test_gpu_rs_host.py -x -q --timeout 120 --timeout-method thread
export QFEC_RS_TRACE=1
for i in 1 2 3; do
  for nt in 1 0; do
    QFEC_RS_NT=$nt step rs_nt${nt}_$i 200 python tools/rs_abi_rate.py --reps 3
  done
done
for nt in 1 0; do echo "== NT $nt"; grep -h "value" $OUT/rs_nt${nt}_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['value'], d['encode_gibs'], d['reconstruct_gibs'])"; grep -h "\[qfec\]" $OUT/rs_nt${nt}_1.log | tail -2 | cut -c1-200; done
