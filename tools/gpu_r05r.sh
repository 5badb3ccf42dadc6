#!/bin/bash
# round 5: send kernel with one payload mask for equal-size rows -- wire / frame tests, then
# alternating processes against the previous build (tools/ab_lib.sh form) on the wire side leg
set -o pipefail
OUT=gpurun_out/${1:-r05r}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 400 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_frames_fused.py tests/test_gpu_net.py -x -q --timeout 120 --timeout-method thread
for i in 1 2 3; do
  for n in txbase txnew; do
    QFEC_LIB=$PWD/tools/_abl/libqfec_$n.so step side_${n}_$i 200 python tools/side_legs.py --steps 50
    python3 -c "
import json,sys
d=json.loads(open('$OUT/side_${n}_$i.log').read().strip().splitlines()[-1])
f=d['framed']
print('$n', d['pack_avg_ms'], d['pack_frac'], d['unpack_avg_ms'], f['pack_frames_avg_ms'], f['pack_frames_frac'], d['verified'], f['verified'])" | tee -a $OUT/summary.txt
  done
done
