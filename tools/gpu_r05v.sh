#!/bin/bash
# round 5: zfec phase times on the final sources, and three plain runs
set -o pipefail
OUT=gpurun_out/${1:-r05v}; mkdir -p $OUT
source tools/gpu_step.sh
QFEC_ZFEC_TIMING=1 step zfec_timing 200 python tools/zfec_rate.py --reps 3
for i in 1 2 3; do step zfec_$i 200 python tools/zfec_rate.py --json; done
grep -h "rep 5\|zfec flush" $OUT/zfec_timing.log | tail -19
for i in 1 2 3; do python3 -c "
import json; d=json.loads(open('$OUT/zfec_$i.log').read().strip().splitlines()[-1]); e=d['e2e']
print(d['send_e2e_gibs'], d['recv_e2e_gibs'], e['pack_inputs_s'], e['send_flush_s'], e['unpack_inputs_s'], e['recv_flush_s'])"; done
