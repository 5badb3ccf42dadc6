#!/bin/bash
# round 5: AVX2 arena copies against memcpy for the zfec input calls, alternating processes
set -o pipefail
OUT=gpurun_out/${1:-r05ae}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 300 python -u -m pytest tests/test_gpu_zfec.py -x -q --timeout 120 --timeout-method thread
step input_ub 120 tools/_build/zfec_input_ub
for i in 1 2 3; do
  for n in zbase znew; do
    QFEC_LIB=$PWD/tools/_build/libqfec_$n.so step z_${n}_$i 200 python tools/zfec_rate.py --json
    python3 -c "
import json; d=json.loads(open('$OUT/z_${n}_$i.log').read().strip().splitlines()[-1]); e=d['e2e']
print('$n', d['send_e2e_gibs'], d['recv_e2e_gibs'], e['pack_inputs_s'], e['send_flush_s'], e['unpack_inputs_s'], e['recv_flush_s'], d['verified'])" | tee -a $OUT/summary.txt
  done
done
grep "unpack_input" $OUT/input_ub.log | tail -2
