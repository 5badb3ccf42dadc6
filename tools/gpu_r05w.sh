#!/bin/bash
# round 5: zfec arenas as registered 2 MiB-page mappings (QFEC_ZFEC_THP=1) against hipHostMalloc,
# alternating processes; the box's THP setting first
set -o pipefail
OUT=gpurun_out/${1:-r05w}; mkdir -p $OUT
source tools/gpu_step.sh
cat /sys/kernel/mm/transparent_hugepage/enabled > $OUT/thp.txt 2>&1
step tests 300 python -u -m pytest tests/test_gpu_zfec.py -x -q --timeout 120 --timeout-method thread
QFEC_ZFEC_THP=1 step tests_thp 300 python -u -m pytest tests/test_gpu_zfec.py -x -q --timeout 120 --timeout-method thread
for i in 1 2 3; do
  for t in 0 1; do
    QFEC_ZFEC_THP=$t step z_t${t}_$i 200 python tools/zfec_rate.py --json
    python3 -c "
import json; d=json.loads(open('$OUT/z_t${t}_$i.log').read().strip().splitlines()[-1]); e=d['e2e']
print('thp$t', d['send_e2e_gibs'], d['recv_e2e_gibs'], e['pack_inputs_s'], e['send_flush_s'], e['unpack_inputs_s'], e['recv_flush_s'], d['verified'])" | tee -a $OUT/summary.txt
  done
done
cat $OUT/thp.txt
