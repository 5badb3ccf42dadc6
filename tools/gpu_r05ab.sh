#!/bin/bash
# round 5: does allocation churn cost the zfec flush? the same runs with glibc keeping freed
# memory (no mmap'd blocks, no trimming) against the default, alternating processes
set -o pipefail
OUT=gpurun_out/${1:-r05ab}; mkdir -p $OUT
source tools/gpu_step.sh
for i in 1 2 3; do
  step z_def_$i 200 python tools/zfec_rate.py --json
  GLIBC_TUNABLES=glibc.malloc.mmap_threshold=4294967295:glibc.malloc.trim_threshold=4294967295 step z_keep_$i 200 python tools/zfec_rate.py --json
done
for f in $OUT/z_*.log; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); e=d['e2e']
print('$(basename $f)', d['send_e2e_gibs'], d['recv_e2e_gibs'], e['pack_inputs_s'], e['send_flush_s'], e['unpack_inputs_s'], e['recv_flush_s'])"; done | tee $OUT/summary.txt
