#!/bin/bash
# round 5: where a module/rs.h host-pointer call spends its time outside the pipeline (pointer
# classification), and which mappings hold device / pinned / pageable pointers
set -o pipefail
OUT=gpurun_out/${1:-r05g}; mkdir -p $OUT
source tools/gpu_step.sh
step maps 120 python tools/maps_probe.py
export QFEC_RS_TRACE=1
step rs_t8_c3000 200 python tools/rs_abi_rate.py --reps 2 --threads 8 --chunk 3000
step rs_default 200 python tools/rs_abi_rate.py --reps 2
cat $OUT/maps.log
grep -h "value\|\[qfec\]" $OUT/rs_*.log | cut -c1-260
QFEC_ZFEC_TIMING=1 step zfec_timing 200 python tools/zfec_rate.py --reps 3
grep -h "rep \|zfec flush" $OUT/zfec_timing.log | tail -40
QFEC_ZFEC_NT=1 QFEC_ZFEC_TIMING=1 step zfec_timing_nt 200 python tools/zfec_rate.py --reps 3
grep -h "rep " $OUT/zfec_timing_nt.log | tail -6
