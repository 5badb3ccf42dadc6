#!/bin/bash
# round 5: rs.h host path with pointer classification by mapping; zfec receive (pooled session
# threads, per-session grouping, callback prefetch) phase times and thread count; unpack_input cost
set -o pipefail
OUT=gpurun_out/${1:-r05h}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 400 python -u -m pytest tests/test_gpu_rs_host.py tests/test_gpu_zfec.py -x -q --timeout 120 --timeout-method thread
export QFEC_RS_TRACE=1
step rs_default 200 python tools/rs_abi_rate.py --reps 2
step rs_t8_c3000 200 python tools/rs_abi_rate.py --reps 2 --threads 8 --chunk 3000
unset QFEC_RS_TRACE
step input_ub 120 tools/_build/zfec_input_ub
for th in 8 12 16; do
  QFEC_ZFEC_RX_THREADS=$th QFEC_ZFEC_TIMING=1 step zfec_t$th 200 python tools/zfec_rate.py --reps 3
done
step zfec_plain 200 python tools/zfec_rate.py --reps 4
grep -h "value\|\[qfec\]" $OUT/rs_*.log | cut -c1-240
cat $OUT/input_ub.log
for th in 8 12 16; do echo "== $th"; grep -h "rep \|zfec flush" $OUT/zfec_t$th.log | tail -18; done
grep -h "rep " $OUT/zfec_plain.log
