#!/bin/bash
# round 5: qfec_zfec_unpack_input per datagram with the huge-page arenas, against a bare copy loop
set -o pipefail
OUT=gpurun_out/${1:-r05ac}; mkdir -p $OUT
source tools/gpu_step.sh
step input_ub 120 tools/_build/zfec_input_ub
cat $OUT/input_ub.log
