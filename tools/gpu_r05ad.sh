#!/bin/bash
# round 5: one core's copy rate for the unpack_input pattern, three copy forms, two page sizes
set -o pipefail
OUT=gpurun_out/${1:-r05ad}; mkdir -p $OUT
source tools/gpu_step.sh
step copy_ub 120 tools/_build/copy_ub
step copy_ub2 120 tools/_build/copy_ub
cat $OUT/copy_ub.log $OUT/copy_ub2.log
