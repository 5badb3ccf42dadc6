#!/bin/bash
# round 5: streaming rate at several read:write mixes (the wire kernels' memory ceilings)
set -o pipefail
OUT=gpurun_out/${1:-r05ai}; mkdir -p $OUT
source tools/gpu_step.sh
step mix 200 python tools/mix_probe.py
step mix2 200 python tools/mix_probe.py
cat $OUT/mix.log $OUT/mix2.log | grep read
