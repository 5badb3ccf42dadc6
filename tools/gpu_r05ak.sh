#!/bin/bash
# round 5: encode / reconstruct against a cap on waves per CU (tools/occ_ab.py)
set -o pipefail
OUT=gpurun_out/${1:-r05ak}; mkdir -p $OUT
source tools/gpu_step.sh
step occ_ab 400 python tools/occ_ab.py
cat $OUT/occ_ab.log
step occ_ab_big 200 python tools/occ_ab.py --rounds 4 --lds 0,163840
cat $OUT/occ_ab_big.log
