#!/bin/bash
# round 5: the encode's residency cap at the per-rank sizes of the strong-scaled config 4
# (250 000 groups over 2, 4, 8 ranks) and at smaller RS(10,3) batches
set -o pipefail
OUT=gpurun_out/${1:-r05ap}; mkdir -p $OUT
source tools/gpu_step.sh
step occ 400 python tools/occ_ab.py --rounds 6 --encode-only --lds=-1,0 --shapes "16,4,1400,125000;16,4,1400,62500;16,4,1400,31250;10,3,1024,50000;10,3,1024,25000;10,3,1024,17000"
cat $OUT/occ.log
