#!/bin/bash
# round 5: encode against a cap on waves per CU over more (k, m) shapes
set -o pipefail
OUT=gpurun_out/${1:-r05am}; mkdir -p $OUT
source tools/gpu_step.sh
step occ 500 python tools/occ_ab.py --rounds 5 --encode-only --lds 0,27000,40960,54272,65536 --shapes "4,2,1024;8,4,1024;12,4,1024;20,4,1024;10,3,1400;16,4,1024;10,3,512;10,3,1024;16,4,1400"
cat $OUT/occ.log
