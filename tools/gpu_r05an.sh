#!/bin/bash
# round 5: the encode's auto residency cap (encode_lds -1) against none (0), over every
# templated shape, the XOR probe beside it (r05an: also the GPU suite and a bench line)
set -o pipefail
OUT=gpurun_out/${1:-r05an}; mkdir -p $OUT
source tools/gpu_step.sh
step occ 500 python tools/occ_ab.py --rounds 5 --probe --lds=-1,0,40960,65536 --shapes "10,3,1024;16,4,1400;2,1,1024;3,2,1024;5,3,1024;6,2,1024;7,1,1024;8,2,1024;4,2,1400;10,3,64;16,4,256"
cat $OUT/occ.log



