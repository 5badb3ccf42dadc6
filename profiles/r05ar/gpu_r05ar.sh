#!/bin/bash
# round 5 (temporary env switches, not kept): reconstruct at mild residency caps; the datagram
# and frame sends compiled for one more wave per SIMD
set -o pipefail
OUT=gpurun_out/${1:-r05ar}; mkdir -p $OUT
source tools/gpu_step.sh
step rlds 300 env QFEC_LIB=tools/_tmplib/libqfec_env.so QFEC_LIB_COMPAT=1 python tools/_rlds_tmp.py  # now profiles/r05ar/rlds_ab.py
step txwv 300 env QFEC_LIB=tools/_tmplib/libqfec_env.so QFEC_LIB_COMPAT=1 python tools/_txwv_tmp.py  # now profiles/r05ar/txwv_ab.py
cat $OUT/rlds.log $OUT/txwv.log
