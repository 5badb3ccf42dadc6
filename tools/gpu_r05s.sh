#!/bin/bash
# round 5: rs.h host-path tests after the maps-read threshold
set -o pipefail
OUT=gpurun_out/${1:-r05s}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 400 python -u -m pytest tests/test_gpu_rs_host.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "rs_ or abi or quirk or edits"
export QFEC_RS_TRACE=1
step rs_default 200 python tools/rs_abi_rate.py --reps 2
grep -h "\[qfec\]\|value" $OUT/rs_default.log | tail -3 | cut -c1-220
