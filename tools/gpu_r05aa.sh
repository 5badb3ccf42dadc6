#!/bin/bash
# round 5: rs.h host path and zfec GPU tests after the classifier moved into qfec_maps.hpp
set -o pipefail
OUT=gpurun_out/${1:-r05aa}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 400 python -u -m pytest tests/test_gpu_rs_host.py tests/test_gpu_zfec.py tests/test_gpu_host.py -x -q --timeout 120 --timeout-method thread
tail -2 $OUT/tests.log
