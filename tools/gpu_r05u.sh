#!/bin/bash
# round 5: the rs.h host path against the reference rs.c itself
set -o pipefail
OUT=gpurun_out/${1:-r05u}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 400 python -u -m pytest tests/test_gpu_rs_host.py tests/test_gpu_host.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "reference"
tail -12 $OUT/tests.log
