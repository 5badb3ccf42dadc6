#!/bin/bash
# Per-call server: its tests, then traced per-call times with inputs in device / host memory.
#   gpurun --timeout 600 -- bash tools/gpu_percall_modes.sh TAG
set -o pipefail
bash tools/gpu_percall.sh ${1:-percall_modes} || exit 2
for v in "percall_resident=1,percall_in=0" "percall_resident=1,percall_in=1"; do
  QFEC_PERCALL_TRACE=1 timeout -k 10 200 python tools/percall_ab.py --variants "$v" --rounds 2 2>&1 | grep -v amdgpu.ids || exit 3
done
