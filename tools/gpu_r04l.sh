#!/bin/bash
# per-call server: the compute stage with and without its output stores (QFEC_PERCALL_TRACE=3)
set -o pipefail
T=${1:-r04l}; OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
for tr in 1 2 3; do
  QFEC_PERCALL_TRACE=$tr timeout -k 10 120 python -u tools/percall_ab.py --variants "percall_split=0" --rounds 1 --reps 1000 > $OUT/trace${tr}.txt 2>&1 || { tail -20 $OUT/trace${tr}.txt; exit 5; }
  echo "trace $tr:"; grep -v amdgpu.ids $OUT/trace${tr}.txt
done
