#!/bin/bash
# per-call server stage times with every request served twice (QFEC_PERCALL_TRACE=2): is the
# compute stage cold-start (instruction fetch after the acquire's invalidate) or the multiply?
set -o pipefail
T=${1:-r04k}; OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
for tr in 1 2; do for sp in 0 1; do
  QFEC_PERCALL_TRACE=$tr timeout -k 10 120 python -u tools/percall_ab.py --variants "percall_split=$sp" --rounds 1 --reps 1000 > $OUT/trace${tr}_split$sp.txt 2>&1 || { tail -20 $OUT/trace${tr}_split$sp.txt; exit 5; }
  echo "trace $tr:"; grep -v amdgpu.ids $OUT/trace${tr}_split$sp.txt
done; done
