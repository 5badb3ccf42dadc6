#!/bin/bash
# reconstruct with s_setprio 1 until the survivor loads are out (prio) vs the r04m build (base)
set -o pipefail
T=${1:-r04s}; OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "recon or rs_" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
for shape in "--k 16 --m 4 --block 1400 --erasures 4 --groups 250000" "--k 10 --m 3 --block 1024 --erasures 3 --groups 100000"; do
  bash tools/ab_lib.sh "python -u tools/ab.py --only recon_auto --rounds 8 --reps 5 $shape" base prio >> $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 3; }
done
grep -E "==|recon auto|RS\(" $OUT/ab.txt
