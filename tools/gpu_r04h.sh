#!/bin/bash
# before/after builds of the reconstruct (tools/_abl/libqfec_<name>.so), alternating processes
set -o pipefail
OUT=gpurun_out/${1:-r04h}; mkdir -p $OUT; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py -x -q --timeout 120 --timeout-method thread -m gpu -k "recon or decode or rs_" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for shape in "--k 16 --m 4 --block 1400 --erasures 4 --groups 200000" "--k 10 --m 3 --block 1400 --erasures 3 --groups 200000" "--k 10 --m 3 --block 1024 --erasures 3 --groups 200000"; do
  bash tools/ab_lib.sh "python -u tools/ab.py --only recon_auto --rounds 6 --reps 5 $shape" "$@" >> $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
done
grep -E "==|recon auto|RS\(" $OUT/ab.txt
