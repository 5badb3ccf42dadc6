#!/bin/bash
# recon impl 9 (persistent grid) parity + interleaved A/B against the auto choice
set -o pipefail
OUT=gpurun_out/${1:-r04g}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "impl" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for shape in "--k 16 --m 4 --block 1400 --erasures 4 --groups 200000" "--k 10 --m 3 --block 1400 --erasures 3 --groups 200000" "--k 10 --m 3 --block 1024 --erasures 3 --groups 200000"; do
  timeout -k 10 200 python -u tools/ab.py --only recon_auto,recon_impl9 --rounds 10 --reps 5 $shape >> $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
done
cat $OUT/ab.txt | grep -v amdgpu.ids
