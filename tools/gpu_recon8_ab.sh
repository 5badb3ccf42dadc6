#!/bin/bash
# 8-B-lane reconstruct A/B (full vs partial last 64-B line) after the reconstruct parity tests.
#   gpurun --timeout 900 -- bash tools/gpu_recon8_ab.sh tag
set -o pipefail
OUT=gpurun_out/${1:-recon8_ab}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "reconstruct" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for shape in "--k 16 --m 4 --block 1400 --erasures 4" "--k 10 --m 3 --block 1400 --erasures 3" "--k 16 --m 4 --block 1024 --erasures 4" "--k 10 --m 3 --block 1012 --erasures 3"; do
  timeout -k 10 300 python tools/ab.py --recon8 $shape > $OUT/ab.tmp 2>&1 || { tail $OUT/ab.tmp; exit 2; }
  grep -v amdgpu.ids $OUT/ab.tmp | tee -a $OUT/ab.txt
done
