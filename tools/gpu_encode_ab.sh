#!/bin/bash
# Encode-body A/B on one box: parity for every body, then interleaved timing.
#   gpurun --timeout 900 -- bash tools/gpu_encode_ab.sh tag
set -o pipefail
OUT=gpurun_out/${1:-encode_ab}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "encode_impls" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for shape in "--k 16 --m 4 --block 1400" "--k 10 --m 3 --block 1024"; do
  timeout -k 10 300 python tools/ab.py --encode-only $shape > $OUT/ab.tmp 2>&1 || { tail $OUT/ab.tmp; exit 2; }
  grep -v amdgpu.ids $OUT/ab.tmp | tee -a $OUT/ab.txt
done
