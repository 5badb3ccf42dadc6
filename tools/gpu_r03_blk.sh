#!/bin/bash
# reconstruct IMPL 8 (one group per block): parity for every body, then A/B at config 4's shape and the headline's
set -o pipefail
OUT=gpurun_out/${1:-r03_blk}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "reconstruct" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for shape in "--k 16 --m 4 --block 1400 --erasures 4 --groups 250000" "--k 10 --m 3 --block 1024 --erasures 3"; do
  timeout -k 10 300 python tools/ab.py --rounds 8 --only "probe,recon_impl3_partial,recon_impl3_(,recon_impl8" $shape > $OUT/ab.tmp 2>&1 || { tail $OUT/ab.tmp; exit 2; }
  grep -v amdgpu.ids $OUT/ab.tmp | tee -a $OUT/ab.txt
done
