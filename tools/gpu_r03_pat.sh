#!/bin/bash
# RS(16,4) B=1400 reconstruct at config 4's 250 000 groups against the number of distinct erasure
# patterns (all 4 844, 500, 50): how much of the gap to the XOR probe is the pattern tables' cache.
set -o pipefail
OUT=gpurun_out/${1:-r03_pat}; mkdir -p $OUT; export TMPDIR=/tmp
for p in 0 500 50; do
  timeout -k 10 200 python tools/ab.py --rounds 6 --only "probe,recon_impl3_partial" --k 16 --m 4 --block 1400 --erasures 4 --groups 250000 --patterns $p > $OUT/ab.tmp 2>&1 || { tail $OUT/ab.tmp; exit 5; }
  echo "== patterns $p" | tee -a $OUT/ab.txt; grep -v amdgpu.ids $OUT/ab.tmp | tee -a $OUT/ab.txt
done
