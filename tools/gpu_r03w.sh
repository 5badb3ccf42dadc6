#!/bin/bash
# doorbell probe (fresh inputs) + RS(16,4) B=1400 reconstruct lanes A/B at config 4's shape
set -o pipefail
OUT=gpurun_out/${1:-r03w}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 60 tools/_build/doorbell_probe > $OUT/probe.txt 2>&1; cat $OUT/probe.txt
timeout -k 10 300 python tools/ab.py --rounds 8 --only "probe,recon_impl3_partial,recon_impl4,recon_impl2" --k 16 --m 4 --block 1400 --erasures 4 --groups 250000 > $OUT/ab.tmp 2>&1 || { tail $OUT/ab.tmp; exit 5; }
grep -v amdgpu.ids $OUT/ab.tmp | tee $OUT/ab.txt
