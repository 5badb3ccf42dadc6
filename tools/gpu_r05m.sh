#!/bin/bash
# round 5: the LDS-staged reconstruct (recon_impl 10) -- parity, then interleaved A/B against the
# auto body (impl 8) at config 4 (RS(16,4) B=1400, 250 000 groups) and at RS(10,3) B=1024
set -o pipefail
OUT=gpurun_out/${1:-r05m}; mkdir -p $OUT
source tools/gpu_step.sh
step parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "reconstruct"
step ab_c4 300 python tools/ab.py --k 16 --m 4 --block 1400 --groups 250000 --rounds 12 --reps 10 --only "recon_impl8,recon_impl10,probe"
step ab_h 300 python tools/ab.py --k 10 --m 3 --block 1024 --groups 100000 --rounds 12 --reps 10 --only "recon_impl8,recon_impl10,probe"
tail -8 $OUT/ab_c4.log; tail -8 $OUT/ab_h.log
