#!/bin/bash
# Round 4, third pass: GPU tests, then encode impl 2 (inputs in halves) against impl 0 at the
# headline and config-4 shapes (interleaved, one process), twice.
#   gpurun --timeout 900 -- bash tools/gpu_r04c.sh
set -o pipefail
OUT=gpurun_out/r04c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/pytest.log | head -30; exit $rc; }
C4="--k 16 --m 4 --block 1400 --groups 250000 --erasures 4 --rounds 8 --reps 5"
for i in 1 2; do
  timeout -k 10 200 python tools/ab.py $C4 --only "encode_impl0,encode_impl2,probe,recon_auto" >> $OUT/ab_c4.txt 2>&1 || { tail $OUT/ab_c4.txt; exit 6; }
  timeout -k 10 200 python tools/ab.py --rounds 8 --reps 5 --only "encode_impl0,encode_impl2,probe,recon_auto" >> $OUT/ab_c1.txt 2>&1 || { tail $OUT/ab_c1.txt; exit 7; }
done
grep -E "RS|median" $OUT/ab_c4.txt $OUT/ab_c1.txt
