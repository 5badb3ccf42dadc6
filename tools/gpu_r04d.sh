#!/bin/bash
# Round 4, fourth pass: parity of the new encode / reconstruct bodies, then the config-4 and
# headline A/B of reconstruct impl 9 / 10 (survivors in halves) against the auto choice.
#   gpurun --timeout 900 -- bash tools/gpu_r04d.sh
set -o pipefail
OUT=gpurun_out/r04d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "impls or large or rs_edits" > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/pytest.log | head -30; exit $rc; }
C4="--k 16 --m 4 --block 1400 --groups 250000 --erasures 4 --rounds 8 --reps 5"
for i in 1 2; do
  timeout -k 10 200 python tools/ab.py $C4 --only "encode_auto,encode_impl0,probe,recon_auto,recon_impl4,recon_impl8,recon_impl9,recon_impl10" >> $OUT/ab_c4.txt 2>&1 || { tail $OUT/ab_c4.txt; exit 6; }
done
timeout -k 10 200 python tools/ab.py --rounds 8 --reps 5 --only "encode_auto,probe,recon_auto,recon_impl9,recon_impl10" >> $OUT/ab_c1.txt 2>&1 || { tail $OUT/ab_c1.txt; exit 7; }
timeout -k 10 200 python tools/ab.py --k 10 --m 3 --block 1400 --groups 100000 --rounds 8 --reps 5 --only "encode_auto,recon_auto,recon_impl4,recon_impl9,recon_impl10" >> $OUT/ab_c1400.txt 2>&1 || { tail $OUT/ab_c1400.txt; exit 8; }
grep -E "RS|median" $OUT/ab_c4.txt $OUT/ab_c1.txt $OUT/ab_c1400.txt
