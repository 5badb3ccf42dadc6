#!/bin/bash
# Round 4, first pass: the new parity tests, then config-4 A/B (round-2 build against HEAD in
# alternating processes; reconstruct impl 8 against 9 in one process).
#   gpurun --timeout 1100 -- bash tools/gpu_r04a.sh
set -o pipefail
OUT=gpurun_out/r04a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py tests/test_gpu_frames_fused.py \
  -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/pytest.log | head -30; exit $rc; }
C4="--k 16 --m 4 --block 1400 --groups 250000 --erasures 4 --rounds 6 --reps 5"
for i in 1 2 3; do
  for n in r02 head; do
    echo "== $n ($i)" >> $OUT/ab_lib.txt
    QFEC_LIB=$PWD/tools/_abl/libqfec_$n.so timeout -k 10 120 python tools/ab.py $C4 \
      --only "encode_impl0,probe,recon_auto" >> $OUT/ab_lib.txt 2>&1 || exit 5
  done
done
tail -30 $OUT/ab_lib.txt
timeout -k 10 200 python tools/ab.py $C4 --only "encode_impl0,probe,recon_impl8,recon_impl9,recon_impl3" > $OUT/ab_c4.txt 2>&1 || exit 6
cat $OUT/ab_c4.txt
timeout -k 10 200 python tools/ab.py --rounds 6 --reps 5 --only "encode_impl0,probe,recon_impl8,recon_impl9" > $OUT/ab_c1.txt 2>&1 || exit 7
cat $OUT/ab_c1.txt
