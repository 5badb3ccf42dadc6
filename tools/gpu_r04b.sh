#!/bin/bash
# Round 4, second pass: all GPU tests, config-4 A/B (round-2 build against HEAD in alternating
# processes; reconstruct impl 8 against 9 in one process), the receive's skip-lost knob, bench.
#   gpurun --timeout 1200 -- bash tools/gpu_r04b.sh
set -o pipefail
OUT=gpurun_out/r04b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/pytest.log | head -30; exit $rc; }
C4="--k 16 --m 4 --block 1400 --groups 250000 --erasures 4 --rounds 6 --reps 5"
for i in 1 2 3; do
  for n in r02 head; do
    echo "== $n ($i)" >> $OUT/ab_lib.txt
    QFEC_LIB=$PWD/tools/_abl/libqfec_$n.so timeout -k 10 120 python tools/ab.py $C4 \
      --only "encode_impl0,probe,recon_auto" >> $OUT/ab_lib.txt 2>&1 || { tail $OUT/ab_lib.txt; exit 5; }
  done
done
grep -E "==|median" $OUT/ab_lib.txt
timeout -k 10 200 python tools/ab.py $C4 --only "encode_impl0,encode_impl2,probe,recon_auto,recon_impl8" > $OUT/ab_c4.txt 2>&1 || { tail $OUT/ab_c4.txt; exit 6; }
cat $OUT/ab_c4.txt
timeout -k 10 200 python tools/ab.py --rounds 6 --reps 5 --only "encode_impl0,encode_impl2,probe,recon_auto,recon_impl8" > $OUT/ab_c1.txt 2>&1 || { tail $OUT/ab_c1.txt; exit 7; }
cat $OUT/ab_c1.txt
timeout -k 10 200 python tools/wire_ab.py --unpack --wire-align 64 --rounds 5 --variants "base;wire_rx_skip_lost=1" > $OUT/ab_rx.txt 2>&1 || { tail $OUT/ab_rx.txt; exit 8; }
cat $OUT/ab_rx.txt
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 9; }
cat $OUT/bench.json
