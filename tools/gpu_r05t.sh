#!/bin/bash
# round 5: datagram send / receive of this round's build against round 4's at 512-B, 1 KiB and
# 1400-B (MTU) payloads, alternating processes (tools/wire_ab.py, every output checked)
set -o pipefail
OUT=gpurun_out/${1:-r05t}; mkdir -p $OUT
source tools/gpu_step.sh
for S in 1024 1400 512; do
  for i in 1 2; do
    for n in r04 cur; do
      QFEC_LIB_COMPAT=1 QFEC_LIB=$PWD/tools/_abl/libqfec_$n.so step rx_${S}_${n}_$i 200 python tools/wire_ab.py --size $S --unpack --variants base --wire-align 64 --rounds 3
      QFEC_LIB_COMPAT=1 QFEC_LIB=$PWD/tools/_abl/libqfec_$n.so step tx_${S}_${n}_$i 200 python tools/wire_ab.py --size $S --variants base --wire-align 64 --rounds 3
    done
  done
done
for f in $OUT/rx_* $OUT/tx_*; do echo "$(basename $f): $(grep -h -i "median\|base" $f | tail -1 | cut -c1-150)"; done | tee $OUT/summary.txt
