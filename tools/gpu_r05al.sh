#!/bin/bash
# round 5: fused send / receive against a cap on waves per CU (tx_lds / rx_lds), and the
# encode / reconstruct caps again on a second box
set -o pipefail
OUT=gpurun_out/${1:-r05al}; mkdir -p $OUT
source tools/gpu_step.sh
step tx 300 python tools/wire_ab.py --wire-align 64 --rounds 8 --variants "base;tx_lds=32768;tx_lds=54272;tx_lds=65536;tx_lds=163840"
step rx 300 python tools/wire_ab.py --wire-align 64 --unpack --rounds 8 --variants "base;rx_lds=14900;rx_lds=20480;rx_lds=27000;rx_lds=32768;rx_lds=40960"
step occ 400 python tools/occ_ab.py --rounds 6 --lds 0,40960,54272,65536
cat $OUT/tx.log $OUT/rx.log $OUT/occ.log
