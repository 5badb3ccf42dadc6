#!/bin/bash
# round 5: per-stage SQ counters of the datagram send (k_pack_wave64): two --pmc passes over the wire
# side leg for the full build and for each stage-ablation build (tools/tx_stage_ablate.sh)
set -o pipefail
OUT=gpurun_out/${1:-r05q}
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in full tx1 tx2 tx4 tx8; do
  if [ $v = full ]; then unset QFEC_LIB; else export QFEC_LIB=$R/tools/_abl/libqfec_$v.so; fi
  j=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
             "SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU"; do
    j=$((j+1))
    timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/$v/sq$j -o p -- \
      python3 $R/tools/side_legs.py --steps 10 --warmup 3 > $R/$OUT/$v/sq$j.log 2>&1 \
      || { echo "$v pass $j failed"; tail -5 $R/$OUT/$v/sq$j.log; exit 3; }
  done
  python3 $R/tools/sq_summary.py $R/$OUT/$v/sq1 $R/$OUT/$v/sq2 > $R/$OUT/$v/sq_summary.txt
  echo "== $v"; grep -A16 "k_pack_wave64<10, 3, 1, 0, 1, 16, 0>" $R/$OUT/$v/sq_summary.txt | grep -E "INSTS_VALU|INSTS_SALU|INSTS_SMEM|INSTS_LDS|VMEM|WAVE_CYCLES|WAIT_ANY|dispatches"
done
