#!/bin/bash
# Where the config-4 reconstruct's wave time goes: SQ busy / wait / issue counters and the
# SMEM / VMEM outstanding-level counters (average latency = LEVEL / INSTS), RS(16,4) B=1400 and
# RS(10,3) B=1400, auto reconstruct only.  One rocprofv3 --pmc pass per counter set.
#   gpurun --timeout 900 -- bash tools/gpu_r04f.sh tag
set -o pipefail
OUT=gpurun_out/${1:-r04f}; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for shape in "--k 16 --m 4 --block 1400 --erasures 4" "--k 10 --m 3 --block 1400 --erasures 3"; do
  i=$((i+1))
  j=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD" \
             "SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY" \
             "SQ_WAVES SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_VMEM_WR"; do
    j=$((j+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/p${i}_$j -o p -- \
      python3 $R/tools/ab.py --only recon_auto --rounds 1 --reps 2 $shape > $R/$OUT/p${i}_$j.log 2>&1 \
      || { echo "pass $i/$j failed"; tail -5 $R/$OUT/p${i}_$j.log; [ $j -eq 3 ] || exit 1; }
  done
done
find $R/$OUT -name "*counter_collection.csv" | head -20
