#!/bin/bash
# SQ instruction/wait counters of the 8-B-lane reconstruct at two shapes (one rocprofv3 --pmc pass each).
#   gpurun --timeout 600 -- bash tools/gpu_recon_pmc.sh tag
set -o pipefail
OUT=gpurun_out/${1:-recon_pmc}; mkdir -p $OUT
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for shape in "--k 16 --m 4 --block 1400 --erasures 4" "--k 10 --m 3 --block 1024 --erasures 3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD \
    --output-format csv -d $R/$OUT/a$i -o p -- python3 $R/tools/ab.py --recon8 --rounds 1 --reps 2 $shape > $R/$OUT/a$i.log 2>&1 || { tail -5 $R/$OUT/a$i.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY \
    --output-format csv -d $R/$OUT/b$i -o p -- python3 $R/tools/ab.py --recon8 --rounds 1 --reps 2 $shape > $R/$OUT/b$i.log 2>&1 || { tail -5 $R/$OUT/b$i.log; exit 1; }
done
find $R/$OUT -name "*.csv" | head
