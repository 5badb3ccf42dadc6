#!/bin/bash
# SQ counters (issue / wait split, instruction mix) of the wire leg's kernels, two rocprofv3 --pmc
# passes over tools/side_legs.py, plus the default bench line first.
#   gpurun --timeout 900 -- bash tools/gpu_sq_side.sh TAG [--no-bench]
set -o pipefail
TAG=${1:-sq}
OUT=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "--no-bench" ]; then
  echo "== bench"
  timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
  tail -c 1500 $OUT/bench.json
fi
cd /tmp
j=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU"; do
  j=$((j+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/sq$j -o p -- \
    python3 $R/tools/side_legs.py --steps 10 --warmup 3 > $R/$OUT/sq$j.log 2>&1 \
    || { echo "pass $j failed"; tail -5 $R/$OUT/sq$j.log; exit 3; }
done
python3 $R/tools/sq_summary.py $R/$OUT/sq1 $R/$OUT/sq2 | tee $R/$OUT/sq_summary.txt
