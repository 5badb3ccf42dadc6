#!/bin/bash
# Instruction mix per kernel (one rocprofv3 --pmc pass, SQ counters only) of a command.
#   bash tools/pmc_insts.sh OUTDIR -- python3 tools/wire_ab.py --unpack --variants base --rounds 1 --reps 2
set -o pipefail
OUT=$1; shift; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM \
  --output-format csv -d $GRAFT_REPO_ROOT/$OUT -o p -- "$@" > $GRAFT_REPO_ROOT/$OUT/run.log 2>&1
