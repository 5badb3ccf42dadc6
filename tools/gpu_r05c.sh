#!/bin/bash
# round 5: full GPU suite on the new receive, then the wire leg's SQ counters
set -o pipefail
OUT=gpurun_out/${1:-r05c}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
bash tools/gpu_sq_side.sh ${1:-r05c}/sq --no-bench > $OUT/sq.log 2>&1; echo "sq rc=$?"
grep -A17 "k_rx<10, 3" $OUT/sq/sq_summary.txt | head -40
