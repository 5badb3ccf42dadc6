#!/bin/bash
# round 5: the whole GPU suite twice in one process each (flakiness check) and smoke
set -o pipefail
OUT=gpurun_out/${1:-r05ah}; mkdir -p $OUT
source tools/gpu_step.sh
step suite1 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step suite2 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:randomly
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $OUT/suite1.log $OUT/suite2.log
