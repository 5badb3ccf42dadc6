#!/bin/bash
# round 5: streaming rate against waves per CU (tools/occ_probe.hip), built on the box
set -o pipefail
OUT=gpurun_out/${1:-r05aj}; mkdir -p $OUT
source tools/gpu_step.sh
mkdir -p /tmp/occ && hipcc --offload-arch=gfx950 -O3 tools/occ_probe.hip -o /tmp/occ/occ_probe || exit 3
step occ 300 /tmp/occ/occ_probe
cat $OUT/occ.log
