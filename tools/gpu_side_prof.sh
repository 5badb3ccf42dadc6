#!/bin/bash
# The wire leg's kernels, reproducibly: event times (tools/side_legs.py), rocprofv3 kernel-trace
# stats of the same command, and PMC FETCH/WRITE passes (traffic.json entry for the wire leg).
#   gpurun --timeout 900 -- bash tools/gpu_side_prof.sh TAG
set -o pipefail
TAG=${1:-side}
OUT=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
export TMPDIR=/tmp
echo "== side legs"
timeout -k 10 200 python tools/side_legs.py --steps 100 > $OUT/side.json 2> $OUT/side.err || { tail -20 $OUT/side.err; exit 2; }
tail -c 3000 $OUT/side.json
echo "== rocprof kernel trace"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/tools/side_legs.py --steps 100 > $R/$OUT/side_prof.json 2> $R/$OUT/side_prof.err) || { tail -20 $OUT/side_prof.err; exit 3; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-200
echo "== PMC"
timeout -k 10 600 python tools/pmc_traffic.py --workload wire --out $OUT/pmc --json $OUT/traffic.json --tag $TAG > $OUT/pmc.log 2>&1 || { tail -30 $OUT/pmc.log; exit 4; }
cat $OUT/pmc.log | head -60
