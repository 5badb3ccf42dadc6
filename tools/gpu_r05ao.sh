#!/bin/bash
# round 5 pass after the encode residency cap and the new reconstruct instances (one gpurun call): GPU suite, smoke, PMC traffic of the headline and
# the wire leg (-> profiles/traffic.json, copied back as $OUT/traffic.json), bench line (reads
# that traffic), rocprofv3 kernel-trace stats of the bench step and of the wire leg, 2-rank
# gloo rehearsal.   gpurun --timeout 1200 -- bash tools/gpu_r05ao.sh r05ao
set -o pipefail
TAG=${1:-r05ao}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(rocminfo 2>/dev/null | grep -m1 -E "Name:\s+gfx" ; lscpu | grep -E "Model name|^CPU\(s\)") > $OUT/host.txt
echo "== pytest -m gpu" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 2; }
tail -1 $OUT/pytest_gpu.log
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
echo "== PMC traffic, headline" && timeout -k 10 400 python tools/pmc_traffic.py --out $OUT/pmc --json profiles/traffic.json --tag $TAG --csv-home profiles/$TAG/pmc > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 6; }
echo "== PMC traffic, wire leg" && timeout -k 10 400 python tools/pmc_traffic.py --workload wire --out $OUT/pmc_wire --json profiles/traffic.json --tag $TAG --csv-home profiles/$TAG/pmc_wire > $OUT/pmc_wire.log 2>&1 || { tail -20 $OUT/pmc_wire.log; exit 6; }
cp profiles/traffic.json $OUT/traffic.json
echo "== bench" && timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 4; }
tail -c 600 $OUT/bench.json
echo "== rocprofv3 kernel trace (bench step + config 4)" && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $R/$OUT/prof -o trace -- python3 $R/bench.py --no-cpu --no-host --no-side > $R/$OUT/bench_prof.json 2> $R/$OUT/prof.err) || { tail -20 $OUT/prof.err; exit 5; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cut -d, -f1-4 $OUT/kernel_stats.csv | head -6
echo "== rocprofv3 kernel trace (wire leg)" && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_wire -o run -- \
  python3 $R/tools/side_legs.py --steps 100 > $R/$OUT/side_prof.json 2> $R/$OUT/side_prof.err) || { tail -20 $OUT/side_prof.err; exit 8; }
find $OUT/prof_wire -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_wire.csv \;
cut -d, -f1-4 $OUT/kernel_stats_wire.csv | head -8 | cut -c1-150
echo "== bench --gpus 2 (gloo rehearsal)" && QFEC_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --no-cpu > $OUT/bench_g2.json 2> $OUT/bench_g2.err || { tail -20 $OUT/bench_g2.err; exit 7; }
cut -c1-300 $OUT/bench_g2.json
echo "== reconstruct of the newly templated shapes, encode caps" && timeout -k 10 300 python tools/occ_ab.py --rounds 3 --probe --lds=-1,0 --shapes "5,3,1024;6,2,1024;7,1,1024;8,2,1024;20,4,1024" > $OUT/occ.log 2>&1 || { tail -20 $OUT/occ.log; exit 9; }
cat $OUT/occ.log
echo done
