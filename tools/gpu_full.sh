#!/bin/bash
# Full measurement pass (one gpurun call): parity tests, smoke, PMC traffic passes (feed
# bench's roofline.traffic), bench (+CPU baseline), rocprofv3 kernel-trace stats, A/B.
#   gpurun --timeout 1200 -- bash tools/gpu_full.sh r01g
set -o pipefail
TAG=${1:-full}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(rocminfo 2>/dev/null | grep -m1 -E "Name:\s+gfx" ; lscpu | grep -E "Model name|^CPU\(s\)") > $OUT/host.txt
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 2; }
tail -1 $OUT/pytest_gpu.log
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
# bench.py reads roofline.traffic from profiles/traffic.json: the headline entry is updated in
# place (the wire leg's entry, from tools/gpu_side_prof.sh, stays), and a copy comes back in $OUT
echo "== PMC traffic" && timeout -k 10 900 python tools/pmc_traffic.py --out $OUT/pmc --json profiles/traffic.json --tag $TAG > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 6; }
cp profiles/traffic.json $OUT/traffic.json
echo "== bench" && timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 4; }
cat $OUT/bench.json
# only the timed step's launches (and config 4's) under the profiler, so each kernel's average is
# the one bench reports (the host / per-call legs launch the same kernels at other sizes)
echo "== rocprofv3 kernel trace" && (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $R/$OUT/prof -o trace -- python3 $R/bench.py --no-cpu --no-host --no-side > $R/$OUT/bench_prof.json 2> $R/$OUT/prof.err) || { tail -20 $OUT/prof.err; exit 5; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cut -d, -f1-4 $OUT/kernel_stats.csv | head -6
echo "== rocprofv3 kernel trace, datagram kernels (bench's wire leg shapes: RS(10,13) 100k x 1 KiB, wire pitch 1088)" && \
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_wire -o wire -- \
   python3 $R/tools/wire_ab.py --wire-align 64 --variants base --rounds 3 > $R/$OUT/wire_ab_prof.txt 2> $R/$OUT/prof_wire.err && \
   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_wire_rx -o wire -- \
   python3 $R/tools/wire_ab.py --unpack --wire-align 64 --variants base --rounds 3 >> $R/$OUT/wire_ab_prof.txt 2>> $R/$OUT/prof_wire.err) \
  || { tail -20 $OUT/prof_wire.err; exit 8; }
grep -h -E "k_pack|k_unpack" $(find $OUT/prof_wire $OUT/prof_wire_rx -name "*kernel_stats.csv") | cut -d, -f1-4 | cut -c1-120
echo "== bench --gpus 2 (gloo rehearsal: the launcher's own ranks share the one GPU)" && QFEC_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 20 --no-cpu > $OUT/bench_g2.json 2> $OUT/bench_g2.err || { tail -20 $OUT/bench_g2.err; exit 7; }
cut -c1-400 $OUT/bench_g2.json
echo done
