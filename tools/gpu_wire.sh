#!/bin/bash
# Datagram-path measurement (one gpurun call): wire GPU tests, wire_bench at 1 KiB and 1400 B
# with the reference CPU pipeline beside it, rocprofv3 kernel-trace stats of the 1 KiB run,
# and the interleaved A/B of both directions.
#   gpurun --timeout 900 -- bash tools/gpu_wire.sh r01q
set -o pipefail
TAG=${1:-wire}
OUT=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
export TMPDIR=/tmp
echo "== wire tests" && timeout -k 10 600 python -m pytest tests/test_gpu_wire.py tests/test_gpu_frame.py tests/test_gpu_net.py -x -q > $OUT/pytest_wire.log 2>&1 || { tail -30 $OUT/pytest_wire.log; exit 2; }
tail -1 $OUT/pytest_wire.log
echo "== wire_bench" && for s in 1024 1400; do timeout -k 10 300 python tools/wire_bench.py --size $s --cpu-seconds 8 >> $OUT/wire_bench.jsonl 2>> $OUT/wire_bench.err || { tail -20 $OUT/wire_bench.err; exit 3; }; done
cat $OUT/wire_bench.jsonl
echo "== rocprofv3" && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $R/$OUT/prof -o trace -- python3 $R/tools/wire_bench.py --cpu-seconds 0 > $R/$OUT/wire_prof.json 2> $R/$OUT/wire_prof.err) || { tail -20 $OUT/wire_prof.err; exit 4; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/wire_kernel_stats.csv \;
cut -d, -f1-4 $OUT/wire_kernel_stats.csv | head -8
echo "== A/B" && timeout -k 10 300 python tools/wire_ab.py > $OUT/wire_ab.txt 2>&1 && timeout -k 10 300 python tools/wire_ab.py --unpack --variants "base;wire_rx=3;wire_rx=0" >> $OUT/wire_ab.txt 2>&1 || { tail -20 $OUT/wire_ab.txt; exit 5; }
cat $OUT/wire_ab.txt
echo done
