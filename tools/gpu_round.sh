#!/bin/bash
# One gpurun call: GPU tests, the default bench line, and a 2-rank gloo rehearsal of the
# --gpus launcher on the one-GPU box.
#   gpurun --timeout 900 -- bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 2; }
tail -1 $OUT/pytest_gpu.log
echo "== bench (N=1)"
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 3; }
cat $OUT/bench.json
echo "== bench --gpus 2 (gloo rehearsal, ranks share the GPU)"
QFEC_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --no-cpu > $OUT/bench_g2.json 2> $OUT/bench_g2.err || { tail -30 $OUT/bench_g2.err; exit 4; }
cat $OUT/bench_g2.json
