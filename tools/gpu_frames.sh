#!/bin/bash
# One-pass framing: its parity tests, the wire/frame regression tests, and the rate tool.
#   gpurun --timeout 900 -- bash tools/gpu_frames.sh TAG
set -o pipefail
TAG=${1:-frames}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest frames + wire + frame"
timeout -k 10 600 python -u -m pytest tests/test_gpu_frames_fused.py tests/test_gpu_frame.py tests/test_gpu_wire.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 2; }
tail -2 $OUT/pytest.log
echo "== rate"
timeout -k 10 200 python tools/frames_bench.py > $OUT/rate.txt 2>&1 || { tail -30 $OUT/rate.txt; exit 3; }
cat $OUT/rate.txt
timeout -k 10 200 python tools/frames_bench.py --session --rounds 3 > $OUT/rate_session.txt 2>&1 || { tail -30 $OUT/rate_session.txt; exit 4; }
cat $OUT/rate_session.txt
