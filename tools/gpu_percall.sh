#!/bin/bash
# Per-call path: its GPU tests, then the spin / stream-sync A/B.
#   gpurun --timeout 600 -- bash tools/gpu_percall.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-percall}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -m gpu -x -v --timeout 120 --timeout-method thread -k "per_packet or percall" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 2; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python tools/percall_ab.py > $OUT/percall_ab.txt 2>&1 || { tail -20 $OUT/percall_ab.txt; exit 3; }
grep -v amdgpu.ids $OUT/percall_ab.txt
