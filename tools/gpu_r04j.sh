#!/bin/bash
# per-call server: 8-wave split layout (percall_split 1) parity and A/B, with the reference on this CPU
set -o pipefail
T=${1:-r04j}; OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread -k "per_packet or percall or group" > $OUT/pytest_host.log 2>&1 || { tail -30 $OUT/pytest_host.log; exit 2; }
tail -1 $OUT/pytest_host.log
timeout -k 10 300 python -u - > $OUT/split_parity.txt 2>&1 <<'PY' || { tail -30 $OUT/split_parity.txt; exit 3; }
import sys
import quicknet_amd as qa
qa.tune("percall_split", 1)
import pytest
sys.exit(pytest.main(["-x", "-q", "-m", "gpu", "--timeout", "120", "--timeout-method", "thread", "-k", "per_packet or percall or group",
                      "-p", "no:cacheprovider", "tests/test_gpu_host.py", "tests/test_abi.py"]))
PY
tail -1 $OUT/split_parity.txt
timeout -k 10 300 python -u tools/percall_ab.py --ref --variants "percall_split=0;percall_split=1" --rounds 6 --reps 2000 > $OUT/percall_ab.txt 2>&1 || { tail -20 $OUT/percall_ab.txt; exit 4; }
grep -v amdgpu.ids $OUT/percall_ab.txt
for sp in 0 1; do
  QFEC_PERCALL_TRACE=1 timeout -k 10 120 python -u tools/percall_ab.py --variants "percall_split=$sp" --rounds 1 --reps 1000 > $OUT/trace_split$sp.txt 2>&1 || { tail -20 $OUT/trace_split$sp.txt; exit 5; }
  grep -v amdgpu.ids $OUT/trace_split$sp.txt
done
