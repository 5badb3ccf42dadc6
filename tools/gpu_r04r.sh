#!/bin/bash
# per-call server: tables from a per-wave LDS copy (percall_lds 1) vs v_readlane
set -o pipefail
T=${1:-r04r}; OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u - > $OUT/lds_parity.txt 2>&1 <<'PY' || { tail -30 $OUT/lds_parity.txt; exit 3; }
import sys
import quicknet_amd as qa
qa.tune("percall_lds", 1)
import pytest
sys.exit(pytest.main(["-x", "-q", "-m", "gpu", "--timeout", "120", "--timeout-method", "thread", "-k", "per_packet or percall or group or abi or fec_",
                      "-p", "no:cacheprovider", "tests/test_gpu_host.py", "tests/test_gpu_parity.py"]))
PY
tail -1 $OUT/lds_parity.txt
timeout -k 10 300 python -u tools/percall_ab.py --ref --variants "percall_lds=0;percall_lds=1" --rounds 6 --reps 2000 > $OUT/percall_ab.txt 2>&1 || { tail -20 $OUT/percall_ab.txt; exit 4; }
grep -v amdgpu.ids $OUT/percall_ab.txt
for u in 0 1; do
  QFEC_PERCALL_TRACE=1 timeout -k 10 120 python -u tools/percall_ab.py --variants "percall_lds=$u" --rounds 1 --reps 1000 > $OUT/trace_lds$u.txt 2>&1 || { tail -20 $OUT/trace_lds$u.txt; exit 5; }
  grep -v amdgpu.ids $OUT/trace_lds$u.txt
done
