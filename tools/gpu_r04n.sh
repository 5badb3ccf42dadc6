#!/bin/bash
# per-call server with straight-line bodies per exact row count: parity, then before/after A/B
set -o pipefail
T=${1:-r04n}; OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "per_packet or percall or group or abi or fec_" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
bash tools/ab_lib.sh "python -u tools/percall_ab.py --variants percall_resident=1 --rounds 3 --reps 2000" pcold pcnew > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 3; }
grep -v amdgpu.ids $OUT/ab.txt
QFEC_PERCALL_TRACE=1 timeout -k 10 120 python -u tools/percall_ab.py --ref --variants "percall_resident=1" --rounds 1 --reps 1000 > $OUT/trace.txt 2>&1 || { tail -20 $OUT/trace.txt; exit 5; }
grep -v amdgpu.ids $OUT/trace.txt
