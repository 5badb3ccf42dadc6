#!/bin/bash
# per-call: group inputs copied while the device computes (ov) against the straight-line build (pcnew)
set -o pipefail
T=${1:-r04q}; OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread -k "per_packet or percall or group" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
bash tools/ab_lib.sh "python -u tools/percall_ab.py --variants percall_resident=1 --rounds 3 --reps 2000" pcnew ov > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 3; }
grep -v amdgpu.ids $OUT/ab.txt
