#!/bin/bash
# round 4 follow-ups: VALU issue rate, reconstruct builds A/B (constant-space tables, clean
# offsets), per-call server with ds_bpermute tables
set -o pipefail
T=${1:-r04i}; OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 60 tools/_abl/valu_rate > $OUT/valu_rate.txt 2>&1 || { cat $OUT/valu_rate.txt; exit 1; }
cat $OUT/valu_rate.txt
timeout -k 10 60 tools/_abl/ptr_probe > $OUT/ptr_probe.txt 2>&1 || { cat $OUT/ptr_probe.txt; exit 1; }
cat $OUT/ptr_probe.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_parity.log 2>&1 || { tail -30 $OUT/pytest_parity.log; exit 2; }
tail -1 $OUT/pytest_parity.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread -k "per_packet or percall or group" > $OUT/pytest_host.log 2>&1 || { tail -30 $OUT/pytest_host.log; exit 2; }
tail -1 $OUT/pytest_host.log
QFEC_PCTEST_BP=1 timeout -k 10 300 python -u - > $OUT/bp_parity.txt 2>&1 <<'PY' || { tail -20 $OUT/bp_parity.txt; exit 3; }
import subprocess, sys
import quicknet_amd as qa
qa.tune("percall_bpermute", 1)
import pytest
sys.exit(pytest.main(["-x", "-q", "-m", "gpu", "--timeout", "120", "--timeout-method", "thread", "-k", "per_packet or percall or group",
                      "-p", "no:cacheprovider", "tests/test_gpu_host.py"]))
PY
tail -1 $OUT/bp_parity.txt
timeout -k 10 300 python -u tools/percall_ab.py --variants "percall_bpermute=0;percall_bpermute=1" --rounds 5 --reps 2000 > $OUT/percall_ab.txt 2>&1 || { tail -20 $OUT/percall_ab.txt; exit 4; }
grep -v amdgpu.ids $OUT/percall_ab.txt
for bp in 0 1; do
  QFEC_PERCALL_TRACE=1 timeout -k 10 120 python -u tools/percall_ab.py --variants "percall_bpermute=$bp" --rounds 1 --reps 1000 > $OUT/trace_bp$bp.txt 2>&1 || { tail -20 $OUT/trace_bp$bp.txt; exit 5; }
  grep -v amdgpu.ids $OUT/trace_bp$bp.txt
done
for shape in "--k 16 --m 4 --block 1400 --erasures 4 --groups 250000" "--k 10 --m 3 --block 1024 --erasures 3 --groups 200000"; do
  timeout -k 10 200 python -u tools/ab.py --only recon_auto,recon_impl8,recon_impl9 --rounds 10 --reps 5 $shape >> $OUT/ab_impl9.txt 2>&1 || { tail -20 $OUT/ab_impl9.txt; exit 6; }
done
grep -v amdgpu.ids $OUT/ab_impl9.txt
bash tools/gpu_r04h.sh $T/recon as4mask clean cap7
