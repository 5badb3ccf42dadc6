#!/bin/bash
# Round-3 iteration: per-call server tests + phase probe, wire/frame tests, reconstruct parity
# (every body) and the RS(16,4) B=1400 reconstruct A/B.
#   gpurun --timeout 900 -- bash tools/gpu_r03p.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r03p}; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_percall.sh ${1:-r03p}/percall || exit 2
timeout -k 10 120 tools/_build/percall_phases > $OUT/phases.txt 2>&1 || { cat $OUT/phases.txt; exit 3; }
cat $OUT/phases.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_frames_fused.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 4; }
tail -1 $OUT/pytest.log
for shape in "--k 16 --m 4 --block 1400 --erasures 4 --groups 250000" "--k 10 --m 3 --block 1024 --erasures 3"; do
  timeout -k 10 300 python tools/ab.py --rounds 8 --only "probe,recon_impl3_(,recon_impl3_partial,recon_impl6" $shape > $OUT/ab.tmp 2>&1 || { tail $OUT/ab.tmp; exit 5; }
  grep -v amdgpu.ids $OUT/ab.tmp | tee -a $OUT/ab.txt
done
