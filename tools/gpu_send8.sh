#!/bin/bash
# 8-byte-lane one-wave send (wire_send_wave 3): parity, then interleaved A/B against the default at
# 1 KiB and 1 400-B payloads, datagrams and one-pass frames.
set -o pipefail
OUT=gpurun_out/${1:-send8}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_frames_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
for args in "--size 1400 --wire-align 64 --variants base;wire_send_wave=4;wire_send_wave=0"; do
  timeout -k 10 200 python tools/wire_ab.py --rounds 6 $args > $OUT/ab.tmp 2>&1 || { tail -20 $OUT/ab.tmp; exit 3; }
  grep -v amdgpu.ids $OUT/ab.tmp | tee -a $OUT/ab.txt
done
for t in ""; do
  for pl in 1400; do
    timeout -k 10 200 python tools/frames_bench.py --payload $pl --rounds 3 --tune "$t" > $OUT/fr.tmp 2>&1 || { tail -20 $OUT/fr.tmp; exit 4; }
    echo "== frames payload $pl tune '$t'" | tee -a $OUT/frames.txt; grep one_pass $OUT/fr.tmp | tee -a $OUT/frames.txt
  done
done
