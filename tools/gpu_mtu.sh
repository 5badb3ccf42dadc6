#!/bin/bash
# MTU-size (1400-B) payloads on the datagram path: wave64 send / frames parity, then interleaved
# A/B of the send (one wave per group in two passes vs body + line-0) and the receive.
#   gpurun --timeout 900 -- bash tools/gpu_mtu.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-mtu}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_frames_fused.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wave64 or frames" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
for args in "--size 1400 --wire-align 64 --variants base;wire_send_wave=0" "--size 1024 --wire-align 64 --variants base;wire_send_wave=0" "--size 1400 --wire-align 64 --unpack --variants base;wire_rx_split=2;wire_rx_lds=2" ${EXTRA_AB:+"$EXTRA_AB"}; do
  timeout -k 10 200 python tools/wire_ab.py --rounds 6 $args > $OUT/ab.tmp 2>&1 || { tail -20 $OUT/ab.tmp; exit 3; }
  grep -v amdgpu.ids $OUT/ab.tmp | tee -a $OUT/ab.txt
done
timeout -k 10 200 python tools/frames_bench.py --payload 1400 --rounds 3 > $OUT/frames.txt 2>&1 || { tail -20 $OUT/frames.txt; exit 4; }
grep -v amdgpu.ids $OUT/frames.txt
