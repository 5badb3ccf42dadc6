#!/bin/bash
# 16-B-lane receive with a 2-dword fused tail (wire_rx_split 4): parity, then A/B at 1400-B payloads
set -o pipefail
OUT=gpurun_out/${1:-rx_tail}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_frames_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python tools/wire_ab.py --rounds 6 --size 1400 --wire-align 64 --unpack --variants "base;wire_rx_split=5;wire_rx_split=4" > $OUT/ab.tmp 2>&1 || { tail -20 $OUT/ab.tmp; exit 3; }
grep -v amdgpu.ids $OUT/ab.tmp | tee $OUT/ab.txt
