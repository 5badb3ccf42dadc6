#!/bin/bash
# Fused send with whole-line rows (A/B against the 16-B-pitch kernels), then the exact layer's
# GPU tests and rate.
set -o pipefail
OUT=gpurun_out/${1:-wline}; mkdir -p $OUT; export TMPDIR=/tmp
for S in 1024 1400; do
timeout -k 10 120 python tools/wire_ab.py --size $S --wire-align 64 --variants "base;wire_line=0" --rounds 8 >> $OUT/pack_ab.txt 2>&1 || { tail $OUT/pack_ab.txt; exit 3; }
timeout -k 10 120 python tools/wire_ab.py --size $S --align 16 --variants "base" --rounds 8 >> $OUT/pack_ab.txt 2>&1 || { tail $OUT/pack_ab.txt; exit 3; }
done
grep -v amdgpu.ids $OUT/pack_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_zfec.py tests/test_gpu_wire.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
QFEC_ZFEC_TIMING=1 timeout -k 10 200 python tools/zfec_rate.py --reps 2 > $OUT/zfec_rate.txt 2>&1 || { tail -20 $OUT/zfec_rate.txt; exit 4; }
grep "rep " $OUT/zfec_rate.txt; grep "zfec flush" $OUT/zfec_rate.txt | tail -9
