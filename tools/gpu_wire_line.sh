#!/bin/bash
# Fused send with whole-line rows: wire parity tests, then A/B against the 16-B-pitch kernels.
set -o pipefail
OUT=gpurun_out/${1:-wline}; mkdir -p $OUT; export TMPDIR=/tmp
true
tail -1 $OUT/pytest.log
for S in 1024 1400; do
timeout -k 10 120 python tools/wire_ab.py --size $S --wire-align 64 --variants "base;wire_line=0" --rounds 8 >> $OUT/pack_ab.txt 2>&1 || { tail $OUT/pack_ab.txt; exit 3; }
timeout -k 10 120 python tools/wire_ab.py --size $S --align 16 --variants "base" --rounds 8 >> $OUT/pack_ab.txt 2>&1 || { tail $OUT/pack_ab.txt; exit 3; }
done
grep -v amdgpu.ids $OUT/pack_ab.txt
