#!/bin/bash
# Before/after A/B of builds of libqfec on one box: alternating processes of the same
# measurement, each build loaded through QFEC_LIB from tools/_abl/libqfec_<name>.so.
#   (at the old commit)  make -C quicknet_amd/csrc && cp quicknet_amd/libqfec.so tools/_abl/libqfec_before.so
#   gpurun -- bash tools/ab_lib.sh "python tools/wire_ab.py --unpack --variants base" before A B
set -o pipefail
CMD=${1:-python tools/wire_ab.py --unpack --variants base}
shift
NAMES=${@:-before}
for i in 1 2 3; do
  for n in $NAMES; do
    echo "== $n ($i)"
    QFEC_LIB_COMPAT=1 QFEC_LIB=$PWD/tools/_abl/libqfec_$n.so timeout -k 10 120 $CMD 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
