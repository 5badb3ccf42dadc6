#!/bin/bash
# Build libqfec variants whose send kernel (k_pack_wave64) drops one stage each (QFEC_TX_ABLATE bits,
# qfec_wire.hip): tools/_abl/libqfec_tx<bits>.so.  Measurement builds only: their outputs are wrong.
# The SQ counters of each against the full build give the per-stage instruction counts
# (tools/gpu_r05q.sh).  The QFEC_TX_ABLATE switches are not in the product source (its hash keys
# the PMC traffic): apply profiles/r05q/tx_ablate.patch first (git apply), revert after.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_abl/rxbuild
C=quicknet_amd/csrc
for bits in 1 2 4 8; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -DQFEC_TX_ABLATE=$bits \
    -c $C/qfec_wire.hip -o tools/_abl/rxbuild/qfec_wire_$bits.o &
done
wait
for bits in 1 2 4 8; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o tools/_abl/libqfec_tx$bits.so \
    $C/build/qfec_kernels.hip.o tools/_abl/rxbuild/qfec_wire_$bits.o $C/build/qfec_percall.hip.o $C/build/qfec_rx.hip.o \
    $C/build/qfec_runtime.cpp.o $C/build/gf256.cpp.o $C/build/qfec_net.cpp.o $C/build/qfec_zfec.cpp.o $C/build/qfec_pool.cpp.o
done
ls -la tools/_abl/libqfec_tx*.so
