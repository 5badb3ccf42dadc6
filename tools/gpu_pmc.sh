#!/bin/bash
# PMC traffic passes only: gpurun --timeout 900 -- bash tools/gpu_pmc.sh tag
set -o pipefail
OUT=gpurun_out/${1:-pmc}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python tools/pmc_traffic.py --out $OUT/pmc --json $OUT/traffic.json > $OUT/pmc.log 2>&1; rc=$?; cat $OUT/pmc.log | head -60; exit $rc
