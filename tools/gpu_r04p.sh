#!/bin/bash
# all GPU tests + smoke + the default bench line on the final per-call server
set -o pipefail
T=${1:-r04p}; OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 2; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -2 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 4; }
python3 -c "
import json; b=json.load(open('$OUT/bench.json'))
print(b['value'], b['roofline']['frac'], b['roofline_other']['frac'], b['config4']['rank0_encode_frac'], b['config4']['rank0_reconstruct_frac'])
print(b['per_call']); print(b['cpu_baseline']['per_call'])"
