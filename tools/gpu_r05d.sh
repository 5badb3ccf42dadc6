#!/bin/bash
# round 5: receive kernel iteration -- wire/frames parity, the wire leg's times, SQ counters
set -o pipefail
OUT=gpurun_out/${1:-r05d}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 600 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_frames_fused.py tests/test_gpu_net.py tests/test_gpu_zfec.py -x -q --timeout 120 --timeout-method thread
step side 200 python tools/side_legs.py --steps 50
step side2 200 python tools/side_legs.py --steps 50
bash tools/gpu_sq_side.sh ${1:-r05d}/sq --no-bench > $OUT/sq.log 2>&1; echo "sq rc=$?"
grep -A17 "k_rx<10, 3" $OUT/sq/sq_summary.txt | grep -E "k_rx|VALU|SALU|WAVE_CYCLES|WAIT_ANY|INSTS_LDS|SMEM"
python - <<PY
import json
for n in ("side", "side2"):
    d = json.loads(open("$OUT/%s.log" % n).read().strip().split("\n")[-1])
    print(n, d["unpack_avg_ms"], d["unpack_frac"], d["framed"]["unpack_frames_avg_ms"], d["framed"]["unpack_frames_frac"], d["verified"], d["framed"]["verified"])
PY
