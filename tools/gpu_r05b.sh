#!/bin/bash
# round 5: the new receive kernel (qfec_rx.hip) and the rs.h host pipeline, first GPU pass
set -o pipefail
OUT=gpurun_out/${1:-r05b}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 600 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_frames_fused.py tests/test_gpu_rs_host.py -x -q --timeout 120 --timeout-method thread
step side 200 python tools/side_legs.py --steps 50
step rs_new 200 python tools/rs_abi_rate.py --reps 3
QFEC_LIB_COMPAT=1 QFEC_LIB=$PWD/tools/_abl/libqfec_r04.so step rs_r04 300 python tools/rs_abi_rate.py --reps 2
step rs_new_t1 200 python tools/rs_abi_rate.py --reps 2 --threads 1
python - <<PY
import json
for n in ("side", "rs_new", "rs_r04", "rs_new_t1"):
    try:
        d = json.loads(open("$OUT/%s.log" % n).read().strip().split("\n")[-1])
    except Exception as e:
        print(n, "?", e); continue
    if n == "side":
        print(n, {k: d.get(k) for k in ("unpack_avg_ms", "unpack_frac", "pack_avg_ms", "verified")}, d.get("framed", {}).get("unpack_frames_avg_ms"), d.get("framed", {}).get("unpack_frames_frac"))
    else:
        print(n, {k: d.get(k) for k in ("value", "encode_gibs", "reconstruct_gibs", "verified", "host_threads")})
PY
