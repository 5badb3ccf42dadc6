#!/bin/bash
# round 5: after the A/B retirement -- full GPU suite, smoke, the default bench line
set -o pipefail
OUT=gpurun_out/${1:-r05e}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
python - <<PY
import json
d = json.loads(open("$OUT/bench.log").read().strip().split("\n")[-1])
print("value", d["value"], "enc", d["roofline"]["frac"], d["roofline_other"]["frac"], "verified", d["verified"])
print("config4", {k: d["config4"].get(k) for k in ("value", "rank0_encode_frac", "rank0_reconstruct_frac")})
w = d["wire"]; print("wire", w["unpack_avg_ms"], w["unpack_frac"], w["framed"]["unpack_frames_avg_ms"], w["framed"]["unpack_frames_frac"], w["pack_frac"])
print("rs_abi_host", {k: d["rs_abi_host"].get(k) for k in ("value", "encode_gibs", "reconstruct_gibs", "verified", "vs_cpu_1thread", "vs_cpu_threads", "reference_check")})
print("zfec", {k: d["zfec"].get(k) for k in ("send_e2e_gibs", "recv_e2e_gibs", "verified")} if isinstance(d.get("zfec"), dict) else d.get("zfec"))
print("cpu", d["cpu_baseline"]["value"], (d.get("cpu_baseline_threads") or {}).get("value"))
PY
