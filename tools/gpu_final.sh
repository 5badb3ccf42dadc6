#!/bin/bash
# End-of-round measurement pass in one gpurun call, so every number the line cites comes from the
# final sources: the wire leg's rocprof + PMC (tools/gpu_side_prof.sh), its traffic entry merged
# into profiles/traffic.json, then tools/gpu_full.sh (GPU tests, smoke, the headline's PMC, bench,
# rocprof, the 2-rank rehearsal).  Copy gpurun_out/TAG_side and gpurun_out/TAG into profiles/
# afterwards (one directory per run).
#   gpurun --timeout 1200 -- bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
bash tools/gpu_side_prof.sh ${TAG}_side || exit $?
python3 - "$TAG" <<'PY' || exit 11
import json, sys
tag = sys.argv[1]
side = json.load(open(f"gpurun_out/{tag}_side/traffic.json"))
main = json.load(open("profiles/traffic.json"))
for k, v in side.items():
    if k.startswith("wire_"):
        main[k] = v
json.dump(main, open("profiles/traffic.json", "w"), indent=1)
print("merged", [k for k in side if k.startswith("wire_")])
PY
bash tools/gpu_full.sh $TAG
