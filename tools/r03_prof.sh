#!/bin/bash
# tools/r03_prof.sh TAG -- one gpurun call: rocprof evidence of the current build for C4 (the bench
# command, profiles/run_rocprof.sh) and C5 (tools/prof_c5.sh), plus the per-section cycle split of both
# (librt_hip_sec.so, RT_SECTIONS=1).  The first failure ends the script.
set -euo pipefail
TAG=${1:-r03}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO"
bash profiles/run_rocprof.sh "$TAG"
bash tools/prof_c5.sh "${TAG}_c5" 64
cd "$REPO"
OUT=$REPO/gpurun_out/sections_$TAG
mkdir -p "$OUT"
timeout -k 10 200 python3 tools/prof_one.py librt_hip_sec.so --sections --spp 256 > "$OUT/sections_c4_256spp.txt" 2>&1
timeout -k 10 200 python3 tools/prof_one.py librt_hip_sec.so --sections --scene c5 --spp 16 > "$OUT/sections_c5_16spp.txt" 2>&1
echo done
