#!/bin/bash
# tools/r03_c5sweep.sh TAG -- C5: waves-per-SIMD builds A/B and the RT_THRESH / RT_STEPS sweep of librt_hip.so
set -euo pipefail
TAG=${1:-c5sweep}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 300 python3 tools/ab_libs.py librt_hip.so librt_hip_w7.so librt_hip_w6.so --scene c5 --width 3840 --height 2160 --spp 64 --rounds 3 > "$OUT/ab_waves.json" 2>&1
cat "$OUT/ab_waves.json"
timeout -k 10 300 python3 tools/sweep_env.py --scene c5 --width 3840 --height 2160 --spp 64 --rounds 3 --set "RT_STEPS=8 RT_THRESH=40" --set "RT_STEPS=4 RT_THRESH=40" --set "RT_STEPS=16 RT_THRESH=40" --set "RT_STEPS=8 RT_THRESH=24" --set "RT_STEPS=8 RT_THRESH=32" --set "RT_STEPS=8 RT_THRESH=48" > "$OUT/sweep.json" 2>&1
cat "$OUT/sweep.json"
