#!/bin/bash
# tools/r03_split2.sh -- C5 split trace: round threshold A/B against the previous build, interleaved
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/split2
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 500 python3 tools/ab_libs.py librt_hip_head.so librt_hip.so librt_hip.so:RT_THRESH=16 librt_hip.so:RT_THRESH=8 librt_hip.so:RT_THRESH=4 librt_hip.so:RT_THRESH=2 librt_hip_s7.so:RT_THRESH=8 --scene c5 --width 3840 --height 2160 --spp 64 --rounds 3 > "$OUT/ab_c5_thresh.json" 2>&1
cat "$OUT/ab_c5_thresh.json"
