#!/bin/bash
# tools/r03_sweep2.sh -- C5 round shape on the LDS-staged split build
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/sweep2
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 500 python3 tools/ab_libs.py librt_hip.so librt_hip.so:RT_THRESH=6 librt_hip.so:RT_THRESH=12 librt_hip.so:RT_THRESH=16 librt_hip.so:RT_STEPS=8 librt_hip.so:RT_STEPS=16 --scene c5 --width 3840 --height 2160 --spp 64 --rounds 4 > "$OUT/ab.json" 2>&1
cat "$OUT/ab.json"
