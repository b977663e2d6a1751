#!/bin/bash
# tools/r03_split3.sh -- C5 split trace (default round threshold 8): the GPU suite, a steps / threshold
# sweep against the previous build, and C5 at 4096 spp
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/split3
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 500 python3 tools/ab_libs.py librt_hip_head.so librt_hip.so librt_hip.so:RT_THRESH=6 librt_hip.so:RT_THRESH=12 librt_hip.so:RT_STEPS=4 librt_hip.so:RT_STEPS=12 librt_hip.so:RT_STEPS=16 --scene c5 --width 3840 --height 2160 --spp 64 --rounds 3 > "$OUT/ab_c5_steps.json" 2>&1
cat "$OUT/ab_c5_steps.json"
timeout -k 10 300 python3 -u tools/bench_configs.py --configs C5 --c5-spp 4096 --reps 1 > "$OUT/c5_4096.jsonl" 2> "$OUT/c5.err"
cat "$OUT/c5_4096.jsonl"
