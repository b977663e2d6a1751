#!/bin/bash
# tools/r03_split.sh -- C5 split trace: the BVH-variant parity tests, the A/B against the previous build
# (librt_hip_head.so), and a sweep of the round threshold on the split build.
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/split
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python3 -u -m pytest tests/test_c5.py tests/test_lbvh.py tests/test_gpu_parity.py tests/test_skip_adversarial.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python3 tools/ab_libs.py librt_hip_head.so librt_hip.so librt_hip_s7.so --scene c5 --width 3840 --height 2160 --spp 64 --rounds 2 > "$OUT/ab_c5.json" 2>&1
cat "$OUT/ab_c5.json"
timeout -k 10 300 python3 -u tools/sweep_env.py --scene c5 --width 3840 --height 2160 --spp 64 --rounds 2 --set "" --set "RT_THRESH=16" --set "RT_THRESH=8" --set "RT_THRESH=48" --set "RT_SPLIT=0" > "$OUT/sweep.jsonl" 2>&1 || true
cat "$OUT/sweep.jsonl"
