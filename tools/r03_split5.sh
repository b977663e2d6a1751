#!/bin/bash
# tools/r03_split5.sh -- split phase with both fresh rays at once (one box loop, one A+B candidate loop):
# C5 / BVH-variant parity and the A/B against the previous build
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/split5
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python3 -u -m pytest tests/test_c5.py tests/test_lbvh.py tests/test_gpu_parity.py tests/test_dist_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 500 python3 tools/ab_libs.py librt_hip_prev.so librt_hip.so --scene c5 --width 3840 --height 2160 --spp 64 --rounds 4 > "$OUT/ab_c5.json" 2>&1
cat "$OUT/ab_c5.json"
