#!/bin/bash
# tools/r03_bw.sh -- C5 split trace: waves per SIMD of the BVH variant (8: 15 VGPR spills, 7: 4, 6: none)
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/bw
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 500 python3 tools/ab_libs.py librt_hip.so librt_hip_bw7.so librt_hip_bw6.so --scene c5 --width 3840 --height 2160 --spp 64 --rounds 4 > "$OUT/ab_c5_waves.json" 2>&1
cat "$OUT/ab_c5_waves.json"
