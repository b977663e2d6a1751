#!/bin/bash
# tools/r03_pp.sh -- camera pre-pass at 8 waves per SIMD (62 VGPRs, 4 spills) vs 7 (68 VGPRs), C4
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/pp
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python3 tools/ab_libs.py librt_hip_pp7.so librt_hip.so --spp 1024 --rounds 4 > "$OUT/ab_c4_prepass_waves.json" 2>&1
cat "$OUT/ab_c4_prepass_waves.json"
timeout -k 10 300 python3 tools/band_split.py --nranks 1 8 > "$OUT/band_split.jsonl" 2>&1
cat "$OUT/band_split.jsonl"
