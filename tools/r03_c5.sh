#!/bin/bash
# tools/r03_c5.sh TAG -- one gpurun call: the GPU suite, the C5 A/B of librt_hip.so against round 2's
# build (bitwise check), and the C5 section profile when librt_hip_sec.so is present.
set -euo pipefail
TAG=${1:-c5}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 tools/ab_libs.py librt_hip_r02.so librt_hip.so --scene c5 --width 3840 --height 2160 --spp 64 --rounds 3 > "$OUT/ab_c5.json" 2>&1
cat "$OUT/ab_c5.json"
if [ -f cpu-based-ray-tracer_amd/librt_hip_sec.so ] && [ "${SECTIONS:-0}" = "1" ]; then
  timeout -k 10 200 python3 tools/prof_one.py librt_hip_sec.so --sections --scene c5 --spp 16 > "$OUT/sections_c5_16spp.txt" 2>&1
  cat "$OUT/sections_c5_16spp.txt"
fi
if [ "${DN:-0}" = "1" ]; then
  bash tools/r03_dn.sh "${TAG}_dn"
fi
