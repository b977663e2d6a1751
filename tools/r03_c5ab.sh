#!/bin/bash
# tools/r03_c5ab.sh TAG LIB... -- C5 A/B of library builds (bitwise check against the first), then an
# RT_STEPS / RT_THRESH sweep of the second.
set -euo pipefail
TAG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 300 python3 tools/ab_libs.py "$@" --scene c5 --width 3840 --height 2160 --spp 64 --rounds 3 > "$OUT/ab_c5.json" 2>&1
cat "$OUT/ab_c5.json"
if [ "${SWEEP:-0}" = "1" ]; then
  timeout -k 10 300 python3 tools/sweep_env.py --scene c5 --width 3840 --height 2160 --spp 64 --lib "$2" --set "RT_STEPS=8 RT_THRESH=40" --set "RT_STEPS=12 RT_THRESH=40" --set "RT_STEPS=16 RT_THRESH=40" --set "RT_STEPS=8 RT_THRESH=24" --set "RT_STEPS=8 RT_THRESH=52" > "$OUT/sweep.json" 2>&1
  cat "$OUT/sweep.json"
fi
