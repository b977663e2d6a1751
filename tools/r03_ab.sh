#!/bin/bash
# tools/r03_ab.sh TAG LIB... -- interleaved A/B of library builds at C4 (bitwise check against the first), plus
# the section profile of librt_hip_sec.so when present.
set -euo pipefail
TAG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 300 python3 tools/ab_libs.py "$@" --spp ${SPP:-1024} --rounds ${ROUNDS:-3} > "$OUT/ab.json" 2>&1
cat "$OUT/ab.json"
if [ -f cpu-based-ray-tracer_amd/librt_hip_sec.so ] && [ "${SECTIONS:-1}" = "1" ]; then
  timeout -k 10 200 python3 tools/prof_one.py librt_hip_sec.so --sections --spp 256 > "$OUT/sections_c4_256spp.txt" 2>&1
  cat "$OUT/sections_c4_256spp.txt"
fi
