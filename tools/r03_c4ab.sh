#!/bin/bash
# tools/r03_c4ab.sh TAG LIB... -- the GPU suite, then the C4 A/B of library builds (bitwise check against
# the first) and the bench line of librt_hip.so.  The first failure ends the script.
set -euo pipefail
TAG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 tools/ab_libs.py "$@" --spp 1024 --rounds 3 > "$OUT/ab_c4.json" 2>&1
cat "$OUT/ab_c4.json"
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log" | cut -c1-900
