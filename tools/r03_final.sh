#!/bin/bash
# tools/r03_final.sh TAG -- one gpurun call on the current build: the GPU suite, smoke, the bench line,
# the C5 rocprof passes (tools/prof_c5.sh) and the C4/C5 section split.  The first failure ends it.
set -euo pipefail
TAG=${1:-r03}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
cat "$OUT/smoke.log"
timeout -k 10 300 python3 bench.py > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
if [ "${PROF:-1}" = "1" ]; then
  bash tools/prof_c5.sh "${TAG}_c5" 64
  cd "$REPO"
fi
timeout -k 10 200 python3 tools/prof_one.py librt_hip_sec.so --sections --spp 256 > "$OUT/sections_c4_256spp.txt" 2>&1
timeout -k 10 200 python3 tools/prof_one.py librt_hip_sec.so --sections --scene c5 --spp 16 > "$OUT/sections_c5_16spp.txt" 2>&1
cat "$OUT/sections_c5_16spp.txt"
