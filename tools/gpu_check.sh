#!/bin/bash
# tools/gpu_check.sh -- one gpurun call: GPU parity tests, smoke, the default bench line, then the
# rocprof recipe (profiles/run_rocprof.sh).  Every GPU step has its own time limit; the first
# failure ends the script.
#   gpurun --timeout 1200 -- 'bash tools/gpu_check.sh r01c'
set -euo pipefail
TAG=${1:-r01}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/check_$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
cat "$OUT/smoke.log"
timeout -k 10 300 python3 bench.py > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
if [ "${PROFILE:-1}" = "1" ]; then
  bash profiles/run_rocprof.sh "$TAG"
fi
if [ "${SECTIONS:-0}" = "1" ] && [ -f cpu-based-ray-tracer_amd/librt_hip_sec.so ]; then
  timeout -k 10 200 python3 tools/prof_one.py librt_hip_sec.so --sections --spp 256 > "$OUT/sections_c4_256spp.txt" 2>&1
  timeout -k 10 200 python3 tools/prof_one.py librt_hip_sec.so --sections --scene c5 --spp 16 > "$OUT/sections_c5_16spp.txt" 2>&1
fi
