#!/bin/bash
# tools/r03_check.sh TAG -- one gpurun call of round 3's kernel work: the GPU suite, the library A/B
# against round 2's build (C4, bitwise check), and the bench line.  Every GPU step has its own time
# limit; the first failure ends the script.
#   gpurun --timeout 900 -- 'bash tools/r03_check.sh r03b'
set -euo pipefail
TAG=${1:-r03}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 tools/ab_libs.py librt_hip_r02.so librt_hip.so --spp 1024 --rounds 3 > "$OUT/ab_r02_vs_new.json" 2>&1
cat "$OUT/ab_r02_vs_new.json"
if [ "${C5:-0}" = "1" ]; then
  timeout -k 10 300 python3 tools/ab_libs.py librt_hip_r02.so librt_hip.so --scene c5 --width 3840 --height 2160 --spp 64 --rounds 2 > "$OUT/ab_r02_vs_new_c5.json" 2>&1
  cat "$OUT/ab_r02_vs_new_c5.json"
fi
timeout -k 10 300 python3 bench.py > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
