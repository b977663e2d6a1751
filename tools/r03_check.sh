#!/bin/bash
# tools/r03_check.sh TAG [MT_CAPS] -- one gpurun call of round 3's kernel work: the GPU suite with the
# Moller-Trumbore cap forced (the carry path exercised), the library A/B against round 2's build, and a
# sweep of the cap.  Every GPU step has its own time limit; the first failure ends the script.
#   gpurun --timeout 900 -- 'bash tools/r03_check.sh r03a "0 4 5 6 7 8"'
set -euo pipefail
TAG=${1:-r03}
CAPS=${2:-"0 6"}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
RT_MT_CAP=${TEST_CAP:-6} timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 tools/ab_libs.py librt_hip_r02.so librt_hip.so --spp 1024 --rounds 3 > "$OUT/ab_r02_vs_new.json" 2>&1
cat "$OUT/ab_r02_vs_new.json"
SETS=""
for c in $CAPS; do SETS="$SETS --set RT_MT_CAP=$c"; done
timeout -k 10 300 python3 tools/sweep_env.py $SETS --spp 1024 --rounds 3 > "$OUT/sweep_mt_cap.jsonl" 2>&1
cat "$OUT/sweep_mt_cap.jsonl"
