#!/bin/bash
# tools/r03_head.sh TAG -- the GPU suite, smoke and the default bench line of the current tree;
# every GPU step has its own time limit and the first failure ends the script.
set -euo pipefail
TAG=${1:-r03}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
cat "$OUT/smoke.log"
timeout -k 10 300 python3 bench.py > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
