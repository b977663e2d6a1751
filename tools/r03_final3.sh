#!/bin/bash
# tools/r03_final3.sh -- the end-of-round evidence of the current build in one gpurun call: the GPU suite,
# smoke, the bench line, every config (C5 also at 4096 spp), then the rocprofv3 passes of the bench
# command (profiles/run_rocprof.sh) and of C5 (tools/prof_c5.sh).  Every GPU step has its own time limit.
set -euo pipefail
TAG=${1:-r03f}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
cat "$OUT/smoke.log"
timeout -k 10 300 python3 bench.py > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log" | cut -c1-400
timeout -k 10 400 python3 -u tools/bench_configs.py > "$OUT/configs.jsonl" 2> "$OUT/configs.err"
timeout -k 10 300 python3 -u tools/bench_configs.py --configs C5 --c5-spp 4096 --reps 1 > "$OUT/c5_4096.jsonl" 2>> "$OUT/configs.err"
cat "$OUT/c5_4096.jsonl"
bash profiles/run_rocprof.sh "$TAG"
bash tools/prof_c5.sh "${TAG}_c5" 64
echo done
