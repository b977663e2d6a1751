#!/bin/bash
# tools/r03_parts.sh -- segment parts: the GPU suite, the per-kernel band-set split, and the A/B against
# short segments (RT_SEG_PARTS_OFF=1) on 8-, 4- and 1-rank band sets.
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/parts
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 200 python3 tools/band_split.py > "$OUT/band_split.jsonl" 2>&1
cat "$OUT/band_split.jsonl"
for N in 8 4 1; do
  timeout -k 10 200 python3 -u tools/sweep_env.py --nranks $N --rank 0 --rounds 3 --set "" --set "RT_SEG_PARTS_OFF=1" >> "$OUT/ab_parts.jsonl" 2>&1
done
cat "$OUT/ab_parts.jsonl"
