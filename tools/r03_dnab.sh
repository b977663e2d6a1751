#!/bin/bash
# tools/r03_dnab.sh TAG -- the denoiser tests, then DN33 / DN65 with 8x32 and 8x64 JBF blocks (RT_JBF_TALL)
set -euo pipefail
TAG=${1:-dnab}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 300 python3 -u -m pytest tests/test_denoiser.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for T in 32 64; do
  RT_JBF_TALL=$T timeout -k 10 200 python3 tools/bench_configs.py --configs DN33,DN65 > "$OUT/dn_tall$T.jsonl" 2>&1
  echo "tall $T"; cat "$OUT/dn_tall$T.jsonl"
done
