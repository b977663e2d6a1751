#!/bin/bash
# tools/round_numbers.sh TAG -- the per-configuration numbers behind DESIGN.md section 6.2 / 7 (one gpurun
# call): every config on the GPU, the reference on the host's cores, and the per-rank time of the
# row-band sets of an N-GPU frame (first and last rank, rendered one at a time on this GPU).
set -euo pipefail
TAG=${1:-r02}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/numbers_$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python3 -u tools/bench_configs.py > "$OUT/configs.jsonl" 2> "$OUT/configs.err"
timeout -k 10 300 python3 -u tools/bench_configs.py --configs C5 --c5-spp 4096 --reps 1 > "$OUT/c5_4096.jsonl" 2>> "$OUT/configs.err"
for N in 2 4 8; do
  for R in 0 $((N - 1)); do
    timeout -k 10 200 python3 -u tools/sweep_env.py --nranks $N --rank $R --set "" >> "$OUT/band_scaling.jsonl" 2>> "$OUT/band.err"
  done
done
[ "${SKIP_CPU:-0}" = "1" ] || timeout -k 10 600 python3 -u tools/cpu_reference_configs.py > "$OUT/cpu_reference_configs.jsonl" 2> "$OUT/cpu.err"
