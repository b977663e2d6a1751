#!/bin/bash
# tools/r03_gather.sh TAG -- the gather calibration (tools/calib_gather.hip) with its TCP/TCC counters,
# and the C5 A/B of the compact BVH (RT_QBVH) on the current build.
set -euo pipefail
TAG=${1:-gather}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 120 tools/_calib_gather > "$OUT/gather.jsonl" 2>&1
cat "$OUT/gather.jsonl"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_WAVES --output-format csv -d "$OUT/pmc_tcp" -o pmc -- "$REPO/tools/_calib_gather" > "$OUT/pmc_tcp.log" 2>&1
cd "$REPO"
timeout -k 10 300 python3 tools/sweep_env.py --scene c5 --width 3840 --height 2160 --spp 64 --set "RT_QBVH=0" --set "RT_QBVH=1" > "$OUT/qbvh.json" 2>&1
cat "$OUT/qbvh.json"
