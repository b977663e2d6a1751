#!/bin/bash
# tools/r03_trace.sh TAG -- rocprofv3 kernel traces (per-kernel times) of C4 and C5 for the current and the
# round-2 library.
set -euo pipefail
TAG=${1:-r03}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for LIB in librt_hip.so librt_hip_r02.so; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4_$LIB" -o t -- python3 "$REPO/tools/prof_one.py" $LIB --spp 256 > "$OUT/c4_$LIB.log" 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5_$LIB" -o t -- python3 "$REPO/tools/prof_one.py" $LIB --scene c5 --width 3840 --height 2160 --spp 32 > "$OUT/c5_$LIB.log" 2>&1
done
for f in $(find "$OUT" -name "*kernel_stats.csv"); do echo "== $f"; cut -d, -f1-8 "$f" | head -8; done
