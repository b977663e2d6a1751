#!/bin/bash
# tools/r03_c1c3.sh -- the Whitted kernels after the C3 rework: C1/C3 parity, the C1 occupancy A/B, every
# config's numbers on the current build, and a rocprofv3 kernel-trace summary of C3.
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/c1c3
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 300 python3 -u -m pytest tests/test_bvh_tracer.py tests/test_c1_spheres.py tests/test_frontend.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python3 tools/ab_libs.py librt_hip.so librt_hip_w5.so --scene c1 --width 640 --height 480 --spp 1 --rounds 20 > "$OUT/ab_c1.json" 2>&1
cat "$OUT/ab_c1.json"
timeout -k 10 400 python3 -u tools/bench_configs.py > "$OUT/configs.jsonl" 2> "$OUT/configs.err"
cat "$OUT/configs.jsonl"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c3" -o c3 -- python3 -u tools/bench_configs.py --configs C3 > "$OUT/prof_c3.log" 2>&1
find "$OUT/prof_c3" -name "*stats*"
