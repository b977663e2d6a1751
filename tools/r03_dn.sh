#!/bin/bash
# tools/r03_dn.sh TAG -- one gpurun call for the denoiser: its GPU tests, DN15/33/65 timings and the
# rocprof kernel trace + PMC passes of DN65 (tools/bench_configs.py).  The first failure ends the script.
set -euo pipefail
TAG=${1:-dn}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 300 python3 -u -m pytest tests/test_denoiser.py tests/test_glibc_math.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python3 tools/bench_configs.py --configs DN15,DN33,DN65 > "$OUT/dn.jsonl" 2>&1
cat "$OUT/dn.jsonl"
cd /tmp && export TMPDIR=/tmp
ARGS="$REPO/tools/bench_configs.py --configs DN65 --reps 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- python3 $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d "$OUT/pmc_sq" -o pmc -- python3 $ARGS > "$OUT/pmc_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$OUT/pmc_sq2" -o pmc -- python3 $ARGS > "$OUT/pmc_sq2.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_tcc" -o pmc -- python3 $ARGS > "$OUT/pmc_tcc.log" 2>&1
echo done
