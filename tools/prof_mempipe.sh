#!/bin/bash
# tools/prof_mempipe.sh TAG PROF_ONE_ARGS... -- the vector memory pipeline's counters for one render shape (round 6:
# what bounds the walks once more loads in flight stopped paying): TA busy and wavefronts, TD busy / stalls, the vL1D
# (TCP) accesses, misses to L2, their latency and the TCP's stall cycles.  Each pass its own run under its own time
# limit, within the per-block slot limits (MI355X_MICROARCH.md: TA 2, TD 2, TCP 4, GRBM 2); the first failure ends it.
#   gpurun -- 'bash tools/prof_mempipe.sh r06g_c3 --scene c3 --width 1280 --height 960 --spp 64'
set -euo pipefail
TAG=${1:?usage: prof_mempipe.sh TAG ARGS...}
shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/mem_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="$REPO/tools/prof_one.py librt_hip.so $*"
n=0
for P in "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
         "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum" \
         "TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum" \
         "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$n" -o pmc -- python3 $ARGS > "$OUT/p$n.log" 2>&1
done
find "$OUT" -name "*counter_collection*.csv" > "$OUT/csv_files.txt"
