#!/bin/bash
# profiles/run_rocprof.sh -- the profiling recipe behind profiles/ (run on the GPU box via gpurun).
#   kernel trace + stats of the default bench command, then separate PMC passes
#   (FETCH_SIZE, WRITE_SIZE, SQ counters) -- never combined with other trace domains.
set -euo pipefail
TAG=${1:-r01}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="$REPO/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-small-configs ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- python3 $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o pmc -- python3 $ARGS > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o pmc -- python3 $ARGS > "$OUT/pmc_write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d "$OUT/pmc_sq" -o pmc -- python3 $ARGS > "$OUT/pmc_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_tcc" -o pmc -- python3 $ARGS > "$OUT/pmc_tcc.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$OUT/pmc_sq2" -o pmc -- python3 $ARGS > "$OUT/pmc_sq2.log" 2>&1
# request-size splits of the L2 -> fabric traffic (bytes = 32/64/128 x count, no FETCH_SIZE factor needed)
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d "$OUT/pmc_rdsz" -o pmc -- python3 $ARGS > "$OUT/pmc_rdsz.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv -d "$OUT/pmc_wrsz" -o pmc -- python3 $ARGS > "$OUT/pmc_wrsz.log" 2>&1
# the same counters on known-byte kernels of the kernel's access shapes (tools/calib_traffic.hip)
if [ -x "$REPO/tools/_calib_traffic" ]; then
  for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"; do
    N=calib_$(echo $P | cut -d' ' -f1)
    timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/$N" -o pmc -- "$REPO/tools/_calib_traffic" > "$OUT/$N.log" 2>&1
  done
fi
find "$OUT" -name "*.csv" > "$OUT/csv_files.txt"
