#!/bin/bash
# traffic of variants: size-split request counters, 256 spp C4
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/tp
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for V in "librt_hip.so RT_RING_PACK=1" "librt_hip.so RT_RING_PACK=2" "librt_hip_nt.so RT_RING_PACK=1" "librt_hip_nt.so RT_RING_PACK=2"; do
  set -- $V
  T=${1%.so}_$2
  timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/$T/rd -o pmc -- python3 $REPO/tools/sweep_env.py --lib $1 --set $2 --spp 256 --rounds 1 > $OUT/$T.rd.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/$T/wr -o pmc -- python3 $REPO/tools/sweep_env.py --lib $1 --set $2 --spp 256 --rounds 1 > $OUT/$T.wr.log 2>&1
done
