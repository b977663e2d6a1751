#!/bin/bash
# tools/gpu_run.sh TAG STEP [STEP ...] -- the one launcher for gpurun calls (replaces round 3's per-experiment
# tools/r03_*.sh).  Each step runs under its own time limit and writes under gpurun_out/TAG/; the first
# failing step ends the call (no GPU step runs after a failure, a timeout or a fault).
#
#   tests                  the GPU suite (pytest -m gpu)                          -> pytest_gpu.log
#   tests:EXPR             only the GPU tests matching -k EXPR                     -> pytest_gpu_k.log
#   smoke                  __graft_entry__.smoke()                                -> smoke.log
#   bench                  the default bench line (C4, N = 1)                     -> bench.log
#   configs                C1..C5 and the denoiser (tools/bench_configs.py)       -> configs.jsonl
#   c5full                 C5 at its full 4096 spp (warm-up at 4096 spp)                            -> c5_4096.jsonl
#   prof                   rocprofv3 trace + PMC passes of the bench command      -> profiles via profiles/run_rocprof.sh
#   profc5                 the same for C5 at 64 spp                              -> tools/prof_c5.sh
#   profc5:K=V             the C5 profile with one knob set (e.g. RT_WALK_ORDER=0)
#   profc3                 trace + PMC passes of C3 (1280x960x64, whitted_kernel)  -> tools/prof_scene.sh
#   ab:ARGS                tools/ab_libs.py ARGS (comma-separated, e.g. ab:librt_hip.so,librt_hip_x.so,--spp,256)
#   sweep:ARGS             tools/sweep_env.py ARGS (comma-separated)
#   sections:LIB:SCENE:SPP[:W:H] wave cycles per kernel section of an RT_SECTIONS build (tools/prof_one.py)
#
#   gpurun --timeout 1200 -- 'bash tools/gpu_run.sh r04a tests smoke bench prof'
set -euo pipefail
TAG=${1:?usage: gpu_run.sh TAG STEP...}
shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
export RT_DEBUG_KNOBS=1   # the A/B tools set knobs (csrc/rt_knobs.h); the product defaults are unaffected
n=0
for step in "$@"; do
  n=$((n + 1))
  echo "== step $n: $step ($(date +%T))"
  case "$step" in
    tests)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
        || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
      tail -2 "$OUT/pytest_gpu.log" ;;
    tests:*)
      timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "${step#tests:}" > "$OUT/pytest_gpu_k.log" 2>&1 \
        || { tail -40 "$OUT/pytest_gpu_k.log"; exit 1; }
      tail -3 "$OUT/pytest_gpu_k.log" ;;
    smoke)
      timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      cat "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 300 python3 bench.py > "$OUT/bench.log" 2>&1
      tail -1 "$OUT/bench.log" | cut -c1-600 ;;
    configs)
      timeout -k 10 400 python3 -u tools/bench_configs.py > "$OUT/configs.jsonl" 2> "$OUT/configs.err"
      cut -c1-300 "$OUT/configs.jsonl" ;;
    c5full)
      timeout -k 10 300 python3 -u tools/bench_configs.py --configs C5 --c5-spp 4096 --reps 1 --full-warmup > "$OUT/c5_4096.jsonl" 2>> "$OUT/configs.err"
      cat "$OUT/c5_4096.jsonl" ;;
    prof)
      bash profiles/run_rocprof.sh "$TAG" ;;
    profc5)
      bash tools/prof_c5.sh "${TAG}_c5" 64 ;;
    profc3)
      bash tools/prof_scene.sh "${TAG}_c3" --scene c3 --width 1280 --height 960 --spp 64 ;;
    profc5:*)
      # the same under one knob (K=V), e.g. profc5:RT_WALK_ORDER=0 -> gpurun_out/prof_TAG_c5_RT_WALK_ORDER0
      kv=${step#profc5:}
      env "$kv" bash tools/prof_c5.sh "${TAG}_c5_${kv//=/}" 64 ;;
    ab:*)
      IFS=',' read -r -a a <<< "${step#ab:}"
      timeout -k 10 400 python3 -u tools/ab_libs.py "${a[@]}" > "$OUT/ab_$n.json" 2>&1 || { tail -20 "$OUT/ab_$n.json"; exit 1; }
      cat "$OUT/ab_$n.json" ;;
    sweep:*)
      IFS=',' read -r -a a <<< "${step#sweep:}"
      timeout -k 10 400 python3 -u tools/sweep_env.py "${a[@]}" > "$OUT/sweep_$n.json" 2>&1 || { tail -20 "$OUT/sweep_$n.json"; exit 1; }
      cat "$OUT/sweep_$n.json" ;;
    sections:*)
      IFS=':' read -r _ lib scene spp w h <<< "$step"
      timeout -k 10 200 python3 tools/prof_one.py "$lib" --sections --scene "$scene" --spp "$spp" --width "${w:-1920}" --height "${h:-1080}" \
        > "$OUT/sections_${scene}_${spp}spp.txt" 2>&1
      cat "$OUT/sections_${scene}_${spp}spp.txt" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
