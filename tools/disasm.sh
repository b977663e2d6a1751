#!/bin/bash
# tools/disasm.sh SRC.hip [OUT.s] -- gfx950 disassembly + register usage of one kernel source, with the
# library's compile flags (cpu-based-ray-tracer_amd/Makefile).
set -euo pipefail
SRC=$1; OUT=${2:-/tmp/$(basename "$SRC" .hip).s}
PKG=$(cd "$(dirname "$0")/../cpu-based-ray-tracer_amd" && pwd)
TMP=$(mktemp -d)
/opt/rocm/bin/hipcc -std=c++20 -O3 -fPIC -I"$PKG/../include" -I"$PKG/csrc" -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize ${KFLAGS:-} --cuda-device-only -c "$SRC" -o "$TMP/k.o" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|Spill|Occupancy" || true
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$TMP/k.o" --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$TMP/d.o"
/opt/rocm/lib/llvm/bin/llvm-objdump -d "$TMP/d.o" > "$OUT"
rm -rf "$TMP"
