"""The vertex kernel's compile-time variants still build (CPU; hipcc cross-compiles for gfx950): the section
timing diagnostics (RT_SECTIONS=1 and the candidate-histogram level 3, tools/prof_one.py) and the
waves-per-SIMD settings measured in DESIGN.md 6.4, the round-4 A/B switches (the drain without the pending
fold, the BVH variant's division kind, the zero-numerator short division) and the round-6 ones (the C5 A + B pair walk,
the walk fallback with the sphere branch; in rt_whitted.hip the shadow-ray pair walk, the half-plane orderings and
the packet walk; in rt_kernels.hip the walk study's K-rays-per-lane kernel, tools/walk_study.py).  The product build is the Makefile's; these compile
rt_coherent.hip alone, device code only, so a diagnostic that is not built by default cannot rot."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "cpu-based-ray-tracer_amd")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("flags", ["-DRT_SECTIONS=1", "-DRT_SECTIONS=3", "-DRT_COH_MIN_WAVES=7 -DRT_COH_BVH_MIN_WAVES=7",
                                   "-DRT_PEND_FOLD=0 -DRT_COH_BVH_PRE_MIN_WAVES=8",
                                   "-DRT_BVH_DIV_FAST=1 -DRT_DIV_ZERO_FAST=0", "-DRT_BVH_PAIR=1 -DRT_COH_SPH=1", "-DRT_MT_LOOP32=0 -DRT_B_TOP_FIRST=1 -DRT_MT_PK=1 -DRT_SPLIT_LOOP32=0",
                                   "@rt_whitted.hip -DRT_WH_PAIR=1 -DRT_WH_WAVES=6", "@rt_whitted.hip -DRT_WH_HALF=1",
                                   "@rt_whitted.hip -DRT_WH_PACKET=1", "@rt_kernels.hip -DRT_WALK_STUDY=1"])
def test_coherent_kernel_variant_compiles(flags, tmp_path):
    cmd = [HIPCC, "-std=c++20", "-O3", "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(PKG, "csrc"), "-ffp-contract=off",
           "-fno-fast-math", "--offload-arch=gfx950", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
           "-fno-slp-vectorize", "--cuda-device-only", "-c", os.path.join(PKG, "csrc", "rt_coherent.hip"), "-o", str(tmp_path / "k.o")]
    words = flags.split()
    if words[0].startswith("@"):   # another kernel source
        cmd[cmd.index(os.path.join(PKG, "csrc", "rt_coherent.hip"))] = os.path.join(PKG, "csrc", words.pop(0)[1:])
    cmd[1:1] = words
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
