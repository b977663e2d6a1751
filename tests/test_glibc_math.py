"""The denoiser's expf / acosf (csrc/rt_glibc_math.h): glibc 2.35's algorithms restated so the joint
bilateral filter's weights (DN/Denoiser.h:195,203: std::acos / std::exp on floats -> glibc acosf /
expf) are the reference's bit for bit.

CPU: the restatement, compiled for the host, against the host libm on a strided sweep of the filter's
domains (expf on [-inf, 0], acosf on [0, 1]); tools/verify_glibc_math.cpp run with stride 1 covers
every float (2.14e9 + 1.07e9; 0 mismatches for the FMA build of expf that x86-64 glibc dispatches,
and for acosf; profiles/r03/verify/glibc_math_exhaustive.json), and the filter's divisions by its
default 2 sigma^2 through Markstein's correction (rt_denoise.hip jbf_div) for every x it takes.
GPU: the device evaluation (rt_math_selftest columns 7-8) against the host libm, bitwise."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import _oracle as O
from _rt import rt

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "verify_glibc_math.cpp")
BIN = os.path.join(REPO, "tests", "_bin", "verify_glibc_math")


def _build():
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src_m = max(os.path.getmtime(SRC), os.path.getmtime(os.path.join(REPO, "cpu-based-ray-tracer_amd", "csrc", "rt_glibc_math.h")))
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < src_m:
        os.makedirs(os.path.dirname(BIN), exist_ok=True)
        subprocess.check_call([hipcc, "-x", "hip", "--offload-arch=gfx950", "-O2", "-ffp-contract=off", "-fno-builtin",
                               "-I" + os.path.join(REPO, "cpu-based-ray-tracer_amd", "csrc"), SRC, "-o", BIN, "-lpthread"])
    return BIN


def test_host_restatement_matches_libm_strided():
    r = subprocess.run([_build(), "1009"], capture_output=True, text=True, timeout=120)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["expf_fma_mismatches"] == 0 and out["acosf_mismatches"] == 0 and out["division_mismatches"] == 0, out
    assert out["expf_floats"] > 2_000_000 and out["acosf_floats"] > 1_000_000


def _domains(stride_e, stride_a):
    neg = np.arange(0x80000000, 0xFF800001, stride_e, dtype=np.uint64).astype(np.uint32).view(np.float32)
    unit = np.arange(0, 0x3F800001, stride_a, dtype=np.uint32).view(np.float32)
    h = float.fromhex
    special = np.array([0.0, -0.0, 1.0, 0.5, h("0x1p-26"), h("-0x1.9fe368p6"), h("-0x1.9fe36ap6"), h("-0x1.9d1d9ep6"), -88.0, -103.5,
                        -np.inf, np.nextafter(np.float32(0.5), np.float32(0))], np.float32)
    return np.concatenate([neg, unit, special])


@pytest.mark.gpu
def test_device_expf_acosf_match_libm():
    x = _domains(997, 499)
    c = rt.Context(0)
    try:
        out = c.math_selftest(x)
    finally:
        c.close()
    e, a = O.libm_exp_acos(x)
    neg = (x < 0) | ((x == 0) & np.signbit(x)) | (x == 0)
    unit = (x >= 0) & (x <= 1)
    assert np.array_equal(out[neg, 7].view(np.uint32), e[neg].view(np.uint32))
    assert np.array_equal(out[unit, 8].view(np.uint32), a[unit].view(np.uint32))
