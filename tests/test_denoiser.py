"""The reference's Denoiser project (DN/ = "Denoiser/8599RayTracerGUI/src/"): a
1-spp path-traced Cornell-box frame through the pixel centres that records a G-buffer
(DN/Renderer.cpp:285-311), the joint bilateral filter and the temporal filter of DN/Denoiser.h, and the
RGBA8 pack (DN/Renderer.cpp:101-283) -- on the GPU (megakernel GB mode + rt_denoise.hip) against
golden frames from oracle/_ref/ref_denoiser (the reference's Denoising::Denoiser compiled as it is, its
DN/ geometry and camera code, the path-tracing glue restated; oracle/gen_golden.py `dn`).  The camera
moves between frames, so the temporal reprojection is exercised.

Tolerance: none.  The G-buffer (color, position, normal, primitive id), the joint bilateral filter's
output, the temporal filter's output and the RGBA8 frames are bit-exact: the filter's weights call
expf/acosf, which the device evaluates with glibc's algorithms (csrc/rt_glibc_math.h,
tests/test_glibc_math.py)."""
import os

import numpy as np
import pytest

import _oracle as O
from _rt import rt

FWD = rt.DEFAULT_CAMERA_FORWARD


@pytest.fixture(scope="module")
def fixture():
    return np.load(os.path.join(O.GOLDEN, "denoiser.npz"))


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def cases(z):
    for name in ("full", "temporal", "jbf16"):
        W, H, n, seed, jh, th, clamp = (int(v) for v in z[f"{name}_params"])
        step, tol, wgt = (float(v) for v in z[f"{name}_fparams"])
        yield name, W, H, n, seed, jh, th, clamp, tol, wgt


def test_camera_matrices_match_reference(fixture):
    for name, W, H, n, *_ in cases(fixture):
        for k in range(n):
            key = f"{name}_f{k + 1}"
            _, proj, view = rt.camera_look_ex(W, H, fixture[f"{key}_campos"], FWD)
            assert np.array_equal(bits(proj), bits(fixture[f"{key}_proj"])), key
            assert np.array_equal(bits(view), bits(fixture[f"{key}_view"])), key


def test_params_defaults_are_the_reference_members():
    p = rt.denoise_params()
    assert (p.jbf_half_size, p.temporal_half_size, p.immediate_clamp) == (7, 3, 1)
    assert np.float32(p.tolerance) == np.float32(1.0) and np.float32(p.current_frame_weighting) == np.float32(0.2)
    assert [np.float32(v) for v in (p.sigma_position, p.sigma_color, p.sigma_normal, p.sigma_coplanarity)] == \
           [np.float32(32.0), np.float32(0.6), np.float32(0.1), np.float32(0.1)]


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["lds32", "lds64", "global"])
@pytest.mark.parametrize("case", ["full", "temporal", "jbf16"])
def test_denoised_frames(fixture, case, path, monkeypatch):
    """path: the LDS-ring filter (jbf_lds_kernel, the default) with 8 x 32 or 8 x 64 pixel blocks
    (RT_JBF_TALL), or the direct-gather one (jbf_kernel, taken for windows wider than the ring;
    RT_JBF_GLOBAL forces it)"""
    if path == "global":
        monkeypatch.setenv("RT_JBF_GLOBAL", "1")
    else:
        monkeypatch.delenv("RT_JBF_GLOBAL", raising=False)
        monkeypatch.setenv("RT_JBF_TALL", path[3:])
    z = fixture
    name, W, H, n, seed, jh, th, clamp, tol, wgt = next(c for c in cases(z) if c[0] == case)
    ctx = rt.Context(0)
    try:
        ctx.upload(rt.Scene.cornell())
        ctx.resize(W, H)
        params = rt.denoise_params(jbf_half_size=jh, temporal_half_size=th, tolerance=tol, current_frame_weighting=wgt, immediate_clamp=clamp)
        for k in range(n):
            key = f"{name}_f{k + 1}"
            cam, proj, view = rt.camera_look_ex(W, H, z[f"{key}_campos"], FWD)
            rgba, out = ctx.render_denoised(cam, proj, view, k + 1, params, seed=seed)
            gb = ctx.gbuffer()
            prim = z[f"{key}_prim"]
            hit = prim != -1
            assert np.array_equal(gb["prim"], prim), key
            assert np.array_equal(hit.astype(np.int32), z[f"{key}_contrib"]), key
            assert np.array_equal(bits(gb["color"][..., :3]), bits(z[f"{key}_color"])), key
            assert np.array_equal(bits(gb["position"][..., :3][hit]), bits(z[f"{key}_pos"][hit])), key
            assert np.array_equal(bits(gb["normal"][..., :3][hit]), bits(z[f"{key}_nrm"][hit])), key
            if jh > 0:
                sp = gb["spatial"][..., :3]
                assert np.array_equal(bits(sp), bits(z[f"{key}_spatial"])), (key, float(np.mean(bits(sp) != bits(z[f"{key}_spatial"]))))
            assert np.array_equal(bits(out[..., :3]), bits(z[f"{key}_temporal"])), key
            assert np.array_equal(rgba, z[f"{key}_rgba"]), key
        st = ctx.stats()
        assert st.last_denoise_ms > 0.0
    finally:
        ctx.close()


@pytest.mark.gpu
def test_restart_drops_the_history(fixture):
    """Renderer::RestartTemporal (DN/Renderer.h:74-77): after a restart the next frame is not blended."""
    z = fixture
    name, W, H, n, seed, jh, th, clamp, tol, wgt = next(c for c in cases(z) if c[0] == "temporal")
    ctx = rt.Context(0)
    try:
        ctx.upload(rt.Scene.cornell())
        ctx.resize(W, H)
        params = rt.denoise_params(jbf_half_size=0, temporal_half_size=th, tolerance=tol, current_frame_weighting=wgt)
        cam, proj, view = rt.camera_look_ex(W, H, z[f"{name}_f1_campos"], FWD)
        ctx.render_denoised(cam, proj, view, 1, params, seed=seed)
        ctx.denoise_restart()
        cam, proj, view = rt.camera_look_ex(W, H, z[f"{name}_f2_campos"], FWD)
        _, out = ctx.render_denoised(cam, proj, view, 2, params, seed=seed)
        assert np.array_equal(bits(out[..., :3]), bits(z[f"{name}_f2_color"]))   # == this frame's G-buffer color
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sig", [(32.0, 0.6, 0.1, 0.1), (1.7, 0.23, 0.41, 0.05), (0.3, 2.5, 0.02, 0.9), (1e-4, 0.6, 0.1, 0.1)])
def test_markstein_divisions_equal_ieee(sig, monkeypatch):
    """The filter divides by 2 sigma^2 with Markstein's correction from the correctly rounded reciprocal
    (rt_denoise.hip jbf_div) when every divisor is in [2^-20, 2^20), the IEEE sequence otherwise.  The
    reference's sigmas are private constants (DN/Denoiser.h:353-356), so only the defaults have golden
    frames (test_denoised_frames); for other sigmas this checks the shortcut against the IEEE divisions
    on the same G-buffer (RT_JBF_IEEE), bit for bit -- the last set's 2e-8 divisor takes the IEEE path."""
    W, H = 96, 72
    sp, sc, sn, sk = sig
    out = []
    for ieee in (False, True):
        if ieee:
            monkeypatch.setenv("RT_JBF_IEEE", "1")
        else:
            monkeypatch.delenv("RT_JBF_IEEE", raising=False)
        c = rt.Context(0)
        try:
            c.upload(rt.Scene.cornell())
            c.resize(W, H)
            params = rt.denoise_params(jbf_half_size=7, temporal_half_size=0, sigma_position=sp, sigma_color=sc, sigma_normal=sn,
                                       sigma_coplanarity=sk)
            cam, proj, view = rt.camera_look_ex(W, H, rt.DEFAULT_CAMERA_POSITION, FWD)
            c.render_denoised(cam, proj, view, 1, params, seed=4)
            out.append(c.gbuffer()["spatial"][..., :3].copy())
        finally:
            c.close()
    assert np.array_equal(bits(out[0]), bits(out[1]))
