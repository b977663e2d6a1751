"""The vertex kernel's exact shortcuts against their A/B switches, bit for bit.

* The direct term's two divisions, (X / dist^2) / light PDF, on Markstein's path (rt_coherent.hip, rt_device.h
  div2_core; each division inside div_fast's verified domain: numerator in [2^-100, 2^100), divisor in
  [2^-20, 2^20)) against RT_DIRECT_DIV2=0 (the IEEE division sequence): the same accumulation, and both equal
  to the reference's golden image.  Until round 6 the host computed the range flag before the light PDF was
  set, so the shortcut never ran.
* The camera pre-pass's sky bits (a camera miss parks nothing; the finalize adds the night sky) against
  RT_SKY_BITS=0 (misses parked as samples) and the pixel-major parked-sample layout (RT_LBUF_PIXEL_MAJOR=1),
  across a render forced into several passes whose frame counts are not multiples of 32, all against the
  megakernel (RT_VERTEX=0), which has neither."""
import os

import numpy as np
import pytest

import _oracle as O
from _rt import rt

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _render(monkeypatch, env, W, H, spp, seed, first_frame=1, rr=0.8):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        rgba, acc = c.render(cam, spp, first_frame=first_frame, seed=seed, rr=rr)
        return rgba, acc, c.stats()
    finally:
        c.close()
        for k in env:
            monkeypatch.delenv(k)


def test_direct_term_division_shortcut_is_exact(monkeypatch):
    g = np.load(os.path.join(O.GOLDEN, "images_cornell.npz"))
    for key in (k for k in g.files if k.startswith("accum_")):   # accum_<W>x<H>_spp<n>_s<seed>_rr<rr>
        _, dims, sppk, sk, rrk = key.split("_")
        W, H = (int(v) for v in dims.split("x"))
        spp, seed, rr = int(sppk[3:]), int(sk[1:]), float(rrk[2:])
        ref = np.ascontiguousarray(g[key], np.float32)
        _, a_on, st_on = _render(monkeypatch, {}, W, H, spp, seed, rr=rr)
        _, a_off, st_off = _render(monkeypatch, {"RT_DIRECT_DIV2": "0"}, W, H, spp, seed, rr=rr)
        assert st_on.kernel == 1 and st_off.kernel == 1   # the leaf-box vertex kernel, where the shortcut lives
        assert np.array_equal(bits(a_on), bits(ref)), key
        assert np.array_equal(bits(a_off), bits(ref)), key
    # a larger frame, every roulette setting of the reference UI: shortcut on == off
    for rr in (0.5, 0.8, 0.9):
        _, x, _ = _render(monkeypatch, {}, 192, 128, 40, 5, rr=rr)
        _, y, _ = _render(monkeypatch, {"RT_DIRECT_DIV2": "0"}, 192, 128, 40, 5, rr=rr)
        assert np.array_equal(bits(x), bits(y)), rr


def test_sky_bits_and_parked_layouts_across_passes(monkeypatch):
    W, H = 96, 64
    # 100 frames from frame 1 and 45 more from frame 101: neither a multiple of 32; a 1 MB budget forces passes
    ref = [_render(monkeypatch, {"RT_VERTEX": "0"}, W, H, n, 7, first_frame=ff)[1] for ff, n in ((1, 100), (101, 45))]
    # the sky is in view: some camera rays miss (else the sky bits would not be exercised)
    _, a1, _ = _render(monkeypatch, {"RT_VERTEX": "0"}, W, H, 1, 7)
    sky = np.array([12 / 255.0, 20 / 255.0, 69 / 255.0], np.float32)
    assert np.any(np.all(a1[..., :3] == sky, axis=-1))
    for env in ({}, {"RT_SKY_BITS": "0"}, {"RT_LBUF_PIXEL_MAJOR": "1"}, {"RT_SKY_BITS": "0", "RT_LBUF_PIXEL_MAJOR": "1"}):
        for (ff, n), r in zip(((1, 100), (101, 45)), ref):
            _, a, st = _render(monkeypatch, dict(env, RT_LBUF_BUDGET_MB="1"), W, H, n, 7, first_frame=ff)
            assert st.kernel == 1 and st.n_passes > 1, (env, ff, st.n_passes)
            assert np.array_equal(bits(a), bits(r)), (env, ff)
        # and in one pass
        _, a, st = _render(monkeypatch, env, W, H, 100, 7)
        assert st.kernel == 1 and st.n_passes == 1
        assert np.array_equal(bits(a), bits(ref[0])), env
