"""EXACT fold-stack overflow and the device primitives that take shortcuts.

* Renderer::shading recurses until Russian roulette stops it (MC/Renderer.cpp:193); at RR 0.9 (a UI
  setting, MC/mainloop.cpp:96-100) deep paths are common enough that a fixed fold ring overflows.  A
  deliberately tiny ring (RT_STACK_DEPTH) forces thousands of overflows: the vertex kernel lists those
  samples and resample_kernel renders them again, so the image must stay bitwise equal to the oracle;
  the megakernel (G-buffer / counter renders) must fail with RT_ERR_OVERFLOW instead of returning a
  wrong image.
* Moller-Trumbore with its float pre-screen (MC/TriangleMesh.h:19-45) and the three slab-test forms
  (MC/BoundingVolume.h:173-215) on the reference's own edge-case fixtures (zero-area triangles,
  parallel rays, zero and axis-aligned directions, NaN slabs), run on the device.
"""
import os

import numpy as np
import pytest

import _oracle as O
from _rt import rt

pytestmark = pytest.mark.gpu
G = O.GOLDEN


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64 if a.dtype == np.float64 else a.dtype)


def context(**env):
    """A context created with knobs in the environment (read by rt_create)."""
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        c = rt.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    c.upload(rt.Scene.cornell())
    return c


@pytest.mark.parametrize("brute,kernel", [(1, 1), (0, 3)], ids=["leaf-box variant", "bvh variant"])
def test_ring_overflow_is_resampled_exactly(brute, kernel):
    W, H, spp, seed, rr = 48, 36, 24, 4, 0.9
    c = context(RT_STACK_DEPTH=3, RT_BRUTE=brute)
    try:
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        rgba, acc = c.render(cam, spp, seed=seed, rr=rr)
        st = c.stats()
        assert st.kernel == kernel and st.stack_depth == 3
        print(f"resampled {st.resampled} of {W * H * spp} samples")
        assert st.resampled > 100 and st.overflow_lost == 0 and st.stack_overflows == st.resampled
        oacc, orgba, _ = O.Scene().render(W, H, spp, seed=seed, rr=rr)
        assert np.array_equal(bits(acc), bits(oacc))
        assert np.array_equal(rgba, orgba)
    finally:
        c.close()


def test_ring_overflow_across_passes():
    # the parked-sample budget splits the render into 4 launches; each pass lists and re-renders its own overflows
    W, H, spp, seed, rr = 160, 120, 64, 2, 0.9
    c = context(RT_STACK_DEPTH=4, RT_LBUF_BUDGET_MB=4)
    try:
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        rgba, acc = c.render(cam, spp, seed=seed, rr=rr)
        st = c.stats()
        assert st.n_passes >= 3 and st.resampled > 1000 and st.overflow_lost == 0
        oacc, _, _ = O.Scene().render(W, H, spp, seed=seed, rr=rr)
        assert np.array_equal(bits(acc), bits(oacc))
    finally:
        c.close()


def test_default_ring_at_rr_0_9_needs_no_resample():
    c = context()
    try:
        c.resize(64, 48)
        cam, _, _ = rt.camera_default(64, 48)
        rgba, acc = c.render(cam, 32, seed=1, rr=0.9)
        st = c.stats()
        assert st.stack_depth >= 300 and st.resampled == 0 and st.overflow_lost == 0
        oacc, _, _ = O.Scene().render(64, 48, 32, seed=1, rr=0.9)
        assert np.array_equal(bits(acc), bits(oacc))
    finally:
        c.close()


def test_megakernel_stack_overflow_fails_loudly():
    c = context(RT_STACK_DEPTH=2, RT_VERTEX=0, RT_LDS_LEVELS=0)
    try:
        c.resize(48, 36)
        cam, _, _ = rt.camera_default(48, 36)
        with pytest.raises(rt.RtError, match="overflow"):
            c.render(cam, 24, seed=4, rr=0.9)
        assert c.stats().overflow_lost > 0
    finally:
        c.close()


def test_overflow_of_an_earlier_async_render_is_reported():
    """the overflow outcome accumulates over asynchronous renders until a synchronisation reads
    it -- a clean second render must not mask the first one's loss."""
    c = context(RT_STACK_DEPTH=2, RT_VERTEX=0, RT_LDS_LEVELS=0)
    try:
        c.resize(48, 36)
        cam, _, _ = rt.camera_default(48, 36)
        c.render(cam, 24, seed=4, rr=0.9, fetch=False)   # loses levels
        c.render(cam, 4, seed=5, rr=0.0, fetch=False)    # rr 0: every path ends at its first vertex, no level
        with pytest.raises(rt.RtError, match="overflow"):
            c.sync()
        assert c.stats().overflow_lost > 0
        # read: the next check is clean again
        c.render(cam, 4, seed=5, rr=0.0, fetch=False)
        c.sync()
        with pytest.raises(rt.RtError, match="overflow"):   # and the read-back entry point reports it too
            c.render(cam, 24, seed=4, rr=0.9, fetch=False)
            c.accumulation()
    finally:
        c.close()


def test_device_primitives_match_reference_fixtures():
    c = rt.Context(0)
    try:
        zm = np.load(os.path.join(G, "mt_cases.npz"))
        zb = np.load(os.path.join(G, "aabb_cases.npz"))
        mh, mt, bh = c.debug_primitives(zm["cases"], zb["cases"])
        assert np.array_equal(mh, zm["hit"])
        hit = zm["hit"] == 1
        assert 0.05 < hit.mean() < 0.95
        assert np.array_equal(bits(mt[hit]), bits(zm["t"][hit]))
        # the std::max/min form on every case; the finite-reciprocal forms where the kernels use them
        assert np.array_equal(bh[:, 0], zb["hit"])
        fin = bh[:, 1] >= 0
        assert np.array_equal(fin, bh[:, 2] >= 0)
        assert 0 < (~fin).sum() < fin.sum()   # the fixture has non-finite reciprocals (zero / axis-aligned directions)
        assert np.array_equal(bh[fin, 1], zb["hit"][fin])
        assert np.array_equal(bh[fin, 2], zb["hit"][fin])
    finally:
        c.close()
