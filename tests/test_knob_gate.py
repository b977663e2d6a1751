"""The library's A/B and diagnostic knobs (RT_VERTEX, RT_SPLIT, RT_STACK_DEPTH, ...) are read
from the environment only behind RT_DEBUG_KNOBS=1 (csrc/rt_knobs.h): a stray RT_* variable in a product
caller's environment must not switch a kernel."""
import pytest

from _rt import rt


def render_kernel(W=32, H=24):
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        c.render(cam, 2, seed=1)
        return c.stats().kernel
    finally:
        c.close()


@pytest.mark.gpu
def test_knobs_ignored_without_the_gate(monkeypatch):
    monkeypatch.delenv("RT_DEBUG_KNOBS", raising=False)
    monkeypatch.setenv("RT_VERTEX", "0")          # would select the megakernel
    monkeypatch.setenv("RT_STACK_DEPTH", "4")     # would force a tiny fold ring
    assert render_kernel() == 1                   # the vertex kernel, the product default


@pytest.mark.gpu
def test_knobs_read_with_the_gate(monkeypatch):
    monkeypatch.setenv("RT_DEBUG_KNOBS", "1")
    monkeypatch.setenv("RT_VERTEX", "0")
    assert render_kernel() == 0                   # RT_KERNEL_MEGA


def test_scene_knobs_ignored_without_the_gate(monkeypatch):
    """The scene build's knobs (RT_WALK_TREE, RT_SAH_BINS) too: without the gate the near-first orderings are
    the default SAH tree's whatever the variables say (host code only, no GPU)."""
    import os
    import numpy as np
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bvh_scene.npz"))
    monkeypatch.setenv("RT_DEBUG_KNOBS", "1")
    base = rt.Scene.bvh_tracer(z["raw_bunny"], z["raw_teapot"]).walk_orders(whitted=True)
    monkeypatch.setenv("RT_SAH_BINS", "2")
    monkeypatch.setenv("RT_WALK_TREE", "0")
    bits = lambda a: np.ascontiguousarray(a).view(np.uint32)   # (the orderings hold NaN fields: compare bits)
    assert not np.array_equal(bits(rt.Scene.bvh_tracer(z["raw_bunny"], z["raw_teapot"]).walk_orders(whitted=True)), bits(base))
    monkeypatch.delenv("RT_DEBUG_KNOBS")
    assert np.array_equal(bits(rt.Scene.bvh_tracer(z["raw_bunny"], z["raw_teapot"]).walk_orders(whitted=True)), bits(base))
