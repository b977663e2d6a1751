"""The near-first orderings' tree and order variants on the GPU (round 5): any tree over the reference's leaf
boxes and any visiting order give the reference's image, since the closest hit is taken by (min t, max DFS
triangle) and a leaf box's own slab test decides whether the reference reaches it (rt_scene.cpp near_first,
DESIGN.md 5.1 / 5.3).  Each variant builds its scene under its knobs (RT_WALK_TREE is read at the scene build)
and renders bitwise against the reference's fixtures:
  * C3 (Whitted, bunny + teapot) at its full 1280x960x64 with the product kernel (no work counters): the SAH
    tree's orderings (default), the reference tree's orderings (RT_WALK_TREE=0), the DFS walk (RT_WH_ORDER=0),
    SAH trees binned 2 and 1024 ways (RT_SAH_BINS: other trees over the same leaves);
  * C5 at 96x54x16 on the BVH variant with the reference tree's orderings (RT_WALK_TREE=0) and the 2- and
    1024-bin SAH trees."""
import hashlib
import os

import numpy as np
import pytest

from _rt import rt

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"RT_WALK_TREE": "0"}, {"RT_WH_ORDER": "0"}, {"RT_SAH_BINS": "2"}, {"RT_SAH_BINS": "1024"}],
                         ids=["sah-orders", "reference-tree-orders", "dfs", "sah-2-bins", "sah-1024-bins"])
def test_c3_full_frame_product_kernel(env, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    f = np.load(os.path.join(G, "bvh_scene.npz"))
    z = np.load(os.path.join(G, "bvh_images.npz"))
    sc = rt.Scene.bvh_tracer(f["raw_bunny"], f["raw_teapot"])
    assert sc.walk_orders(whitted=True) is not None   # built for every Whitted scene; RT_WH_ORDER=0 leaves them unused
    c = rt.Context(0)
    try:
        c.upload(sc)
        c.resize(1280, 960)
        rgba, acc = c.render(rt.camera_bvh_tracer(1280, 960), 64, whitted=True)
        assert c.stats().kernel == 2   # RT_KERNEL_WHITTED
    finally:
        c.close()
    assert hashlib.sha256(np.ascontiguousarray(acc).tobytes()).hexdigest() == str(z["sha_accum_1280x960_spp64"])
    assert hashlib.sha256(np.ascontiguousarray(rgba).tobytes()).hexdigest() == str(z["sha_rgba_1280x960_spp64"])


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"RT_WALK_TREE": "0"}, {"RT_SAH_BINS": "2"}, {"RT_SAH_BINS": "1024"}],
                         ids=["reference-tree-orders", "sah-2-bins", "sah-1024-bins"])
def test_c5_tree_variants(env, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    bunny = np.load(os.path.join(G, "bvh_scene.npz"))["raw_bunny"]
    sc = rt.Scene.cornell_c5(bunny)
    c = rt.Context(0)
    try:
        c.upload(sc)
        c.resize(96, 54)
        cam, _, _ = rt.camera_default(96, 54)
        rgba, acc = c.render(cam, 16, seed=0)
        assert c.stats().kernel == 3
    finally:
        c.close()
    fx = np.load(os.path.join(G, "c5_scene.npz"))
    assert np.array_equal(bits(acc), bits(fx["accum_96x54_spp16_s0"]))
    assert np.array_equal(rgba, fx["rgba_96x54_spp16_s0"])
