"""Configuration C5: the Cornell box plus a synthesized 79,488-triangle mesh (the
Stanford bunny subdivided 1:4 twice, `c5_mesh`), added through the reference's own TriangleMesh + BVH
(MC/TriangleMesh.h:148-186, MC/Renderer.h:78-86, MC/BVH.h:131-214) -- a 159,039-node tree that no
longer fits in LDS, so the megakernel traverses it from HBM/L2/MALL.

Golden vectors: tests/golden/c5_scene.npz from oracle/_ref/ref_harness (the reference's BVH, triangle,
material and camera code; oracle/gen_golden.py `c5`).  Everything is bit-exact: the host BVH build
(SHA-256 of the flattened tree), 4096 closest-hit rays, the float4 accumulation of a 96x54x16 image,
and the SHA-256 of the full 3840x2160 frame at 1 spp."""
import hashlib
import os

import numpy as np
import pytest

import _oracle as O
from _rt import rt

G = O.GOLDEN


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64 if a.dtype == np.float64 else a.dtype)


@pytest.fixture(scope="module")
def fixture():
    return np.load(os.path.join(G, "c5_scene.npz"))


@pytest.fixture(scope="module")
def bunny_raw():
    return np.load(os.path.join(G, "bvh_scene.npz"))["raw_bunny"]


@pytest.fixture(scope="module")
def scene(bunny_raw):
    return rt.Scene.cornell_c5(bunny_raw)


def test_asset_is_the_reference_input(bunny_raw, fixture):
    raw = rt.c5_mesh(bunny_raw)
    assert raw.shape == (79488, 9)
    assert hashlib.sha256(raw.tobytes()).hexdigest() == str(fixture["raw_sha"])


def test_subdivision_is_watertight_and_area_preserving(bunny_raw):
    sub = rt.subdivide_midpoint(bunny_raw[:50], 1).reshape(-1, 3, 3).astype(np.float64)
    src = np.ascontiguousarray(bunny_raw[:50]).reshape(-1, 3, 3).astype(np.float64)
    area = lambda t: 0.5 * np.linalg.norm(np.cross(t[:, 1] - t[:, 0], t[:, 2] - t[:, 0]), axis=1)
    assert np.allclose(area(sub).reshape(-1, 4).sum(1), area(src), rtol=1e-5)
    # the four children of a triangle share exactly its vertices and edge midpoints
    assert np.array_equal(sub[0::4, 0], src[:, 0]) and np.array_equal(sub[1::4, 1], src[:, 1]) and np.array_equal(sub[2::4, 2], src[:, 2])


def test_scene_build_matches_reference(scene, fixture):
    import importlib.util
    spec = importlib.util.spec_from_file_location("gg", os.path.join(O.ORACLE_DIR, "gen_golden.py"))
    gg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gg)
    nf, ni, tf, ti = scene.export()
    nodes = np.zeros(nf.shape[0], gg.NODE_DT)
    nodes["mn"], nodes["mx"], nodes["area"] = nf[:, 0:3], nf[:, 3:6], nf[:, 6]
    for k, col in (("left", 0), ("right", 1), ("tri", 2), ("mesh", 3), ("top", 4)):
        nodes[k] = ni[:, col]
    tris = np.zeros(tf.shape[0], gg.TRI_DT)
    for k, sl in (("a", slice(0, 3)), ("b", slice(3, 6)), ("c", slice(6, 9)), ("n", slice(9, 12))):
        tris[k] = tf[:, sl]
    tris["mesh"] = ti[:, 0]
    assert len(nodes) == int(fixture["n_nodes"]) == 159039 and len(tris) == int(fixture["n_tris"]) == 79520
    head = fixture["nodes_head"].view(gg.NODE_DT)
    for f in gg.NODE_DT.names:
        assert np.array_equal(bits(nodes[f][: len(head)]), bits(head[f])), f
    assert gg.scene_digest(nodes, tris) == str(fixture["digest"])


def test_split_trace_tables(scene):
    """The split trace's host tables (rt_scene.cpp): the walked subtree is the deepest one leaving at most
    32 leaves outside it -- in C5 the bunny's mesh subtree, with the Cornell box's 32 triangles outside --
    the outside leaves are exactly the leaves outside [split_root, split_end), every one inside all its
    ancestor boxes, and the subtree's root box inside every ancestor's (leaf-box monotonicity)."""
    info = scene.info()
    nf, ni, tf, ti = scene.export()
    r, e = info.split_root, info.split_end
    assert r > 0 and e > r and info.n_split_leaves == 32 and 0 < info.n_split_boxes <= 32   # <= 32 outside leaves
    leaf = ni[:, 2] >= 0
    assert int(leaf[:r].sum() + leaf[e:].sum()) == info.n_split_leaves
    inside = ni[r:e, 2][leaf[r:e]]
    assert set(ti[inside, 0].tolist()) == {int(np.argmax(np.bincount(ti[:, 0])))}   # the bunny mesh only
    # a node's subtree is [k, k + size): the ancestors of node i are the internal nodes k < i whose subtree
    # covers it; their boxes contain node i's
    n = len(nf)
    size = np.ones(n, np.int64)
    for k in range(n - 1, -1, -1):
        if ni[k, 2] < 0:
            size[k] = 1 + size[ni[k, 0]] + size[ni[k, 1]]
    assert r + size[r] == e
    for i in [r] + [k for k in range(n) if leaf[k] and not (r <= k < e)]:
        anc = [k for k in range(i) if ni[k, 2] < 0 and k + size[k] > i]
        for k in anc:
            assert np.all(nf[k, 0:3] <= nf[i, 0:3]) and np.all(nf[k, 3:6] >= nf[i, 3:6]), (i, k)
    # the small Cornell scene has its leaf-box table instead, no split; the light-plane skip masks of the
    # split's outside slots (rt_scene.cpp) mark as many candidates as the Cornell box's own (its light's two
    # triangles and the ceiling's two, per light triangle)
    c = rt.Scene.cornell().info()
    assert c.split_root == 0 and c.n_split_leaves == 0 and c.n_leaf_boxes > 0
    assert info.n_light_skip == c.n_light_skip == 8


def test_oracle_small_image(bunny_raw, fixture):
    meshes = O.cornell_meshes() + [("c5", rt.c5_mesh(bunny_raw), np.array([0.7, 0.7, 0.7], np.float32), np.zeros(3, np.float32))]
    acc, rgba, _ = O.Scene(meshes).render(96, 54, 16, seed=0, threads=min(8, os.cpu_count() or 1))
    assert np.array_equal(bits(acc), bits(fixture["accum_96x54_spp16_s0"]))
    assert np.array_equal(rgba, fixture["rgba_96x54_spp16_s0"])


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def ctx(scene):
    c = rt.Context(0)
    c.upload(scene)
    yield c
    c.close()


@pytest.mark.gpu
def test_closest_hit_rays(ctx, fixture):
    tri, t = ctx.trace(fixture["ray_org"], fixture["ray_dir"])
    hit = fixture["ray_hit"] != 0
    assert np.array_equal(tri >= 0, hit)
    assert np.array_equal(tri[hit], fixture["ray_tri"][hit])
    assert np.array_equal(bits(t[hit]), bits(fixture["ray_t"][hit]))


@pytest.mark.gpu
def test_small_image_bitwise(ctx, fixture):
    ctx.resize(96, 54)
    cam, _, _ = rt.camera_default(96, 54)
    rgba, acc = ctx.render(cam, 16, seed=0, count=True)
    assert np.array_equal(bits(acc), bits(fixture["accum_96x54_spp16_s0"]))
    assert np.array_equal(rgba, fixture["rgba_96x54_spp16_s0"])
    st = ctx.stats()
    ref = fixture["stats_96x54_spp16_s0"]   # rays, draws, shading calls, overflow, samples
    assert st.rays == int(ref[0])           # the same rays are traced as in the reference
    _, fast = ctx.render(cam, 16, seed=0, exact=False)
    a = np.clip(fast[..., :3] / 16, 0, 1).astype(np.float64)
    b = np.clip(fixture["accum_96x54_spp16_s0"][..., :3] / 16, 0, 1).astype(np.float64)
    assert float(np.sqrt(np.mean((a - b) ** 2))) < 1e-4


@pytest.mark.gpu
def test_full_frame_digest(ctx, fixture):
    """The C5 frame at its full 3840x2160 size (1 spp): accumulation and RGBA8 by SHA-256."""
    ctx.resize(3840, 2160)
    cam, _, _ = rt.camera_default(3840, 2160)
    rgba, acc = ctx.render(cam, 1, seed=0)
    assert hashlib.sha256(np.ascontiguousarray(acc).tobytes()).hexdigest() == str(fixture["sha_accum_3840x2160_spp1_s0"])
    assert hashlib.sha256(np.ascontiguousarray(rgba).tobytes()).hexdigest() == str(fixture["sha_rgba_3840x2160_spp1_s0"])


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"RT_RING_PACK": "0"}, {"RT_RING_PACK": "1"},
                                 {"RT_SPLIT": "0"}, {"RT_FORCE_WALK": "1"}, {"RT_THRESH": "0", "RT_STEPS": "1"},
                                 {"RT_THRESH": "64"}, {"RT_BVH_PREPASS": "0"}, {"RT_BVH_PREPASS": "0", "RT_FORCE_WALK": "1"},
                                 {"RT_PRE_DEFER": "0"}, {"RT_WALK_ORDER": "0"}, {"RT_WALK_ORDER": "0", "RT_BVH_PREPASS": "0"}])
def test_vertex_bvh_variant_bitwise(scene, fixture, env, monkeypatch):
    """The vertex kernel's BVH variant (the C5 path) on the reference's 96x54x16 accumulation, with the
    fold-level materials in their own array or in the direct term's sign bits, and
    with the materials and light tables in LDS (default) or read from HBM; the camera rays traced by the
    split scene's pre-pass (default; the rays that enter the walked subtree's box are recorded as camera rays
    and traced by the path kernel, RT_PRE_DEFER=0: walked by the pre-pass) or by the path kernel itself
    (RT_BVH_PREPASS=0).  The split trace (default:
    the 32 Cornell leaves by their boxes, the bunny's subtree walked; closest hit by (min t, max
    triangle); the subtree walked in the near-first ordering of the ray's direction octant, or in the
    reference's DFS order with RT_WALK_ORDER=0) against the whole-tree walk (RT_SPLIT=0), the reference's
    per-lane traversal for every ray (RT_FORCE_WALK=1: the split's non-finite-direction path), and extreme
    round shapes"""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    c = rt.Context(0)
    c.upload(scene)
    c.resize(96, 54)
    cam, _, _ = rt.camera_default(96, 54)
    rgba, acc = c.render(cam, 16, seed=0)
    assert c.stats().kernel == 3   # RT_KERNEL_VERTEX_BVH
    assert np.array_equal(bits(acc), bits(fixture["accum_96x54_spp16_s0"]))
    assert np.array_equal(rgba, fixture["rgba_96x54_spp16_s0"])
    c.close()
