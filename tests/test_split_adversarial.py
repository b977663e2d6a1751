"""Adversarial scenes for the BVH variant's split trace (kernel 3, rt_coherent.hip), against
the oracle, bitwise.

The split trace tests the <= 32 leaves outside a walked subtree by their own boxes, walks the subtree, and
takes the closest hit by (min t, max DFS triangle) -- the reference's "later leaf wins ties" of
BVH::traverse_BVH_from_node (MC/BVH.h:97-100) -- and it drops shadow-ray candidates near-coplanar with the
sampled light triangle by the light-plane masks over its outside slots (rt_scene.cpp; MC/Renderer.cpp:172-189).
These scenes sit where the two shortcuts could go wrong:

* test_skip_adversarial.py's scene A (small quads at 0.5 / 0.9 / 0.99 eta below and above the light, tilted
  to |cos| ~ 0.9995; side walls whose shading points send shadow rays meeting the light at |cos| in
  [0.25, 0.3]), plus a 160-triangle tessellated block: 194 triangles, so the BVH variant runs and the split
  puts the block's subtree in the walk and the scene-A triangles among the outside leaves -- the near quads'
  masks then act in the split phase;
* coincident duplicate triangles with another material: copies of block-face triangles in meshes of their
  own, so that a copy among the outside leaves ties EXACTLY (same vertices, same t) with the walked subtree's
  original, both before the subtree in DFS order (the walked copy must win) and after it (the outside copy
  must win); one copy pair also lies wholly inside the walked subtree.  Every hit on these triangles is a tie,
  and the two materials (red / green against the block's white) make a wrong winner visible;
* the bound-fails variant: a far triangle makes 0.006 + 6e-5 x extent exceed 0.008, so no mask may be set
  (n_light_skip == 0) and the split runs without the skip."""
import numpy as np
import pytest

import _oracle as O
import test_skip_adversarial as A
from _rt import rt


def grid_face(p0, du, dv, n):
    """an n x n grid of quads (two triangles each, first vertex a right-angle corner) spanning p0 + [0,1]du + [0,1]dv"""
    out = []
    for i in range(n):
        for j in range(n):
            a = p0 + du * (i / n) + dv * (j / n)
            b = p0 + du * ((i + 1) / n) + dv * (j / n)
            c = p0 + du * ((i + 1) / n) + dv * ((j + 1) / n)
            d = p0 + du * (i / n) + dv * ((j + 1) / n)
            out.append(np.concatenate([a, b, c]))
            out.append(np.concatenate([c, d, a]))
    return np.array(out, np.float32)


def block_faces(n=4):
    x0, x1, y0, y1, z0, z1 = 360.0, 460.0, 0.0, 150.0, 280.0, 400.0
    P = lambda *v: np.array(v, np.float64)
    return {"front": grid_face(P(x0, y0, z0), P(x1 - x0, 0, 0), P(0, y1 - y0, 0), n),
            "back": grid_face(P(x1, y0, z1), P(x0 - x1, 0, 0), P(0, y1 - y0, 0), n),
            "left": grid_face(P(x0, y0, z1), P(0, 0, z0 - z1), P(0, y1 - y0, 0), n),
            "right": grid_face(P(x1, y0, z0), P(0, 0, z1 - z0), P(0, y1 - y0, 0), n),
            "top": grid_face(P(x0, y1, z0), P(x1 - x0, 0, 0), P(0, 0, z1 - z0), n)}


def split_scene(far=False):
    f = block_faces()
    block = np.concatenate(list(f.values()))
    dups = [("dup_front", f["front"][10:12]), ("dup_top", f["top"][20:22]), ("dup_left", f["left"][12:14]),
            ("dup_right", f["right"][6:8]), ("dup_back", f["back"][2:4])]
    base = A.scene_a(far=far)
    return (base[:-1] + [("block", block, A.WHITE, A.NOEM)] +
            [(nm, t, A.RED if k % 2 == 0 else A.GREEN, A.NOEM) for k, (nm, t) in enumerate(dups)] + base[-1:])


def layout(meshes):
    sc = A.build_rt(meshes)
    info = sc.info()
    nf, ni, tf, ti = sc.export()
    leaf = ni[:, 2] >= 0
    where = {}
    for k, (nm, _, _, _) in enumerate(meshes):
        idx = np.where(leaf & (ni[:, 3] == k))[0]
        where[nm] = (int(idx.min()), int(idx.max()))
    return sc, info, where


def test_split_tables_of_the_adversarial_scene():
    sc, info, where = layout(split_scene())
    r, e = info.split_root, info.split_end
    assert info.n_tris == 194 and info.n_leaf_boxes == 0   # > 64 triangles: the BVH variant
    assert r > 0 and e > r and info.n_split_leaves <= 32
    inside = lambda nm: r <= where[nm][0] and where[nm][1] < e
    assert inside("block") and not inside("near") and not inside("light")
    # ties across the split boundary in both DFS orders, and one pair wholly inside the walk
    outside_dups = [nm for nm in where if nm.startswith("dup_") and not inside(nm)]
    assert any(where[nm][1] < r for nm in outside_dups) and any(where[nm][0] >= e for nm in outside_dups)
    assert any(inside(nm) for nm in where if nm.startswith("dup_"))
    # the light-plane masks over the outside slots: each light triangle masks both light triangles and the
    # twelve near-coplanar quad triangles, as in the small scene A
    assert info.n_light_skip == 2 * 14, info.n_light_skip


def test_split_bound_fails_no_mask():
    _, info, _ = layout(split_scene(far=True))
    assert info.split_root > 0 and info.n_light_skip == 0


@pytest.mark.gpu
@pytest.mark.parametrize("far", [False, True])
@pytest.mark.parametrize("env", [{}, {"RT_SPLIT": "0"}, {"RT_FORCE_WALK": "1"}, {"RT_BVH_PREPASS": "0"}, {"RT_PRE_DEFER": "0"},
                                 {"RT_WALK_ORDER": "0"}])
def test_split_adversarial_matches_oracle(far, env, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    meshes = split_scene(far=far)
    W, H, spp, seed = 128, 96, 16, 5
    sc = A.build_rt(meshes)
    c = rt.Context(0)
    try:
        c.upload(sc)
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        rgba, acc = c.render(cam, spp, seed=seed)
        assert c.stats().kernel == 3   # RT_KERNEL_VERTEX_BVH: the split trace lives there
    finally:
        c.close()
    oacc, orgba, _ = O.Scene(meshes).render(W, H, spp, seed=seed)
    same = np.mean(np.all(A.bits(acc) == A.bits(oacc), axis=-1))
    assert np.array_equal(A.bits(acc), A.bits(oacc)), f"{same:.4%} of pixels bitwise equal"
    assert np.array_equal(rgba, orgba)


@pytest.mark.gpu
def test_scene_beyond_the_prepass_limit_takes_the_bvh_variant():
    """A scene of 2^19 triangles and more (the camera pre-pass records carry the triangle in 19 bits) still
    runs the vertex kernel's BVH variant, without the pre-pass (no megakernel fallback below
    2^31), bitwise against the oracle: the block of the adversarial split scene tessellated into 526,338
    triangles (a 513 x 513 grid on each of two faces) inside scene A"""
    def grid_fast(p0, du, dv, n):   # grid_face's triangles, vectorized
        i, j = [g.reshape(-1, 1) for g in np.meshgrid(np.arange(n), np.arange(n), indexing="ij")]
        P = lambda a, b: p0 + du * (a / n) + dv * (b / n)
        a, b, c, d = P(i, j), P(i + 1, j), P(i + 1, j + 1), P(i, j + 1)
        return np.stack([np.concatenate([a, b, c], 1), np.concatenate([c, d, a], 1)], 1).reshape(-1, 9).astype(np.float32)
    g0 = grid_fast(np.array([360.0, 0.0, 280.0]), np.array([100.0, 0.0, 0.0]), np.array([0.0, 150.0, 0.0]), 513)
    grid = np.concatenate([g0[: 263169], grid_fast(np.array([360.0, 150.0, 280.0]), np.array([100.0, 0.0, 0.0]), np.array([0.0, 0.0, 120.0]), 513)[: 263169]])
    base = A.scene_a()
    meshes = base[:-1] + [("grid", grid, A.WHITE, A.NOEM)] + base[-1:]
    sc = A.build_rt(meshes)
    assert sc.info().n_tris >= (1 << 19)
    W, H, spp, seed = 48, 36, 4, 3
    c = rt.Context(0)
    try:
        c.upload(sc)
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        rgba, acc = c.render(cam, spp, seed=seed)
        st = c.stats()
        assert st.kernel == 3 and st.last_prepass_ms == 0.0
    finally:
        c.close()
    oacc, orgba, _ = O.Scene(meshes).render(W, H, spp, seed=seed)
    assert np.array_equal(A.bits(acc), A.bits(oacc))
    assert np.array_equal(rgba, orgba)


@pytest.mark.gpu
def test_light_tables_beyond_lds_take_the_megakernel():
    """The BVH variant keeps the materials and light tables in LDS (rt_capi.cpp kMaxBvhSmallLds): a scene whose
    light is a 3200-triangle mesh (its tables ~200 KB) renders on the megakernel instead, bitwise against the
    oracle"""
    base = A.scene_a()
    light = grid_face(np.array([213.0, A.LY, 227.0]), np.array([130.0, 0.0, 0.0]), np.array([0.0, 0.0, 105.0]), 40)
    meshes = base[:-1] + [("light", light, base[-1][2], base[-1][3])]
    W, H, spp, seed = 48, 36, 4, 9
    sc = A.build_rt(meshes)
    assert sc.info().n_light_tris == 3200
    c = rt.Context(0)
    try:
        c.upload(sc)
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        rgba, acc = c.render(cam, spp, seed=seed)
        st = c.stats()
        assert st.kernel == 0   # RT_KERNEL_MEGA
        assert st.kernel_reason == rt.KERNEL_REASON_TABLES_LDS   # the fallback is visible to the caller
    finally:
        c.close()
    oacc, orgba, _ = O.Scene(meshes).render(W, H, spp, seed=seed)
    assert np.array_equal(A.bits(acc), A.bits(oacc))
    assert np.array_equal(rgba, orgba)
