"""Whitted::Sphere entities in the path-traced scene: the reference's Entity extension point,
MC/Entity.h:19-55 / MC/Sphere.h:16-108, through Renderer::Add + GenerateBVH (MC/Renderer.h:78-86).

The fixture tests/golden/cornell_spheres.npz comes from the reference's OWN Sphere, BVH, TriangleMesh and camera
code (oracle/_ref/ref_harness, `oracle/gen_golden.py spheres`): the Cornell box plus four spheres (one white on
the floor, one green above the short box, one white half inside the tall box, one with the light's emissive
material near the ceiling), its flattened two-level tree, 4096 closest hits and three images.

CPU: the host builder's tree (rt_scene_add_sphere + rt_scene_build) against the reference's, node for node, and
the scene-API errors.  GPU: closest hits (slot and double t) and the float4 accumulation, bit for bit, on the
megakernel (rt_stats.kernel_reason == RT_KERNEL_REASON_SPHERES)."""
import os

import numpy as np
import pytest

import _oracle as O
from _rt import rt

G = O.GOLDEN
FX = os.path.join(G, "cornell_spheres.npz")
ALBEDO = [(0.63, 0.065, 0.05), (0.1, 0.5, 0.1), (0.7, 0.7, 0.7), (0.7, 0.7, 0.7)]   # red, green, white, light (MC/Renderer.cpp:28-35)
EMISSION = [(0, 0, 0), (0, 0, 0), (0, 0, 0), (47.8, 38.6, 31.1)]


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64 if a.dtype == np.float64 else a.dtype)


def scene(fx):
    s = rt.Scene()
    s._check(rt.lib().rt_scene_add_cornell_box(s.h), "rt_scene_add_cornell_box")
    for c, r, m in zip(fx["spheres_center"], fx["spheres_radius"], fx["spheres_material"]):
        s.add_sphere(c, float(r), ALBEDO[int(m)], EMISSION[int(m)])
    return s.build()


@pytest.fixture(scope="module")
def fx():
    return np.load(FX)


def test_tree_matches_reference(fx):
    import importlib.util
    spec = importlib.util.spec_from_file_location("gg", os.path.join(O.ORACLE_DIR, "gen_golden.py"))
    gg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gg)
    nodes, tris = fx["nodes"].view(gg.NODE_DT), fx["tris"].view(gg.TRI_DT)
    s = scene(fx)
    info = s.info()
    assert info.n_spheres == 4 and info.n_meshes == 10
    assert info.n_leaf_boxes == 0 and info.split_root == 0   # the triangle-only structures are not built
    nf, ni, tf, ti = s.export()
    assert nf.shape[0] == len(nodes) and tf.shape[0] == len(tris)
    assert np.array_equal(bits(nf[:, 0:3]), bits(nodes["mn"])) and np.array_equal(bits(nf[:, 3:6]), bits(nodes["mx"]))
    assert np.array_equal(bits(nf[:, 6]), bits(nodes["area"]))   # a sphere leaf's area: 4 * PI * r^2 (MC/Sphere.h:22)
    for k, col in (("left", 0), ("right", 1), ("tri", 2), ("mesh", 3), ("top", 4)):
        assert np.array_equal(ni[:, col], nodes[k]), k
    for k, sl in (("a", slice(0, 3)), ("b", slice(3, 6)), ("c", slice(6, 9)), ("n", slice(9, 12))):
        assert np.array_equal(bits(tf[:, sl]), bits(tris[k])), k
    assert np.array_equal(bits(tf[:, 12]), bits(tris["area"]))
    sph = ti[:, 1] == -2   # rt_scene_export marks a sphere's slot
    assert int(sph.sum()) == 4 and np.array_equal(ti[:, 0], tris["mesh"])


def test_scene_api_errors(fx):
    # the first emissive entity may not be a sphere: SamplingAreaLight would call the empty Sphere::Sampling
    s = rt.Scene()
    s.add_sphere((1.0, 1.0, 1.0), 0.5, (0.7, 0.7, 0.7), (5.0, 5.0, 5.0))
    s._check(rt.lib().rt_scene_add_cornell_box(s.h), "rt_scene_add_cornell_box")
    assert rt.lib().rt_scene_build(s.h) == -1   # RT_ERR_INVALID
    s = rt.Scene()
    with pytest.raises(rt.RtError):
        s.add_sphere((1.0, 1.0, 1.0), 0.0, (0.7, 0.7, 0.7))
    with pytest.raises(rt.RtError):
        s.add_sphere((1.0, 1.0, 1.0), float("nan"), (0.7, 0.7, 0.7))


@pytest.mark.gpu
def test_closest_hits_match_reference(fx):
    s = scene(fx)
    c = rt.Context(0)
    try:
        c.upload(s)
        tri, t = c.trace(fx["org"], fx["dir"])
    finally:
        c.close()
    hit = fx["hit"] == 1
    assert np.array_equal(tri >= 0, hit)
    assert np.array_equal(tri[hit], fx["tri"][hit])
    assert np.array_equal(bits(t[hit]), bits(fx["t"][hit]))
    # a sphere's hit: t is its float root (the record's double holds a float), location ray(t), normal
    # Whitted::normalize(location - center) (MC/Sphere.h:89-94)
    _, _, tf, ti = s.export()
    on = hit & (ti[np.maximum(tri, 0), 1] == -2)
    assert on.sum() > 1000
    t32 = fx["t"][on].astype(np.float32)
    assert np.array_equal(t32.astype(np.float64), fx["t"][on])
    o, d = fx["org"][on], fx["dir"][on]
    loc = (o + t32[:, None] * d).astype(np.float32)
    assert np.array_equal(bits(loc), bits(fx["loc"][on]))


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["128x128_spp64_s0_rr0.8", "96x72_spp16_s3_rr0.5", "64x48_spp32_s11_rr0.9"])
def test_images_match_reference(fx, key):
    dims, sppk, sk, rrk = key.split("_")
    W, H = (int(v) for v in dims.split("x"))
    spp, seed, rr = int(sppk[3:]), int(sk[1:]), float(rrk[2:])
    c = rt.Context(0)
    try:
        c.upload(scene(fx))
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        rgba, acc = c.render(cam, spp, seed=seed, rr=rr)
        st = c.stats()
    finally:
        c.close()
    assert st.kernel == 0 and st.kernel_reason == rt.KERNEL_REASON_SPHERES
    assert np.array_equal(bits(acc), bits(fx[f"accum_{key}"]))
    assert np.array_equal(np.ascontiguousarray(rgba).view(np.uint32).reshape(H, W), fx[f"rgba_{key}"])
