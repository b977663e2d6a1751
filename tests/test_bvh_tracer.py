"""The reference's BVH Ray Tracer (config C3: Whitted shading of the Stanford bunny and the Utah
teapot with two point lights, BV/ = "BVH Ray Tracer/8599RayTracerGUI/src/") against golden vectors
from oracle/_ref/ref_whitted_bvh (the reference's own BVH / triangle-mesh / camera code compiled from
/root/reference, shading glue restated; generator oracle/gen_golden.py).

The renderer is deterministic (no RNG), so every check is bit-exact: the host BVH build (SHA-256 of
the flattened topology and geometry), the camera matrices, 4096 closest-hit rays, the float4
accumulation of two small images, and the SHA-256 of the full C3 accumulation (1280x960, 64 spp)."""
import hashlib
import importlib.util
import os

import numpy as np
import pytest

import _oracle as O
from _rt import rt

G = O.GOLDEN


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64 if a.dtype == np.float64 else a.dtype)


def gen_golden():
    spec = importlib.util.spec_from_file_location("gg", os.path.join(O.ORACLE_DIR, "gen_golden.py"))
    gg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gg)
    return gg


@pytest.fixture(scope="module")
def fixture():
    return np.load(os.path.join(G, "bvh_scene.npz"))


@pytest.fixture(scope="module")
def scene(fixture):
    return rt.Scene.bvh_tracer(fixture["raw_bunny"], fixture["raw_teapot"])


def exported_records(scene):
    """Our flattened scene as the harness's NODE_DT / TRI_DT records."""
    gg = gen_golden()
    nf, ni, tf, ti = scene.export()
    nodes = np.zeros(nf.shape[0], gg.NODE_DT)
    nodes["mn"], nodes["mx"], nodes["area"] = nf[:, 0:3], nf[:, 3:6], nf[:, 6]
    for k, col in (("left", 0), ("right", 1), ("tri", 2), ("mesh", 3), ("top", 4)):
        nodes[k] = ni[:, col]
    tris = np.zeros(tf.shape[0], gg.TRI_DT)
    for k, sl in (("a", slice(0, 3)), ("b", slice(3, 6)), ("c", slice(6, 9)), ("n", slice(9, 12))):
        tris[k] = tf[:, sl]
    tris["mesh"] = ti[:, 0]
    return gg, nodes, tris


def test_scene_build_matches_reference(scene, fixture):
    gg, nodes, tris = exported_records(scene)
    assert len(nodes) == int(fixture["n_nodes"]) == 22575 and len(tris) == int(fixture["n_tris"]) == 11288
    head = fixture["nodes_head"].view(gg.NODE_DT)
    for f in gg.BV_NODE_FIELDS:
        assert np.array_equal(bits(nodes[f][: len(head)]), bits(head[f])), f
    assert gg.scene_digest(nodes, tris) == str(fixture["digest"])


def test_camera_matches_reference():
    z = np.load(os.path.join(G, "bvh_images.npz"))
    for (W, H) in ((16, 12), (1280, 960)):
        cam = rt.camera_bvh_tracer(W, H)
        mats = z[f"mats_{W}x{H}"]   # proj, inv proj, view, inv view (column-major)
        assert np.array_equal(bits(np.array(cam.inv_projection, np.float32)), bits(mats[1].reshape(16)))
        assert np.array_equal(bits(np.array(cam.inv_view, np.float32)), bits(mats[3].reshape(16)))
        assert np.array_equal(bits(np.array(cam.position, np.float32)), bits(z[f"vec_{W}x{H}"][:3]))


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def ctx(scene):
    c = rt.Context(0)
    c.upload(scene)
    yield c
    c.close()


@pytest.mark.gpu
def test_closest_hit_rays(ctx):
    z = np.load(os.path.join(G, "bvh_rays.npz"))
    tri, t = ctx.trace(z["org"], z["dir"])
    hit = z["hit"] != 0
    assert np.array_equal(tri >= 0, hit)
    assert np.array_equal(tri[hit], z["tri"][hit])
    assert np.array_equal(bits(t[hit]), bits(z["t"][hit]))


def render(ctx, W, H, spp, first_frame=1, band=8, rank=0, nranks=1, count=False):
    ctx.resize(W, H, band, rank, nranks)
    cam = rt.camera_bvh_tracer(W, H)
    return ctx.render(cam, spp, first_frame=first_frame, whitted=True, count=count)


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,spp", [(160, 120, 3), (97, 61, 2)])
def test_small_images_bitwise(ctx, W, H, spp):
    z = np.load(os.path.join(G, "bvh_images.npz"))
    rgba, acc = render(ctx, W, H, spp)
    key = f"{W}x{H}_spp{spp}"
    assert np.array_equal(bits(acc), bits(z[f"accum_{key}"]))
    assert np.array_equal(rgba, z[f"rgba_{key}"])


@pytest.mark.gpu
def test_c3_full_image_digest(ctx):
    """C3 as BASELINE.json names it: 1280x960, 64 spp; the accumulation and RGBA8 frame are
    compared by SHA-256 with the reference's."""
    z = np.load(os.path.join(G, "bvh_images.npz"))
    rgba, acc = render(ctx, 1280, 960, 64, count=True)
    assert hashlib.sha256(np.ascontiguousarray(acc).tobytes()).hexdigest() == str(z["sha_accum_1280x960_spp64"])
    assert hashlib.sha256(np.ascontiguousarray(rgba).tobytes()).hexdigest() == str(z["sha_rgba_1280x960_spp64"])
    st = ctx.stats()
    rays_per_pixel_frame = st.rays / (1280 * 960 * 64)
    ref = z["stats_1280x960_spp64"]
    assert abs(rays_per_pixel_frame - ref[0] / ref[1]) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("half", ["1", "0"], ids=["half-nodes", "float-nodes"])
def test_c3_full_image_node_formats(scene, monkeypatch, half):
    """The 32-byte float orderings (the product) and, with RT_WH_HALF=1, the upload of the 16-byte half-plane
    orderings (round 6, rt_whitted.hip walk_half: outward-rounded boxes, exact leaf boxes from the vertices; walked by
    a -DRT_WH_HALF=1 build, an A/B measured -3 %) give the reference's C3 frame bit for bit on the product
    (non-counting) kernel."""
    z = np.load(os.path.join(G, "bvh_images.npz"))
    monkeypatch.setenv("RT_WH_HALF", half)
    c = rt.Context(0)
    try:
        c.upload(scene)
        rgba, acc = render(c, 1280, 960, 64)
    finally:
        c.close()
    assert hashlib.sha256(np.ascontiguousarray(acc).tobytes()).hexdigest() == str(z["sha_accum_1280x960_spp64"])
    assert hashlib.sha256(np.ascontiguousarray(rgba).tobytes()).hexdigest() == str(z["sha_rgba_1280x960_spp64"])


@pytest.mark.gpu
def test_incremental_and_row_bands(ctx):
    """Render(+1 spp) x3 == one 3-spp launch; a 3-rank band split reassembles to the same bits."""
    z = np.load(os.path.join(G, "bvh_images.npz"))
    W, H = 160, 120
    for f in (1, 2, 3):
        rgba, acc = render(ctx, W, H, 1, first_frame=f)
    assert np.array_equal(bits(acc), bits(z[f"accum_{W}x{H}_spp3"]))
    full = np.zeros((H, W, 4), np.float32)
    for r in range(3):
        _, a = render(ctx, W, H, 3, band=4, rank=r, nranks=3)
        rows = [y for b in range(r, (H + 3) // 4, 3) for y in range(b * 4, min(b * 4 + 4, H))]
        full[rows] = a
    assert np.array_equal(bits(full), bits(z[f"accum_{W}x{H}_spp3"]))
