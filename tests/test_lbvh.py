"""The BVH built on the device (rt_upload_scene_gpu_bvh, csrc/rt_lbvh.hip): a Karras LBVH as a non-parity
fast path for large meshes (the reference builds on the host, MC/BVH.h:131-214).

CPU: the same algorithm run on the host (rt_scene_lbvh_host) gives a well-formed tree in the traversal
layout -- DFS pre-order with skip pointers, every internal box the exact union of its children's, every
leaf box its triangle's vertex box, the triangle records a permutation of the scene's.
GPU: the device tree equals the host tree bit for bit; rays find the same closest t as on the reference
tree (the Moller-Trumbore operations do not depend on the tree; a tie between two triangles at one t may
resolve to the other triangle); the C5 96x54x16 accumulation is the reference's wherever no such tie
occurs (parity against the reference fixture, measured, not assumed)."""
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
def scenes():
    raw = np.load(os.path.join(G, "bvh_scene.npz"))["raw_bunny"]
    return {"cornell": rt.Scene.cornell(), "c5": rt.Scene.cornell_c5(raw)}


def check_tree(nodes, tris, tf, ti):
    n = tris.shape[0]
    m = nodes.shape[0]
    assert m == 2 * n - 1
    skip = nodes[:, 6].view(np.int32)
    tri = nodes[:, 7].view(np.int32)
    leaf = tri >= 0
    # leaves in DFS order carry triangles 0..n-1 in order; a leaf's skip is the next node
    assert np.array_equal(tri[leaf], np.arange(n))
    assert np.array_equal(skip[leaf], np.nonzero(leaf)[0] + 1)
    assert skip[0] == m
    # internal node i: left child i + 1, right child skip[i + 1], subtree ends at skip[i] == skip[right]
    inner = np.nonzero(~leaf)[0]
    lc = inner + 1
    rc = skip[lc]
    assert np.all(rc < m) and np.array_equal(skip[rc], skip[inner])
    lo, hi = nodes[:, 0:3], np.concatenate([nodes[:, 3:4], nodes[:, 4:6]], axis=1)
    assert np.array_equal(bits(lo[inner]), bits(np.minimum(lo[lc], lo[rc])))
    assert np.array_equal(bits(hi[inner]), bits(np.maximum(hi[lc], hi[rc])))
    # the records are the scene's (a, material, e1 = b - a, e2 = c - a, n), permuted; leaf box = vertex box
    a, b, c = tf[:, 0:3], tf[:, 3:6], tf[:, 6:9]
    ref = np.concatenate([a, ti[:, 0:1].view(np.float32), b - a, c - a, tf[:, 9:12]], axis=1)
    got = np.concatenate([tris[:, 0:4], tris[:, 4:7], tris[:, 8:11], tris[:, 12:15]], axis=1)
    key = lambda x: np.lexsort(bits(x).T[::-1])
    assert np.array_equal(bits(got[key(got)]), bits(ref[key(ref)]))
    vb = {bits(ref[i]).tobytes(): (np.minimum(np.minimum(a[i], b[i]), c[i]), np.maximum(np.maximum(a[i], b[i]), c[i])) for i in range(len(ref))}
    leaves = np.nonzero(leaf)[0]
    for k in range(0, n, max(1, n // 2000)):
        vlo, vhi = vb[bits(got[k]).tobytes()]
        assert np.array_equal(bits(lo[leaves[k]]), bits(vlo)) and np.array_equal(bits(hi[leaves[k]]), bits(vhi))


@pytest.mark.parametrize("name", ["cornell", "c5"])
def test_host_tree_is_well_formed(scenes, name):
    sc = scenes[name]
    nodes, tris = sc.lbvh_host()
    _, _, tf, ti = sc.export()
    check_tree(nodes, tris, tf, ti)
    n2, t2 = sc.lbvh_host()
    assert np.array_equal(bits(nodes), bits(n2)) and np.array_equal(bits(tris), bits(t2))


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell", "c5"])
def test_device_tree_equals_host_tree(scenes, name):
    sc = scenes[name]
    nodes, tris = sc.lbvh_host()
    c = rt.Context(0)
    ms = c.upload_gpu_bvh(sc)
    dn, dt = c.debug_scene_arrays(nodes.shape[0], tris.shape[0])
    c.close()
    assert np.array_equal(bits(dn), bits(nodes))
    assert np.array_equal(bits(dt), bits(tris))
    print(f"{name}: {tris.shape[0]} triangles, device build {ms:.3f} ms")


def negzero_scene():
    """Triangles whose centroids sit at x = -0.0 (every vertex x is -0.0) in waves of
    their own, and triangles at negative x: the device's centroid-bound atomics must order -0.0 above every
    negative float (rt_lbvh.hip atomic_min_f), as the host's fminf does."""
    rng = np.random.default_rng(7)
    neg = rng.uniform(-100.0, -50.0, (64, 9)).astype(np.float32)
    neg[:, 1::3] = rng.uniform(0, 500, (64, 3)); neg[:, 2::3] = rng.uniform(0, 500, (64, 3))
    nz = rng.uniform(0, 500, (256, 9)).astype(np.float32)
    nz[:, 0::3] = np.float32(-0.0)
    sc = rt.Scene()   # (no +0.0 coordinate anywhere: unions of +-0 are not ordered alike by every fminf)
    sc.add_mesh(np.concatenate([neg, nz]), (0.5, 0.5, 0.5), (0.0, 0.0, 0.0))
    return sc.build()


def test_host_tree_with_negative_zero_centroids_is_well_formed():
    sc = negzero_scene()
    nodes, tris = sc.lbvh_host()
    _, _, tf, ti = sc.export()
    check_tree(nodes, tris, tf, ti)


@pytest.mark.gpu
def test_device_tree_equals_host_tree_with_negative_zero_centroids():
    sc = negzero_scene()
    nodes, tris = sc.lbvh_host()
    c = rt.Context(0)
    try:
        c.upload_gpu_bvh(sc)
        dn, dt = c.debug_scene_arrays(nodes.shape[0], tris.shape[0])
    finally:
        c.close()
    assert np.array_equal(bits(dn), bits(nodes))
    assert np.array_equal(bits(dt), bits(tris))


@pytest.mark.gpu
def test_rays_and_image_match_reference_tree(scenes):
    sc = scenes["c5"]
    fx = np.load(os.path.join(G, "c5_scene.npz"))
    info = sc.info()
    ref = rt.Context(0)
    ref.upload(sc)
    _, ref_tris = ref.debug_scene_arrays(info.n_nodes, info.n_tris)
    c = rt.Context(0)
    c.upload_gpu_bvh(sc)
    _, gpu_tris = c.debug_scene_arrays(2 * info.n_tris - 1, info.n_tris)
    tri_r, t_r = ref.trace(fx["ray_org"], fx["ray_dir"])
    tri_g, t_g = c.trace(fx["ray_org"], fx["ray_dir"])
    assert np.array_equal(tri_r >= 0, tri_g >= 0)
    hit = tri_r >= 0
    assert np.array_equal(bits(t_r[hit]), bits(t_g[hit]))
    # the same primitive (record word 7) unless two triangles tie at t
    pid_r = ref_tris[tri_r[hit], 7].view(np.int32)
    pid_g = gpu_tris[tri_g[hit], 7].view(np.int32)
    assert np.mean(pid_r != pid_g) <= 1e-3
    print(f"rays: {hit.sum()} hits, t bitwise equal, {int((pid_r != pid_g).sum())} resolved to another triangle at a tie")
    c.resize(96, 54)
    cam, _, _ = rt.camera_default(96, 54)
    rgba, acc = c.render(cam, 16, seed=0)
    assert c.stats().kernel == 3   # the BVH variant walks the device-built tree
    same = np.all(bits(acc) == bits(fx["accum_96x54_spp16_s0"]), axis=-1)
    assert same.mean() >= 0.999, same.mean()
    print(f"96x54x16 accumulation: {same.mean() * 100:.3f} % of pixels bitwise equal to the reference's")
    ref.close()
    c.close()
