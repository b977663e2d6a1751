"""The split trace's near-first walk orders (rt_scene.cpp FlatScene::wcopies, rt_scene_walk_orders; DESIGN.md
5.1), on the CPU.

A split scene's walked subtree is stored in 8 pre-orders, one per ray-direction octant, each visiting the
nearer child first -- of the reference's subtree itself (RT_WALK_TREE=0) or (default) of a binned-SAH tree
built over the subtree's leaves (the same leaf boxes and triangles, internal boxes their unions).  The kernel
walks them stacklessly (hit: next node, miss or leaf: the node's skip pointer) and ends when the pointer reads
n_nodes.  The GPU tests check the images bitwise (test_c5.py, test_split_adversarial.py); these check the
tables themselves: every ordering holds the subtree's leaves exactly once (and, for the reference's tree, its
internal nodes too), every internal box contains its children's (so a leaf box's own slab test decides
whether the walk reaches it), its skip pointers describe a well-formed pre-order that ends at n_nodes, and a
walk under any box predicate reaches the same leaves as the reference's DFS walk of the subtree -- the
kernel keeps the closest hit by (min t, max DFS triangle), so neither the tree nor the visit order changes
its result."""
import numpy as np
import pytest

import test_split_adversarial as SA
from _rt import rt


def original(sc):
    """the DFS pre-order's nodes as (boxes (n, 6), skip (n,), tri (n,)) from rt_scene_export"""
    nf, ni, _, _ = sc.export()
    n = len(nf)
    size = np.ones(n, np.int64)
    for i in range(n - 1, -1, -1):   # children follow their parent in pre-order
        if ni[i, 2] < 0:
            size[i] = 1 + size[ni[i, 0]] + size[ni[i, 1]]
    return nf[:, :6].copy(), np.arange(n) + size, ni[:, 2].copy()


def copy_fields(W, octant):
    """one ordering's (boxes as lo.xyz hi.xyz, skip, tri) from its rows, whose boxes are stored as the octant's
    (near.xyz, far.xyz) planes: axis a's planes are (hi, lo) when bit a of the octant (d_a < 0) is set"""
    near, far = W[:, 0:3], W[:, 3:6]
    neg = np.array([(octant >> a) & 1 for a in range(3)], bool)
    lo = np.where(neg, far, near)
    hi = np.where(neg, near, far)
    return np.concatenate([lo, hi], axis=1), W[:, 6].view(np.int32).astype(np.int64), W[:, 7].view(np.int32).astype(np.int64)


def walk(boxes, skip, tri, start, stop, base, hit):
    """the kernel's stackless walk: leaves reached, and nodes visited (indices are absolute; row = index - base)"""
    ti, leaves, visits = start, [], 0
    while ti < stop:
        k = ti - base
        visits += 1
        h = hit(boxes[k])
        if h and tri[k] < 0:
            ti += 1
        else:
            if h:
                leaves.append(int(tri[k]))
            ti = int(skip[k])
    return leaves, visits


def slab(o, d):
    inv = np.divide(1.0, d, out=np.full(3, np.inf), where=d != 0)
    def hit(b):
        t1 = (b[:3] - o) * inv
        t2 = (b[3:] - o) * inv
        lo = np.nanmax(np.minimum(t1, t2))
        hi = np.nanmin(np.maximum(t1, t2))
        return hi >= max(lo, 0.0)
    return hit


def check_orders(sc, n_rays, seed, same_tree, whitted=False):
    info = sc.info()
    NN = info.n_nodes
    r, e = (0, NN) if whitted else (info.split_root, info.split_end)
    assert whitted or r > 0
    boxes, skip, tri = original(sc)
    Wall = sc.walk_orders(whitted=whitted)
    M = e - r
    assert Wall.shape == (8, M, 8)
    rows_of = lambda b, t, m: np.sort(np.concatenate([b[m], t[m, None].astype(np.float32)], axis=1).view(np.uint32), axis=0)
    sub_tri = tri[r:e]
    ref_rows = rows_of(boxes[r:e], sub_tri, np.ones(len(sub_tri), bool) if same_tree else sub_tri >= 0)
    rng = np.random.default_rng(seed)
    lo, hi = boxes[r, :3].astype(np.float64), boxes[r, 3:].astype(np.float64)
    for oct_ in range(8):
        bx, sk, tr = copy_fields(Wall[oct_], oct_)
        # the same leaves (box, triangle), each once; for the reference's tree every node
        assert len(bx) == M
        rows = rows_of(bx, tr, np.ones(M, bool) if same_tree else tr >= 0)
        assert np.array_equal(rows, ref_rows)
        # a well-formed pre-order: a leaf's skip is the next row, an internal node's first child is the next
        # row and its second child's skip equals its own; every pointer stays in [r + 1, e) or reads NN
        idx = r + np.arange(M)
        sk_in = np.where(sk == NN, e, sk)
        assert np.all((sk_in > idx) & (sk_in <= e))
        leaf = tr >= 0
        assert np.all(sk_in[leaf] == idx[leaf] + 1)
        inner = np.where(~leaf)[0]
        right = sk_in[inner + 1]
        assert np.all(right < sk_in[inner])
        assert np.all(sk_in[right - r] == sk_in[inner])
        assert sk[0] == NN   # the walk ends at n_nodes
        # every internal box contains both children's boxes (float compares: exact containment)
        first, second = inner + 1, right - r
        for ch in (first, second):
            assert np.all(bx[inner, :3] <= bx[ch, :3]) and np.all(bx[inner, 3:] >= bx[ch, 3:])
        # everything hit: all M nodes in row order
        leaves, visits = walk(bx, sk, tr, r, NN, r, lambda b: True)
        assert visits == M and len(leaves) == int(leaf.sum())
    # rays through the subtree's box: the ordering of the ray's octant reaches the DFS walk's leaves (with the
    # same boxes tested when the tree is the reference's)
    for _ in range(n_rays):
        tgt = lo + (hi - lo) * rng.random(3)
        o = tgt + rng.normal(size=3) * (hi - lo).max()
        d = tgt - o
        d /= np.linalg.norm(d)
        oct_ = int(d[0] < 0) | int(d[1] < 0) << 1 | int(d[2] < 0) << 2
        hit = slab(o, d)
        ref_leaves, ref_visits = walk(boxes, skip, tri, r, e, 0, hit)
        bx, sk, tr = copy_fields(Wall[oct_], oct_)
        leaves, visits = walk(bx, sk, tr, r, NN, r, hit)
        assert sorted(leaves) == sorted(ref_leaves)
        if same_tree:
            assert visits == ref_visits


@pytest.mark.parametrize("walk_tree", ["0", "1"], ids=["reference-subtree", "sah-tree"])
def test_walk_orders_of_the_adversarial_split_scene(walk_tree, monkeypatch):
    monkeypatch.setenv("RT_WALK_TREE", walk_tree)
    sc = SA.A.build_rt(SA.split_scene())
    check_orders(sc, n_rays=300, seed=1, same_tree=walk_tree == "0")


@pytest.mark.parametrize("walk_tree", ["0", "1"], ids=["reference-subtree", "sah-tree"])
def test_walk_orders_of_c5(walk_tree, monkeypatch):
    monkeypatch.setenv("RT_WALK_TREE", walk_tree)
    bvh = np.load(SA.A.__file__.replace("test_skip_adversarial.py", "golden/bvh_scene.npz"))
    sc = rt.Scene.cornell_c5(bvh["raw_bunny"])
    check_orders(sc, n_rays=40, seed=2, same_tree=walk_tree == "0")


def test_small_scenes_have_no_walk_orders():
    assert rt.Scene.cornell().walk_orders() is None
    assert rt.Scene.cornell().walk_orders(whitted=True) is None


@pytest.mark.parametrize("walk_tree", ["0", "1"], ids=["reference-tree", "sah-tree"])
def test_whitted_orders_of_c3(walk_tree, monkeypatch):
    """C3's whole tree (bunny + teapot, point lights) in the Whitted kernel's 8 near-first orderings
    (rt_whitted.hip whitted_traverse; closest hit by (min t, max DFS triangle))."""
    monkeypatch.setenv("RT_WALK_TREE", walk_tree)
    z = np.load(SA.A.__file__.replace("test_skip_adversarial.py", "golden/bvh_scene.npz"))
    sc = rt.Scene.bvh_tracer(z["raw_bunny"], z["raw_teapot"])
    assert sc.walk_orders() is None   # no split: the path tracer's vertex kernel does not walk this scene
    check_orders(sc, n_rays=30, seed=3, same_tree=walk_tree == "0", whitted=True)


def test_whitted_half_orders_contain_the_float_boxes():
    """The Whitted kernel's 16-byte orderings (rt_scene.cpp compact_orderings): node for node the float orderings'
    structure (skip of an internal node, triangle of a leaf, whose successor is the next node), and every half
    plane rounded OUTWARD -- the near plane toward the ray's origin side and the far plane away, i.e. a low plane
    down and a high plane up -- so the decoded box contains the exact box (the walk visits a superset; leaves are
    then tested on their exact vertex boxes, rt_whitted.hip walk_half)."""
    z = np.load(SA.A.__file__.replace("test_skip_adversarial.py", "golden/bvh_scene.npz"))
    sc = rt.Scene.bvh_tracer(z["raw_bunny"], z["raw_teapot"])
    fo = sc.walk_orders(whitted=True)
    ho = sc.whitted_orders_half()
    assert ho is not None and ho.shape[:2] == fo.shape[:2]
    fi = np.ascontiguousarray(fo).view(np.int32)
    skip, tri = fi[..., 6], fi[..., 7]
    leaf = tri >= 0
    w3 = ho[..., 3]
    assert np.array_equal(w3[leaf] & 0x7FFFFFFF, tri[leaf].astype(np.uint32)) and np.all(w3[leaf] >> 31 == 1)
    assert np.array_equal(w3[~leaf], skip[~leaf].astype(np.uint32))
    k = np.arange(fo.shape[1])
    assert np.all((skip == k[None, :] + 1)[leaf])   # a leaf's successor is the next node
    half = lambda w: (w & 0xFFFF).astype(np.uint16).view(np.float16).astype(np.float32)
    for a in range(3):
        neg = ((np.arange(8) >> a) & 1).astype(bool)[:, None]
        near_h, far_h = half(ho[..., a]), half(ho[..., a] >> 16)
        near_f, far_f = fo[..., a], fo[..., 3 + a]
        lo_ok = np.where(neg, far_h <= far_f, near_h <= near_f)    # the low plane rounded down
        hi_ok = np.where(neg, near_h >= near_f, far_h >= far_f)    # the high plane rounded up
        assert np.all(lo_ok) and np.all(hi_ok), a
        # and by at most one half-ulp (the nearest half, stepped once when on the wrong side)
        err = np.abs(near_h.astype(np.float64) - near_f) / np.maximum(np.abs(near_f.astype(np.float64)), 2.0 ** -14)
        assert float(err.max()) <= 2.0 ** -10


@pytest.mark.parametrize("bins", ["2", "1024"])
def test_sah_bins_build_other_trees(bins, monkeypatch):
    """RT_SAH_BINS (the A/B knob of the SAH build's bins per axis) builds another tree over the same leaves: its
    orderings differ from the default 16-bin tree's and still give the reference's leaf set for every ray
    (test_walk_variants_gpu.py renders with them)."""
    z = np.load(SA.A.__file__.replace("test_skip_adversarial.py", "golden/bvh_scene.npz"))
    base = rt.Scene.bvh_tracer(z["raw_bunny"], z["raw_teapot"]).walk_orders(whitted=True)
    monkeypatch.setenv("RT_SAH_BINS", bins)
    sc = rt.Scene.bvh_tracer(z["raw_bunny"], z["raw_teapot"])
    other = sc.walk_orders(whitted=True)
    bits = lambda a: np.ascontiguousarray(a).view(np.uint32)   # (the orderings hold NaN fields: compare bits)
    assert other.shape == base.shape and not np.array_equal(bits(other), bits(base))
    check_orders(sc, n_rays=20, seed=4, same_tree=False, whitted=True)
