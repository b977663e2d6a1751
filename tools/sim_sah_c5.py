#!/usr/bin/env python3
"""Design study: box tests per walking ray on C5's walked subtree (the bunny) for the reference's median-split
tree and for a binned-SAH tree over the SAME leaf boxes, both walked as the BVH variant walks them -- a stackless
pre-order walk in the near-first ordering of the ray's direction octant, boxes entered beyond the bound skipped
(closest hit: the best t so far; shadow rays: the light distance, the first blocking hit ends them).

Any tree whose internal boxes contain their children's gives the reference's candidate set for finite rays (the
leaf box decides), and the closest hit is taken by (min t, max reference DFS triangle), so the tree
is free; this measures what a better one saves.

    python tools/sim_sah_c5.py [--rays 800]
"""
import argparse
import importlib.util
import json
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_rt():
    spec = importlib.util.spec_from_file_location("rt", os.path.join(REPO, "cpu-based-ray-tracer_amd", "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


class Flat:
    """A binary tree as arrays: lo, hi (n, 3), left, right, tri (-1 internal)."""

    def __init__(self, lo, hi, left, right, tri):
        self.lo, self.hi, self.left, self.right, self.tri = lo, hi, left, right, tri


def subtree(nf, ni, root, end):
    idx = np.arange(root, end)
    lo, hi = nf[idx, 0:3].astype(np.float64), nf[idx, 3:6].astype(np.float64)
    left = np.where(ni[idx, 2] < 0, ni[idx, 0] - root, -1)
    right = np.where(ni[idx, 2] < 0, ni[idx, 1] - root, -1)
    return Flat(lo, hi, left, right, ni[idx, 2].copy())


def build_sah(leaf_lo, leaf_hi, leaf_tri, bins=16, max_leaf=1):
    """Binned SAH over centroids (1 primitive per leaf: the same node count as the reference's subtree)."""
    n = len(leaf_tri)
    cen = 0.5 * (leaf_lo + leaf_hi)
    lo, hi, left, right, tri = [], [], [], [], []

    def area(bl, bh):
        e = np.maximum(bh - bl, 0.0)
        return 2.0 * (e[..., 0] * e[..., 1] + e[..., 1] * e[..., 2] + e[..., 2] * e[..., 0])

    def new(bl, bh):
        lo.append(bl); hi.append(bh); left.append(-1); right.append(-1); tri.append(-1)
        return len(lo) - 1

    stack = [(np.arange(n), None)]
    root = None
    while stack:
        ids, parent_slot = stack.pop()
        bl, bh = leaf_lo[ids].min(0), leaf_hi[ids].max(0)
        me = new(bl, bh)
        if parent_slot is not None:
            p, side = parent_slot
            (left if side == 0 else right)[p] = me
        else:
            root = me
        if len(ids) <= max_leaf:
            tri[me] = int(leaf_tri[ids[0]])
            continue
        c = cen[ids]
        cl, ch = c.min(0), c.max(0)
        best = (np.inf, None, None)
        for ax in range(3):
            if ch[ax] <= cl[ax]:
                continue
            if len(ids) <= 2 * bins:
                order = np.argsort(c[:, ax], kind="stable")
                s = ids[order]
                pl = np.minimum.accumulate(leaf_lo[s], 0); ph = np.maximum.accumulate(leaf_hi[s], 0)
                sl = np.minimum.accumulate(leaf_lo[s][::-1], 0)[::-1]; sh = np.maximum.accumulate(leaf_hi[s][::-1], 0)[::-1]
                k = np.arange(1, len(s))
                cost = area(pl[k - 1], ph[k - 1]) * k + area(sl[k], sh[k]) * (len(s) - k)
                j = int(np.argmin(cost))
                if cost[j] < best[0]:
                    best = (cost[j], s[: j + 1], s[j + 1:])
                continue
            b = np.minimum(((c[:, ax] - cl[ax]) / (ch[ax] - cl[ax]) * bins).astype(np.int64), bins - 1)
            cnt = np.bincount(b, minlength=bins)
            blo = np.full((bins, 3), np.inf); bhi = np.full((bins, 3), -np.inf)
            np.minimum.at(blo, b, leaf_lo[ids]); np.maximum.at(bhi, b, leaf_hi[ids])
            pl = np.minimum.accumulate(blo, 0); ph = np.maximum.accumulate(bhi, 0)
            sl = np.minimum.accumulate(blo[::-1], 0)[::-1]; sh = np.maximum.accumulate(bhi[::-1], 0)[::-1]
            pc = np.cumsum(cnt); sc = np.cumsum(cnt[::-1])[::-1]
            for k in range(1, bins):
                if pc[k - 1] == 0 or sc[k] == 0:
                    continue
                cost = area(pl[k - 1], ph[k - 1]) * pc[k - 1] + area(sl[k], sh[k]) * sc[k]
                if cost < best[0]:
                    m = b < k
                    best = (cost, ids[m], ids[~m])
        if best[1] is None:   # all centroids equal: split in half
            h = len(ids) // 2
            best = (0, ids[:h], ids[h:])
        stack.append((best[2], (me, 1)))
        stack.append((best[1], (me, 0)))
    return Flat(np.array(lo), np.array(hi), np.array(left), np.array(right), np.array(tri)), root


def ordering(T, root, octant):
    """Pre-order with, at every internal node, the child whose centre is nearer along the axis separating the
    two centres most (for the octant's direction signs) first; returns node order and skip pointers."""
    order, skip = [], {}
    st = [root]
    pos = {}
    while st:
        i = st.pop()
        pos[i] = len(order)
        order.append(i)
        if T.tri[i] < 0:
            l, r = T.left[i], T.right[i]
            cl = 0.5 * (T.lo[l] + T.hi[l]); cr = 0.5 * (T.lo[r] + T.hi[r])
            ax = int(np.argmax(np.abs(cr - cl)))
            neg = (octant >> ax) & 1
            first, second = (l, r) if ((cl[ax] <= cr[ax]) != bool(neg)) else (r, l)
            st.append(second)
            st.append(first)
    n = len(order)
    # skip pointer of node at position p: the position after its subtree
    size = {}
    for i in reversed(order):
        size[i] = 1 if T.tri[i] >= 0 else 1 + size[T.left[i]] + size[T.right[i]]
    return np.array(order), np.array([pos[i] + size[i] for i in order]), n


def walk(T, order, skipp, o, d, tris, bound0, shadow):
    inv = 1.0 / d
    lo, hi = T.lo[order], T.hi[order]
    t0 = (lo - o) * inv; t1 = (hi - o) * inv
    tin = np.max(np.minimum(t0, t1), 1); tout = np.min(np.maximum(t0, t1), 1)
    hit = (tout >= 0) & (tin <= tout)
    leaf = T.tri[order] >= 0
    best = np.inf
    p, n, tests, leaves = 0, len(order), 0, 0
    while p < n:
        tests += 1
        bnd = bound0 if shadow else best
        if hit[p] and tin[p] <= bnd * 1.00001 + 1e-5:
            if leaf[p]:
                leaves += 1
                t = tris(T.tri[order[p]], o, d)
                if shadow and t < bound0:
                    return tests, leaves, t
                if t < best:
                    best = t
                p = skipp[p]
            else:
                p += 1
        else:
            p = skipp[p]
    return tests, leaves, best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=800)
    args = ap.parse_args()
    rt = load_rt()
    sc = rt.Scene.cornell_c5(np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz"))["raw_bunny"])
    info = sc.info()
    nf, ni, tf, ti = sc.export()
    R, E = info.split_root, info.split_end
    ref = subtree(nf, ni, R, E)
    leaf = ref.tri >= 0
    sah, sroot = build_sah(ref.lo[leaf], ref.hi[leaf], ref.tri[leaf])
    print(json.dumps({"subtree_nodes": E - R, "sah_nodes": len(sah.tri)}), flush=True)
    A, B, C = tf[:, 0:3].astype(np.float64), tf[:, 3:6].astype(np.float64), tf[:, 6:9].astype(np.float64)

    def tri_t(k, o, d):
        e1, e2 = B[k] - A[k], C[k] - A[k]
        p = np.cross(d, e2); det = e1 @ p
        if abs(det) < 1e-14:
            return np.inf
        inv = 1.0 / det
        s = o - A[k]; u = (s @ p) * inv
        q = np.cross(s, e1); v = (d @ q) * inv; t = (e2 @ q) * inv
        return t if (u > 0 and v > 0 and u + v < 1 and t > 0) else np.inf

    ords = {}
    for name, T, root in (("reference", ref, 0), ("sah", sah, sroot)):
        ords[name] = (T, [ordering(T, root, o) for o in range(8)])
    rng = np.random.default_rng(3)
    blo, bhi = ref.lo[0], ref.hi[0]
    stats = {k: {"camera_or_bounce": [0, 0, 0], "shadow": [0, 0, 0]} for k in ords}
    lc = np.array([2.78, 5.487, 2.795])
    nr = 0
    while nr < args.rays:
        # rays that enter the bunny's box: from random room points toward random points of the bunny box
        o = rng.uniform([0, 0, 0], [5.56, 5.488, 5.592])
        tgt = rng.uniform(blo, bhi)
        d = tgt - o
        d /= np.linalg.norm(d)
        res = {}
        for name, (T, od) in ords.items():
            oc = int(d[0] < 0) | (int(d[1] < 0) << 1) | (int(d[2] < 0) << 2)
            order, skipp, _ = od[oc]
            tests, leaves, best = walk(T, order, skipp, o, d, tri_t, np.inf, False)
            res[name] = best
            s = stats[name]["camera_or_bounce"]; s[0] += tests; s[1] += leaves; s[2] += 1
            if np.isfinite(best):
                p = o + best * d - 1e-5 * d
                lp = lc + np.array([rng.uniform(-0.6, 0.6), 0, rng.uniform(-0.5, 0.5)]) if name == "reference" else lp
                sd = lp - p; sl = np.linalg.norm(sd)
                sdir = sd / sl
                oc2 = int(sdir[0] < 0) | (int(sdir[1] < 0) << 1) | (int(sdir[2] < 0) << 2)
                order, skipp, _ = od[oc2]
                tests, leaves, _ = walk(T, order, skipp, p, sdir, tri_t, sl - 0.01, True)
                s = stats[name]["shadow"]; s[0] += tests; s[1] += leaves; s[2] += 1
        assert res["reference"] == res["sah"], res
        nr += 1
    out = {k: {kind: {"box_tests": round(v[0] / max(v[2], 1), 2), "leaf_tests": round(v[1] / max(v[2], 1), 2), "rays": v[2]}
               for kind, v in s.items()} for k, s in stats.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
