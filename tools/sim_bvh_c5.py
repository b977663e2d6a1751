#!/usr/bin/env python3
"""Node-visit counts of C5's rays under alternative BVH traversals (design study for the BVH variant).

The reference visits every node whose box the ray hits (MC/BVH.h:82-101), in DFS order, with no pruning
by the best hit so far; the vertex kernel's BVH variant does the same walk (skip pointers).  This counts,
on the exported C5 tree (rt_scene_export) and path-like rays (camera rays, cosine bounces from their hits,
shadow rays to the light):
  all      -- box tests of the reference's walk (every child of a hit internal node)
  dfs_prune-- the same DFS order, a hit internal node not descended when its entry t > best t
  ord_prune-- near child first (by entry t), pruned by best t (a stack walk)
  wide4    -- ord_prune counted in 4-wide node fetches (the binary tree collapsed two levels)
Closest-hit rays prune at best t; shadow rays at the light distance (any hit ends them).

    python tools/sim_bvh_c5.py [--rays 600]
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


def slab(lo, hi, o, d):
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t0 = (lo - o) * inv
        t1 = (hi - o) * inv
    tmin = np.nanmax(np.minimum(t0, t1), axis=1)
    tmax = np.nanmin(np.maximum(t0, t1), axis=1)
    return (tmax >= np.maximum(tmin, 0.0)), np.maximum(tmin, 0.0)


def mt(a, b, c, o, d):
    e1, e2 = b - a, c - a
    p = np.cross(d, e2)
    det = np.einsum("ij,ij->i", e1, p)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / det
        s = o - a
        u = np.einsum("ij,ij->i", s, p) * inv
        q = np.cross(s, e1)
        v = (q @ d) * inv
        t = np.einsum("ij,ij->i", e2, q) * inv
    ok = (np.abs(det) > 1e-12) & (u >= 0) & (v >= 0) & (u + v <= 1) & (t > 0)
    return np.where(ok, t, np.inf)


class Tree:
    def __init__(self, nf, ni, tf):
        self.lo, self.hi = nf[:, 0:3].astype(np.float64), nf[:, 3:6].astype(np.float64)
        self.left, self.right, self.tri = ni[:, 0], ni[:, 1], ni[:, 2]
        self.a, self.b, self.c = tf[:, 0:3].astype(np.float64), tf[:, 3:6].astype(np.float64), tf[:, 6:9].astype(np.float64)
        self.n = tf[:, 9:12].astype(np.float64)

    def trace(self, o, d, tmax=np.inf, shadow=False):
        hit, tin = slab(self.lo, self.hi, o, d)
        leaves = np.nonzero(hit & (self.tri >= 0))[0]
        tt = np.full(len(self.lo), np.inf)
        if len(leaves):
            k = self.tri[leaves]
            tt[leaves] = mt(self.a[k], self.b[k], self.c[k], np.broadcast_to(o, (len(k), 3)), d)
        # the reference's walk: every child of a hit internal node is tested
        internal_hit = hit & (self.tri < 0)
        all_tests = 1 + 2 * int(np.count_nonzero(internal_hit))
        best_t = np.min(tt) if len(leaves) else np.inf
        res = {"all": all_tests, "all_leaf": int(len(leaves))}

        def bound():
            return tmax if shadow else best

        # DFS order with pruning
        best = np.inf
        tests = 0
        leaf_tests = 0
        stack = [0]
        while stack:
            nidx = stack.pop()
            tests += 1
            if not hit[nidx] or tin[nidx] > bound():
                continue
            if self.tri[nidx] >= 0:
                leaf_tests += 1
                if tt[nidx] <= best:
                    best = tt[nidx]
                if shadow and tt[nidx] < tmax:
                    break
                continue
            stack.append(self.right[nidx])
            stack.append(self.left[nidx])
        res["dfs_prune"], res["dfs_prune_leaf"] = tests, leaf_tests
        # near child first
        best = np.inf
        tests = 0
        leaf_tests = 0
        wide = 0
        stack = [0]
        while stack:
            nidx = stack.pop()
            tests += 1
            if not hit[nidx] or tin[nidx] > bound():
                continue
            if self.tri[nidx] >= 0:
                leaf_tests += 1
                if tt[nidx] <= best:
                    best = tt[nidx]
                if shadow and tt[nidx] < tmax:
                    break
                continue
            l, r = self.left[nidx], self.right[nidx]
            if tin[r] < tin[l]:
                l, r = r, l
            stack.append(r)
            stack.append(l)
        res["ord_prune"], res["ord_prune_leaf"] = tests, leaf_tests
        # 4-wide: a fetch tests up to 4 grandchildren (children that are leaves count as themselves)
        best = np.inf
        stack = [0]
        fetches = 0
        leaf_tests = 0
        while stack:
            nidx = stack.pop()
            if self.tri[nidx] >= 0:
                leaf_tests += 1
                if tt[nidx] <= best:
                    best = tt[nidx]
                if shadow and tt[nidx] < tmax:
                    break
                continue
            fetches += 1
            kids = []
            for ch in (self.left[nidx], self.right[nidx]):
                if self.tri[ch] >= 0 or not hit[ch]:
                    kids.append(ch)
                else:
                    kids += [self.left[ch], self.right[ch]]
            kids = [k for k in kids if hit[k] and tin[k] <= bound()]
            kids.sort(key=lambda k: -tin[k])
            stack += kids
        res["wide4"], res["wide4_leaf"] = fetches, leaf_tests
        # 4-wide in DFS order (no sorting): children of a fetched node pushed in reverse DFS order; the
        # deepest stack and the box tests (4 per fetch, children that exist)
        best = np.inf
        stack = [0]
        fetches = boxes = leaf_tests = maxst = 0
        while stack:
            nidx = stack.pop()
            if self.tri[nidx] >= 0:
                leaf_tests += 1
                if tt[nidx] <= best:
                    best = tt[nidx]
                if shadow and tt[nidx] < tmax:
                    break
                continue
            fetches += 1
            kids = []
            for ch in (self.left[nidx], self.right[nidx]):
                if self.tri[ch] >= 0:
                    kids.append(ch)
                else:
                    kids += [self.left[ch], self.right[ch]]
            boxes += len(kids)
            kids = [k for k in kids if hit[k] and tin[k] <= bound()]
            stack += kids[::-1]
            maxst = max(maxst, len(stack))
        res["wide4_dfs"], res["wide4_dfs_boxes"], res["wide4_dfs_leaf"], res["wide4_dfs_maxstack"] = fetches, boxes, leaf_tests, maxst
        # the kernel's wide walk (rt_coherent.hip walk_w): leaves postponed, the first hit internal slot next,
        # the others pushed in slot order onto a 4-entry stack; a push past it = overflow (binary restart)
        best = np.inf
        cur, st, fetches, over = 0, [], 0, 0
        while cur is not None:
            fetches += 1
            kids = []
            for ch in (self.left[cur], self.right[cur]):
                kids += [ch] if self.tri[ch] >= 0 else [self.left[ch], self.right[ch]]
            nxt = None
            for k in kids:
                if not (hit[k] and tin[k] <= bound()):
                    continue
                if self.tri[k] >= 0:
                    if tt[k] <= best:
                        best = tt[k]
                elif nxt is None:
                    nxt = k
                elif len(st) < 4:
                    st.append(k)
                else:
                    over = 1
            if over:
                break
            if nxt is None and st:
                nxt = st.pop()
            cur = nxt
        res["walk_w_fetches"], res["walk_w_overflow"] = fetches, over
        return res, best_t, (np.argmin(tt) if len(leaves) and np.isfinite(best_t) else -1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=600)
    args = ap.parse_args()
    rt = load_rt()
    sc = rt.Scene.cornell_c5(np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz"))["raw_bunny"])
    nf, ni, tf, ti = sc.export()
    T = Tree(nf, ni, tf)
    rng = np.random.default_rng(1)
    W, H = 384, 216
    cam, _, _ = rt.camera_default(W, H)
    pos = np.array(cam.position, np.float64)
    ip = np.array(cam.inv_projection, np.float64).reshape(4, 4).T
    iv = np.array(cam.inv_view, np.float64).reshape(4, 4).T
    light_tris = np.nonzero(tf[:, 12] > 0)[0] if tf.shape[1] > 12 else []
    lc = np.array([2.78, 5.487, 2.795])
    tot = {"camera": {}, "bounce": {}, "shadow": {}}
    cnt = {"camera": 0, "bounce": 0, "shadow": 0}

    def add(kind, r):
        cnt[kind] += 1
        for k, v in r.items():
            tot[kind][k] = tot[kind].get(k, 0) + v

    for _ in range(args.rays):
        x, y = rng.uniform(0, W), rng.uniform(0, H)
        ndc = np.array([2 * x / W - 1, 2 * y / H - 1, 1, 1])
        tg = ip @ ndc
        d = (iv @ np.array([*(tg[:3] / tg[3]), 0]))[:3]
        d /= np.linalg.norm(d)
        o = pos
        for depth in range(3):
            r, t, leaf = T.trace(o, d)
            add("camera" if depth == 0 else "bounce", r)
            if not np.isfinite(t):
                break
            k = T.tri[leaf]
            p = o + t * d
            n = T.n[k] / np.linalg.norm(T.n[k])
            if np.dot(n, d) > 0:
                n = -n
            # shadow ray towards a point on the light
            lp = lc + np.array([rng.uniform(-0.6, 0.6), 0, rng.uniform(-0.5, 0.5)])
            sd = lp - p
            sl = np.linalg.norm(sd)
            rs, _, _ = T.trace(p, sd / sl, tmax=sl - 0.01, shadow=True)
            add("shadow", rs)
            # cosine bounce
            u1, u2 = rng.uniform(), rng.uniform()
            phi = 2 * np.pi * u1
            tvec = np.cross(n, [1.0, 0, 0] if abs(n[0]) < 0.9 else [0, 1.0, 0])
            tvec /= np.linalg.norm(tvec)
            bvec = np.cross(n, tvec)
            d = np.sqrt(u2) * (np.cos(phi) * tvec + np.sin(phi) * bvec) + np.sqrt(1 - u2) * n
            d /= np.linalg.norm(d)
            o = p
    out = {k: {m: round(v / max(cnt[k], 1), 2) for m, v in tot[k].items()} for k in tot}
    out["rays"] = cnt
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
