#!/usr/bin/env python3
"""Design study ("the walk's top levels in LDS"): how much of C5's bunny walk a per-block LDS copy
of each near-first ordering's top L tree levels could serve.  A wave waits for its slowest lane's node load, so a
walk step is served from LDS only when EVERY lane still walking sits on a top-level node; this replays waves of 64
rays (the sim_sah_c5.py ray model: room points toward the bunny's box, then shadow rays to the light) started
together -- the best case, the kernel's lanes start their walks at different rounds -- and reports that fraction
next to the per-lane fraction (which only moves L2 traffic).

    python tools/sim_top_lds.py [--waves 6]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import sim_sah_c5 as S  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEVELS = (3, 4, 5, 6)


def walk_depths(T, order, skipp, depth_pos, o, d, tri_t, bound0, shadow):
    """sim_sah_c5.walk, returning the tree depth of every visited node and the closest hit"""
    inv = 1.0 / d
    lo, hi = T.lo[order], T.hi[order]
    t0 = (lo - o) * inv; t1 = (hi - o) * inv
    tin = np.max(np.minimum(t0, t1), 1); tout = np.min(np.maximum(t0, t1), 1)
    hit = (tout >= 0) & (tin <= tout)
    leaf = T.tri[order] >= 0
    best, p, n, seq = np.inf, 0, len(order), []
    while p < n:
        seq.append(depth_pos[p])
        bnd = bound0 if shadow else best
        if hit[p] and tin[p] <= bnd * 1.00001 + 1e-5:
            if leaf[p]:
                t = tri_t(T.tri[order[p]], o, d)
                if shadow and t < bound0:
                    return np.array(seq), t
                best = min(best, t)
                p = skipp[p]
            else:
                p += 1
        else:
            p = skipp[p]
    return np.array(seq), best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--waves", type=int, default=6)
    args = ap.parse_args()
    rt = S.load_rt()
    sc = rt.Scene.cornell_c5(np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz"))["raw_bunny"])
    info = sc.info()
    nf, ni, tf, _ = sc.export()
    ref = S.subtree(nf, ni, info.split_root, info.split_end)
    leaf = ref.tri >= 0
    T, root = S.build_sah(ref.lo[leaf], ref.hi[leaf], ref.tri[leaf])
    depth = np.zeros(len(T.tri), int)
    st = [(root, 0)]
    while st:
        i, dd = st.pop()
        depth[i] = dd
        if T.tri[i] < 0:
            st += [(T.left[i], dd + 1), (T.right[i], dd + 1)]
    A, B, C = tf[:, 0:3].astype(np.float64), tf[:, 3:6].astype(np.float64), tf[:, 6:9].astype(np.float64)

    def tri_t(k, o, d):
        e1, e2 = B[k] - A[k], C[k] - A[k]
        p = np.cross(d, e2); det = e1 @ p
        if abs(det) < 1e-14:
            return np.inf
        inv = 1.0 / det; s = o - A[k]; u = (s @ p) * inv
        q = np.cross(s, e1); v = (d @ q) * inv; t = (e2 @ q) * inv
        return t if (u > 0 and v > 0 and u + v < 1 and t > 0) else np.inf

    od = [S.ordering(T, root, o) for o in range(8)]
    dpos = [depth[o[0]] for o in od]
    octant = lambda d: int(d[0] < 0) | (int(d[1] < 0) << 1) | (int(d[2] < 0) << 2)
    rng = np.random.default_rng(5)
    blo, bhi = ref.lo[0], ref.hi[0]
    lc = np.array([2.78, 5.487, 2.795])
    wave_top = {L: 0 for L in LEVELS}; wave_tot = 0
    lane_top = {L: 0 for L in LEVELS}; lane_tot = 0
    for _ in range(args.waves):
        for kind in ("A", "B"):
            seqs = []
            for _ in range(64):
                o = rng.uniform([0, 0, 0], [5.56, 5.488, 5.592])
                d = rng.uniform(blo, bhi) - o
                d /= np.linalg.norm(d)
                oc = octant(d)
                seq, best = walk_depths(T, od[oc][0], od[oc][1], dpos[oc], o, d, tri_t, np.inf, False)
                if kind == "B":
                    if not np.isfinite(best):
                        continue
                    p = o + best * d - 1e-5 * d
                    sd = lc + np.array([rng.uniform(-0.6, 0.6), 0, rng.uniform(-0.5, 0.5)]) - p
                    sl = np.linalg.norm(sd); sdir = sd / sl
                    oc = octant(sdir)
                    seq, _ = walk_depths(T, od[oc][0], od[oc][1], dpos[oc], p, sdir, tri_t, sl - 0.01, True)
                seqs.append(seq)
            for s_ in range(max(len(s) for s in seqs)):
                deepest = max(s[s_] for s in seqs if s_ < len(s))
                wave_tot += 1
                for L in LEVELS:
                    wave_top[L] += deepest <= L
            for s in seqs:
                lane_tot += len(s)
                for L in LEVELS:
                    lane_top[L] += int((s <= L).sum())
    print(json.dumps({"waves": args.waves, **{f"top_{L + 1}_levels": {
        "nodes_per_octant": 2 ** (L + 1) - 1, "lds_bytes_8_octants": 8 * 32 * (2 ** (L + 1) - 1),
        "wave_steps_all_lanes_top": round(wave_top[L] / wave_tot, 4), "lane_steps_top": round(lane_top[L] / lane_tot, 4)} for L in LEVELS}}, indent=1))


if __name__ == "__main__":
    main()
