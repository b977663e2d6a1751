#!/usr/bin/env python3
"""Walk study: C5's subtree walk as a kernel of its own, K independent rays per lane (VERDICT r05 item 2's lever,
measured in isolation).  Needs the variant library (the product library has none of it):

    make -C cpu-based-ray-tracer_amd LIB=librt_hip_ws.so BUILD=build_ws KFLAGS=-DRT_WALK_STUDY=1 librt_hip_ws.so
    python tools/walk_study.py --lib librt_hip_ws.so --width 1920 --height 1080

Rays: C5's camera rays (a pinhole at the reference camera's position and direction, MC/Camera.h:19-21), one bounce
from each camera hit (rt_trace's closest hit, a uniform direction in the hemisphere facing the camera), and from the
same points one ray toward a uniform point of the walked subtree's root box (the rays that walk it).  Every K's (triangle, t) must
equal K = 1's bit for bit, and rt_trace's wherever rt_trace's hit lies in the walked subtree.
"""
import argparse
import ctypes as C
import importlib.util
import json
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "cpu-based-ray-tracer_amd")


def load(libname):
    spec = importlib.util.spec_from_file_location("rt_amd_ws", os.path.join(PKG, "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m.LIB_PATH = os.path.join(PKG, libname)
    return m


def camera_rays(rt, W, H):
    p = np.asarray(rt.DEFAULT_CAMERA_POSITION, np.float32)
    f = np.asarray(rt.DEFAULT_CAMERA_FORWARD, np.float32)
    f = f / np.linalg.norm(f)
    right = np.cross(f, np.float32([0, 1, 0])); right /= np.linalg.norm(right)
    up = np.cross(right, f)
    th = np.tan(np.radians(45.0) / 2)
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float32)
    u = ((xs + 0.5) / W * 2 - 1) * th * W / H
    v = (1 - (ys + 0.5) / H * 2) * th
    d = f[None, None] + u[..., None] * right[None, None] + v[..., None] * up[None, None]
    d = (d / np.linalg.norm(d, axis=-1, keepdims=True)).reshape(-1, 3).astype(np.float32)
    o = np.broadcast_to(p, d.shape).astype(np.float32).copy()
    return o, d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="librt_hip_ws.so")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--ks", default="1,2,3,4")
    ap.add_argument("--steps", default="12")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--mult", type=int, default=16)
    ap.add_argument("--modes", default="lock,refill", help="lock: a lane's K slots in lockstep until all are done; refill: a persistent grid refilling free slots")
    ap.add_argument("--sets", default="bounce,at_subtree")
    args = ap.parse_args()
    rt = load(args.lib)
    L = rt.lib()
    fn = L.rt_debug_walk_study
    fn.restype = C.c_int32
    fn.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    bvh = np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz"))
    sc = rt.Scene.cornell_c5(bvh["raw_bunny"])
    ctx = rt.Context(0)
    ctx.upload(sc)
    orders = sc.walk_orders()                       # (8, n_sub, 8) floats: the leaves' triangle bits in [..., 7]
    tri_bits = orders[0, :, 7].copy().view(np.int32)
    sub_tris = np.unique(tri_bits[tri_bits >= 0])
    W, H = args.width, args.height
    o_cam, d_cam = camera_rays(rt, W, H)
    tri_c, t_c = ctx.trace(o_cam, d_cam)
    trace_ms = ctx.stats().last_kernel_ms
    rng = np.random.default_rng(args.seed)
    hitm = tri_c >= 0
    loc = o_cam[hitm] + t_c[hitm].astype(np.float32)[:, None] * d_cam[hitm]
    loc = loc - 1e-4 * d_cam[hitm]                  # off the surface toward the camera
    # each surface point --mult times (fresh directions each time): enough waves to fill the chip K times over
    loc = np.tile(loc, (args.mult, 1)); din = np.tile(d_cam[hitm], (args.mult, 1))
    v = rng.normal(size=loc.shape).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    v = np.where((v * din).sum(1, keepdims=True) > 0, -v, v).astype(np.float32)
    # rays at the walked subtree: from the same surface points toward uniform points of the subtree's root box
    # (ordering 0 holds octant (+, +, +)'s near planes first: lo.xyz, hi.x | hi.y, hi.z)
    lo = orders[0, 0, 0:3].astype(np.float64); hi = np.array([orders[0, 0, 3], orders[0, 0, 4], orders[0, 0, 5]], np.float64)
    tgt = lo + rng.random(size=loc.shape) * (hi - lo)
    w = (tgt - loc).astype(np.float32)
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    sets = {"camera": (o_cam, d_cam), "bounce": (np.ascontiguousarray(loc, np.float32), np.ascontiguousarray(v, np.float32)),
            "at_subtree": (np.ascontiguousarray(loc, np.float32), np.ascontiguousarray(w, np.float32))}
    out = []
    for name in args.sets.split(","):
        o, d = sets[name]
        n = len(o)
        tri_r, t_r = ctx.trace(o, d)
        ref_ms = ctx.stats().last_kernel_ms
        in_sub = np.isin(tri_r, sub_tris)
        base = None
        rounds = {}
        for steps in [int(s) for s in args.steps.split(",")]:   # (ray, round) pairs: a ray's rounds are the same in every mode
            tri = np.zeros(n, np.int32); t = np.zeros(n, np.float64); ms = np.zeros(1, np.float32); cnt = np.zeros(1, np.uint64)
            if fn(ctx.h, n, o.ctypes.data, d.ctypes.data, 0x201, steps, 1, tri.ctypes.data, t.ctypes.data, ms.ctypes.data, cnt.ctypes.data) != 0:
                raise SystemExit("rt_debug_walk_study (count) failed")
            rounds[steps] = int(cnt[0])
        for steps in [int(s) for s in args.steps.split(",")]:
            for mode, k in [(m, int(s)) for m in args.modes.split(",") for s in args.ks.split(",")]:
                tri = np.zeros(n, np.int32); t = np.zeros(n, np.float64); ms = np.zeros(args.reps, np.float32)
                st = fn(ctx.h, n, o.ctypes.data, d.ctypes.data, k | (0x100 if mode == "refill" else 0), steps, args.reps, tri.ctypes.data, t.ctypes.data, ms.ctypes.data, None)
                if st != 0:
                    raise SystemExit(f"rt_debug_walk_study failed {st}")
                if base is None:
                    base = (tri.copy(), t.copy())
                same_k1 = bool(np.array_equal(tri, base[0]) and np.array_equal(t.view(np.uint64), base[1].view(np.uint64)))
                agree = bool(np.array_equal(tri[in_sub], tri_r[in_sub]) and np.array_equal(t[in_sub].view(np.uint64), t_r[in_sub].view(np.uint64)))
                med = float(np.median(ms))
                diff = np.nonzero((tri != base[0]) | (t.view(np.uint64) != base[1].view(np.uint64)))[0]
                rec = {"rays": name, "n": n, "mode": mode, "k": k, "steps": steps, "ms": round(med, 3), "all_ms": [round(float(x), 3) for x in ms],
                       "mrays_per_s": round(n / med / 1e3, 1), "rounds_per_ray": round(rounds[steps] / n, 3),
                       "g_lane_rounds_per_s": round(rounds[steps] / med / 1e6, 2), "bitwise_vs_k1": same_k1, "n_diff_k1": int(len(diff)), "diff_examples": [[int(i), int(tri[i]), int(base[0][i]), float(t[i]), float(base[1][i])] for i in diff[:4]], "bitwise_vs_rt_trace_in_subtree": agree,
                       "n_in_subtree": int(in_sub.sum()), "rt_trace_ms": round(ref_ms, 3)}
                out.append(rec)
                print(json.dumps(rec), flush=True)
    print(json.dumps({"camera_trace_ms": round(trace_ms, 3), "subtree_tris": int(len(sub_tris)), "camera_hits": int(hitm.sum()),
                      "subtree_box": [lo.tolist(), hi.tolist()]}))
    ctx.close()


if __name__ == "__main__":
    main()
