#!/usr/bin/env python3
"""A/B of context-level knobs read from the environment at rt_create (RT_THRESH, RT_STEPS,
RT_CHUNKS, RT_ITEMS_PER_LANE, RT_MIN_PX_PER_LANE) and at the scene build (RT_WALK_TREE) in ONE process, interleaved rounds, optionally on a
row band of an N-rank frame (--rank/--nranks) to see multi-GPU per-rank behaviour on one GPU.

    python tools/sweep_env.py --set "RT_CHUNKS=1" --set "RT_CHUNKS=2" --nranks 8
"""
import argparse
import json
import os

os.environ.setdefault("RT_DEBUG_KNOBS", "1")   # the library reads its A/B knobs only behind this gate (csrc/rt_knobs.h)
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from _rt import rt  # noqa: E402

KNOBS = ("RT_RING_PACK", "RT_LBUF_PIXEL_MAJOR", "RT_VERTEX", "RT_VERTEX_BVH", "RT_BRUTE", "RT_FORCE_WALK", "RT_LDS_LEVELS", "RT_LDS_PAD", "RT_THRESH", "RT_STEPS", "RT_CHUNKS", "RT_ITEMS_PER_LANE", "RT_MIN_PX_PER_LANE", "RT_MIN_CHUNK_FRAMES", "RT_SEG_PARTS_OFF", "RT_SPLIT", "RT_WALK_ORDER", "RT_BVH_PREPASS", "RT_PRE_DEFER", "RT_WALK_TREE", "RT_SKY_BITS", "RT_SAH_BINS", "RT_SEG_MIN_PARTS", "RT_SEG_PART_LF", "RT_SEG_TAIL_PARTS", "RT_SEG_TAIL_EXTRA", "RT_WORK_QUEUES")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", action="append", default=[], help="space/comma/colon separated K=V assignments for one variant")
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--nranks", type=int, default=1)
    ap.add_argument("--fast", action="store_true")
    ap.add_argument("--scene", default="cornell", choices=["cornell", "c5", "c3"])
    ap.add_argument("--lib", default=None, help="library file in the package directory (default librt_hip.so)")
    args = ap.parse_args()
    if args.lib:
        rt.LIB_PATH = os.path.join(REPO, "cpu-based-ray-tracer_amd", args.lib)
    W, H, spp = args.width, args.height, args.spp
    bvh = np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz")) if args.scene in ("c5", "c3") else None
    cam = rt.camera_bvh_tracer(W, H) if args.scene == "c3" else rt.camera_default(W, H)[0]
    kw = dict(whitted=True) if args.scene == "c3" else dict(exact=not args.fast)
    variants = args.set or [""]
    ctxs = []
    for v in variants:
        for k in KNOBS:
            os.environ.pop(k, None)
        for a in v.replace(",", " ").replace(":", " ").split():   # (":" too: tools/gpu_run.sh splits its steps on commas)
            k, val = a.split("=")
            os.environ[k] = val
        # the scene is built under the variant's knobs too (RT_WALK_TREE is read by the scene build)
        scene = (rt.Scene.cornell_c5(bvh["raw_bunny"]) if args.scene == "c5" else
                 rt.Scene.bvh_tracer(bvh["raw_bunny"], bvh["raw_teapot"]) if args.scene == "c3" else rt.Scene.cornell())
        c = rt.Context(0)
        c.upload(scene)
        c.resize(W, H, 8, args.rank, args.nranks)
        ctxs.append((v, c, []))
    for r in range(args.rounds + 1):
        for v, c, res in ctxs:
            c.render(cam, spp, fetch=False, **kw)
            if r > 0:
                res.append(c.stats().last_kernel_ms)
    for v, c, res in ctxs:
        ms = float(np.median(res))
        print(json.dumps({"set": v, "rank": args.rank, "nranks": args.nranks, "kernel_ms": round(ms, 2), "all_ms": [round(x, 1) for x in res], "n_chunks": c.stats().n_chunks, "grid": c.stats().grid,
                          "msamples_per_s_rank": round(c.local_rows * W * spp / ms / 1e3, 1)}), flush=True)
        c.close()


if __name__ == "__main__":
    main()
