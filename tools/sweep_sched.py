#!/usr/bin/env python3
"""Sweep the megakernel's traversal scheduling knobs (RT_THRESH, RT_STEPS; read at rt_create) in ONE
process, interleaved rounds (cdna guide rule 24).  Prints one JSON line per setting.

    python tools/sweep_sched.py --thresh 8,16,24 --steps 8,12,16 --spp 64
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--thresh", default="8,16,24,32")
    ap.add_argument("--steps", default="12")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--fast", action="store_true")
    ap.add_argument("--scene", default="cornell", choices=["cornell", "c5"])
    args = ap.parse_args()
    W, H, spp = args.width, args.height, args.spp
    if args.scene == "c5":
        scene = rt.Scene.cornell_c5(np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz"))["raw_bunny"])
    else:
        scene = rt.Scene.cornell()
    cam, _, _ = rt.camera_default(W, H)
    ctxs = {}
    for th in args.thresh.split(","):
        for st in args.steps.split(","):
            os.environ["RT_THRESH"], os.environ["RT_STEPS"] = th, st
            c = rt.Context(0)
            c.upload(scene)
            c.resize(W, H)
            ctxs[(int(th), int(st))] = c
    res = {k: [] for k in ctxs}
    for r in range(args.rounds + 1):
        for k, c in ctxs.items():
            c.render(cam, spp, fetch=False, exact=not args.fast)
            ms = c.stats().last_kernel_ms
            if r > 0:
                res[k].append(W * H * spp / ms / 1e3)
    for k, v in res.items():
        print(json.dumps({"thresh": k[0], "steps": k[1], "msamples_per_s": round(float(np.median(v)), 1),
                          "fast": args.fast, "scene": args.scene}), flush=True)
    for c in ctxs.values():
        c.close()


if __name__ == "__main__":
    main()
