#!/usr/bin/env python3
"""A/B of whole library builds (e.g. different kernel compile flags) in ONE process, interleaved rounds.

    make -C cpu-based-ray-tracer_amd LIB=librt_hip_lb5.so BUILD=build_lb5 KFLAGS=-DRT_MIN_WAVES=5 librt_hip_lb5.so
    python tools/ab_libs.py librt_hip.so librt_hip_lb5.so --spp 64
"""
import argparse
import importlib.util
import json
import os

os.environ.setdefault("RT_DEBUG_KNOBS", "1")   # the library reads its A/B knobs only behind this gate (csrc/rt_knobs.h)

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "cpu-based-ray-tracer_amd")


def load(libname):
    spec = importlib.util.spec_from_file_location("rt_amd_" + libname.replace(".", "_"), os.path.join(PKG, "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m.LIB_PATH = os.path.join(PKG, libname)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--fast", action="store_true")
    ap.add_argument("--scene", default="cornell", choices=["cornell", "c5", "c3", "c1"])
    ap.add_argument("--nranks", type=int, default=1, help="render rank --rank's row bands of an N-rank frame")
    ap.add_argument("--rank", type=int, default=0)
    args = ap.parse_args()
    W, H, spp = args.width, args.height, args.spp
    runs = {}
    for spec in args.libs:
        # "lib.so:K=V,K=V": environment knobs read at this library's context creation (rt_create)
        name, _, env = spec.partition(":")
        kv = [e.split("=", 1) for e in env.split(",") if e]
        for k, v in kv:
            os.environ[k] = v
        rt = load(name)
        bvh = np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz"))
        if args.scene == "c5":
            sc = rt.Scene.cornell_c5(bvh["raw_bunny"])
        elif args.scene == "c1":   # Whitted two spheres (C1: 640x480x1)
            sc = rt.Scene.two_spheres()
        elif args.scene == "c3":   # Whitted bunny + teapot (C3: 1280x960x64)
            sc = rt.Scene.bvh_tracer(bvh["raw_bunny"], bvh["raw_teapot"])
        else:
            sc = rt.Scene.cornell()
        ctx = rt.Context(0)
        ctx.upload(sc)
        ctx.resize(W, H, 8, args.rank, args.nranks)
        cam = rt.camera_bvh_tracer(W, H) if args.scene == "c3" else (rt.camera_two_spheres(W, H) if args.scene == "c1" else rt.camera_default(W, H)[0])
        for k, _ in kv:
            os.environ.pop(k, None)
        runs[spec] = (rt, ctx, cam, [], sc, [], [])
    kw = dict(whitted=True) if args.scene in ("c1", "c3") else dict(exact=not args.fast)
    ref = None
    for r in range(args.rounds + 1):
        for name, (rt, ctx, cam, res, _, pre, main) in runs.items():
            ctx.render(cam, spp, fetch=False, **kw)
            if r > 0:
                st = ctx.stats()
                res.append(ctx.local_rows * W * spp / st.last_kernel_ms / 1e3)
                pre.append(st.last_prepass_ms)
                main.append(st.last_main_ms)
    out = {}
    for name, (rt, ctx, cam, res, _, pre, main) in runs.items():
        _, acc = ctx.render(cam, 4, **kw)
        same = None if ref is None else bool(np.array_equal(acc.view(np.uint32), ref.view(np.uint32)))
        ref = acc if ref is None else ref
        out[name] = {"median_msps": round(float(np.median(res)), 1), "grid": ctx.stats().grid, "bitwise_equal_to_first": same,
                     "prepass_ms": round(float(np.median(pre)), 3), "path_kernel_ms": round(float(np.median(main)), 3)}
        ctx.close()
    print(json.dumps({"config": f"{W}x{H}x{spp} {args.scene} {'fast' if args.fast else 'exact'}", "rank": args.rank, "nranks": args.nranks, "libs": out}, indent=1))


if __name__ == "__main__":
    main()
