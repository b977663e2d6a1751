#!/usr/bin/env python3
"""C5 with the reference-identical host BVH vs the device-built LBVH (rt_upload_scene_gpu_bvh): host build
time, device build time, and the render rate on each tree (one JSON line each).

    python tools/lbvh_bench.py --spp 16
"""
import argparse
import importlib.util
import json
import os
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rt_amd", os.path.join(REPO, "cpu-based-ray-tracer_amd", "__init__.py"))
rt = importlib.util.module_from_spec(spec)
spec.loader.exec_module(rt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    args = ap.parse_args()
    raw = np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz"))["raw_bunny"]
    t0 = time.perf_counter()
    sc = rt.Scene.cornell_c5(raw)
    host_s = time.perf_counter() - t0
    W, H = args.width, args.height
    cam, _, _ = rt.camera_default(W, H)
    for tree in ("host", "device"):
        c = rt.Context(0)
        build_ms = None
        if tree == "host":
            c.upload(sc)
        else:
            build_ms = c.upload_gpu_bvh(sc)
            build_ms = min(build_ms, c.upload_gpu_bvh(sc))   # the second build has a warm allocator
        c.resize(W, H)
        c.render(cam, args.spp, fetch=False)
        c.render(cam, args.spp, fetch=False)
        ms = c.stats().last_kernel_ms
        print(json.dumps({"tree": tree, "scene_build_s_host_incl_obj": round(host_s, 3) if tree == "host" else None,
                          "device_build_ms": None if build_ms is None else round(build_ms, 3), "width": W, "height": H,
                          "spp": args.spp, "kernel_ms": round(ms, 3), "msamples_per_s": round(W * H * args.spp / ms / 1e3, 1)}), flush=True)
        c.close()


if __name__ == "__main__":
    main()
