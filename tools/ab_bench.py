#!/usr/bin/env python3
"""A/B of megakernel variants in ONE process, interleaved rounds (cdna guide rule 24).
    python tools/ab_bench.py --width 1920 --height 1080 --spp 128 --rounds 3
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

VARIANTS = {
    "exact_lds": dict(exact=True, global_scene=False),
    "exact_lds_gstack": dict(exact=True, global_scene=False, global_stack=True),
    "exact_global": dict(exact=True, global_scene=True),
    "fast_lds": dict(exact=False, global_scene=False),
    "fast_global": dict(exact=False, global_scene=True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--count", action="store_true")
    args = ap.parse_args()
    W, H, spp = args.width, args.height, args.spp
    ctx = rt.Context(0)
    ctx.upload(rt.Scene.cornell())
    ctx.resize(W, H)
    cam, _, _ = rt.camera_default(W, H)
    names = args.variants.split(",")
    res = {n: [] for n in names}
    images = {}
    for r in range(args.rounds + 1):
        for n in names:
            ctx.render(cam, spp, fetch=False, **VARIANTS[n])
            st = ctx.stats()
            if r > 0:
                res[n].append(W * H * spp / (st.last_kernel_ms / 1e3) / 1e6)
            if r == args.rounds:
                rgba, acc = ctx.render(cam, 4, **VARIANTS[n])
                images[n] = acc
    out = {n: {"median_msps": float(np.median(v)), "min": float(np.min(v)), "max": float(np.max(v))} for n, v in res.items()}
    if args.count:
        for n in names:
            ctx.render(cam, spp, fetch=False, count=True, **VARIANTS[n])
            st = ctx.stats()
            out[n].update(rays_per_sample=st.rays / st.samples, nodes_per_ray=st.node_tests / st.rays, tris_per_ray=st.tri_tests / st.rays,
                          grid=st.grid, step_lane_eff=st.node_tests / max(1, 64 * st.wave_steps),
                          mt_lane_eff=st.tri_tests / max(1, 64 * st.wave_tri_tests),
                          wave_steps_per_sample=st.wave_steps / st.samples, wave_mt_per_sample=st.wave_tri_tests / st.samples,
                          wave_rounds_per_sample=st.wave_rounds / st.samples, wave_service_per_sample=st.wave_service / st.samples,
                          wave_fold_per_sample=st.wave_fold / st.samples,
                          service_lane_eff=st.service_lanes / max(1, 64 * st.wave_service))
            cyc = st.cycles_service + st.cycles_queue + st.cycles_trace
            out[n].update(cycle_share={"service": st.cycles_service / cyc, "queue_camera": st.cycles_queue / cyc,
                                       "trace": st.cycles_trace / cyc},
                          wave_cycles_per_sample=cyc / st.samples)
    base = images[names[0]].view(np.uint32)
    for n in names[1:]:
        out[n]["bitwise_equal_to_" + names[0]] = bool(np.array_equal(images[n].view(np.uint32), base))
    print(json.dumps({"config": f"{W}x{H}x{spp}", "variants": out}, indent=1))


if __name__ == "__main__":
    main()
