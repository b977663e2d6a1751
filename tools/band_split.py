#!/usr/bin/env python3
"""Per-kernel split of one rank's band set of an N-rank C4 frame, rendered on this GPU:
pre-pass, path kernel, and the rest of rt_render (resample + in-order finalize + gaps).

    python tools/band_split.py [--nranks 1 2 4 8] [--reps 3]
"""
import argparse
import importlib.util
import json
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--spp", type=int, default=1024)
    a = ap.parse_args()
    spec = importlib.util.spec_from_file_location("rt", os.path.join(REPO, "cpu-based-ray-tracer_amd", "__init__.py"))
    rt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rt)
    W, H = 1920, 1080
    ctx = rt.Context(0)
    ctx.upload(rt.Scene.cornell())
    cam, _, _ = rt.camera_default(W, H)
    for n in a.nranks:
        for rank in sorted({0, n - 1}):
            ctx.resize(W, H, 8, rank, n)
            ctx.render(cam, a.spp, fetch=False)
            tot, pre, main = [], [], []
            for _ in range(a.reps):
                ctx.render(cam, a.spp, fetch=False)
                st = ctx.stats()
                tot.append(st.last_kernel_ms); pre.append(st.last_prepass_ms); main.append(st.last_main_ms)
            t, p, m = (float(np.median(x)) for x in (tot, pre, main))
            print(json.dumps({"nranks": n, "rank": rank, "rows": ctx.local_rows, "kernel_ms": round(t, 3), "prepass_ms": round(p, 3),
                              "main_ms": round(m, 3), "rest_ms": round(t - p - m, 3), "passes": ctx.stats().n_passes,
                              "chunks": ctx.stats().n_chunks}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
