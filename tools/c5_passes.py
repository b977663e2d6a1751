#!/usr/bin/env python3
"""C5 at high spp: time and pass structure under different parked-sample budgets (RT_LBUF_BUDGET_MB),
one context per budget, in one process.   python tools/c5_passes.py --spp 4096 --budgets 98304,32768"""
import argparse
import json
import os

os.environ.setdefault("RT_DEBUG_KNOBS", "1")   # the library reads its A/B knobs only behind this gate (csrc/rt_knobs.h)
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from _rt import rt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=4096)
    ap.add_argument("--budgets", default="98304,32768")
    args = ap.parse_args()
    W, H = 3840, 2160
    sc = rt.Scene.cornell_c5(np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz"))["raw_bunny"])
    cam, _, _ = rt.camera_default(W, H)
    for b in args.budgets.split(","):
        os.environ["RT_LBUF_BUDGET_MB"] = b
        ctx = rt.Context(0)
        ctx.upload(sc)
        ctx.resize(W, H)
        ctx.render(cam, 8, fetch=False)
        t0 = time.perf_counter()
        ctx.render(cam, args.spp, fetch=False)
        ctx.synchronize() if hasattr(ctx, "synchronize") else None
        wall = time.perf_counter() - t0
        st = ctx.stats()
        print(json.dumps({"budget_mb": int(b), "spp": args.spp, "wall_s": round(wall, 3), "kernel_ms": round(st.last_kernel_ms, 1),
                          "main_ms": round(st.last_main_ms, 1), "passes": st.n_passes, "chunks": st.n_chunks,
                          "msamples_per_s": round(W * H * args.spp / (st.last_kernel_ms / 1e3) / 1e6, 1)}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
