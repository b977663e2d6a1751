#!/usr/bin/env python3
"""Per-configuration throughput on ONE MI355X.

bench.py reports the headline (C4); this prints one JSON line per configuration with the render's kernel
time (HIP events on its stream), Msamples/s, and for the path-traced configs the VALU roofline bench.py
uses: the REFERENCE's work per sample (rays, node and triangle tests per ray, shading
calls) priced at 18 flops per box test, 54 per triangle test and 150 per shading call, against the
157.3 TFLOP/s fp32 VALU peak.  (The scene is on chip for C2/C4; C5's traffic is in its PMC summary,
DESIGN.md 5.1.)  C5 runs at a reduced spp (frames are i.i.d. and the kernel time is linear in spp); the spp
used is in each line.

    python tools/bench_configs.py                 # all configs
    python tools/bench_configs.py --configs C5 --c5-spp 64
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

VALU_PEAK_TFLOPS = 157.3
# reference work per sample, SURVEY.md 8(d): rays/sample, node tests/ray, triangle tests/ray; shading calls
# per sample measured for C4 (1.4723 = 0.4036 per ray) and scaled by rays for C2/C5
WORK = {"C1": None, "C2": (5.700, 27.84, 4.06), "C3": None, "C4": (3.645, 24.61, 3.57), "C5": (3.660, 31.30, 3.85)}


# Whitted renders, priced the same way:
#  * C3 (BVH bunny + teapot): SURVEY.md 8(d)'s 1.446 rays/sample, 38.26 box tests and 2.57 triangle tests per ray
#    = 1196 flops/sample (SURVEY's "~1.2 kflop"; the Phong shading is not priced, as there);
#  * C1 (two spheres): 2.3078 rays/sample (the reference's own count, tests/golden/c1_spheres.npz stats), each
#    ray tested brute force against 2 spheres (~25 flops: QuadraticFormula, WH/Sphere.h:26-59) and the 2
#    chessboard triangles (54), plus 150 for the Phong / Fresnel shading = 308 flops per ray.
WHITTED_FLOPS = {"C3": 1.446 * (38.26 * 18 + 2.57 * 54), "C1": 2.3078 * (2 * 25 + 2 * 54 + 150)}
# the joint bilateral filter's tap (DN/Denoiser.h:188-205), counted op by op: position / color / normal /
# coplanarity distances (differences, dots, the four 2 sigma^2 products and divisions, normalize, squares;
# acosf ~20 and expf ~15 operations), the weight and the weighted color sum: ~97 fp32 operations
JBF_FLOPS_PER_TAP = 97.0


def counters_for(kname, W, H, spp, mode, passes):
    """The PMC summary of a rocprofv3 pass of THIS build (sha-256 of librt_hip.so) on THIS shape, as bench.py
    attaches it (profiles/**/pmc_summary.json from profiles/summarize_pmc.py); None without a matching pass."""
    import glob
    import hashlib
    lib = os.path.join(REPO, "cpu-based-ray-tracer_amd", "librt_hip.so")
    digest = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16] if os.path.exists(lib) else None
    key = f"{kname}:{W}x{H}x{spp}_{mode}_n1_p{passes}"
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "**", "pmc_summary*.json"), recursive=True), reverse=True):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("key") == key and digest is not None and d.get("lib_sha256") == digest:
            return {"file": os.path.relpath(p, REPO), "kernel_ms_profiled": d.get("kernel_ms"),
                    **{k: d.get(k) for k in ("valu_issue_frac", "valu_lane_utilization", "valu_wave_insts_per_sample",
                                              "salu_wave_insts_per_sample", "hbm_bytes_per_sample", "split_read_bytes_per_sample",
                                              "split_write_bytes_per_sample", "wait_any_frac", "l2_hit_rate")}}
    return None


def c5_parity(ctx, W, H, spp):
    """C5's timed frame against the reference harness's: the rows of
    tests/golden/full_c5.npz (256 spp, whole frame hashed) or full_c5_4096.npz (4096 spp, every 64th row
    hashed) bitwise, as bench.py's parity field does for C4; None when no fixture has this shape."""
    import hashlib
    for name in ("full_c5", "full_c5_4096"):
        p = os.path.join(REPO, "tests", "golden", f"{name}.npz")
        if not os.path.exists(p):
            continue
        z = np.load(p)
        if (int(z["W"]), int(z["H"]), int(z["spp"])) != (W, H, spp):
            continue
        acc = ctx.accumulation()
        rows = z["rows"]
        same = np.all(acc[rows, :, :3].view(np.uint32) == z["accum_rows"].view(np.uint32), axis=-1)
        sel = np.ascontiguousarray(acc[rows] if bool(z["rows_only"]) else acc)
        return {"fixture": f"tests/golden/{name}.npz", "rows_checked": int(len(rows)), "bitwise_frac": round(float(same.mean()), 6),
                "sha_accum_match": hashlib.sha256(sel.tobytes()).hexdigest() == str(z["sha_accum"]),
                "scope": "every 64th row" if bool(z["rows_only"]) else "whole frame"}
    return None


def flops_per_sample(c):
    if c in WHITTED_FLOPS:
        return WHITTED_FLOPS[c]
    r, n, t = WORK[c]
    return r * (n * 18 + t * 54) + 0.4036 * r * 150


def run(ctx, cam, W, H, spp, reps, full_warmup=False, **kw):
    ctx.resize(W, H)
    # warm-up; a render longer than the warm-up allocates its parked-sample and camera-record buffers
    # (tens of GB at C5 4096 spp) inside its first timed call unless the warm-up renders the full spp
    ctx.render(cam, spp if full_warmup else min(spp, 8), fetch=False, **kw)
    ms = []
    for _ in range(reps):
        ctx.render(cam, spp, fetch=False, **kw)
        ms.append(ctx.stats().last_kernel_ms)
    return float(np.median(ms))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C2,C3,C4,C5,DN15,DN33,DN65")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--c5-spp", type=int, default=64)
    ap.add_argument("--fast", action="store_true")
    ap.add_argument("--full-warmup", action="store_true", help="warm up at the measured spp (steady-state buffers)")
    ap.add_argument("--lib", default=None, help="library file in the package directory (A/B builds; default librt_hip.so)")
    args = ap.parse_args()
    if args.lib:
        rt.LIB_PATH = os.path.join(REPO, "cpu-based-ray-tracer_amd", args.lib)
    bvh = np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz"))
    for c in args.configs.split(","):
        if c.startswith("DN"):
            # the Denoiser project at 1920x1080: G-buffer frame + joint bilateral filter of the UI's
            # 15/33/65-pixel kernel (half sizes 3/16/32) + temporal filter (7-pixel kernel), per frame
            W, H = 1920, 1080
            half = {"DN15": 3, "DN33": 16, "DN65": 32}[c]
            ctx = rt.Context(0)
            ctx.upload(rt.Scene.cornell())
            ctx.resize(W, H)
            params = rt.denoise_params(jbf_half_size=half, temporal_half_size=3)
            gms, dms = [], []
            for f in range(1, 2 + args.reps):
                cam, proj, view = rt.camera_look_ex(W, H, rt.DEFAULT_CAMERA_POSITION, rt.DEFAULT_CAMERA_FORWARD)
                ctx.render_denoised(cam, proj, view, f, params, fetch=False)
                st = ctx.stats()
                if f > 1:
                    gms.append(st.last_kernel_ms); dms.append(st.last_denoise_ms)
            taps = W * H * (2 * half + 1) ** 2
            dn_s = float(np.median(dms)) / 1e3
            roof = {"bound": "valu", "flops_per_tap": JBF_FLOPS_PER_TAP, "achieved_tflops": round(taps * JBF_FLOPS_PER_TAP / dn_s / 1e12, 3),
                    "peak_tflops": VALU_PEAK_TFLOPS, "frac": round(taps * JBF_FLOPS_PER_TAP / dn_s / 1e12 / VALU_PEAK_TFLOPS, 4),
                    "time": "joint bilateral + temporal kernels (the temporal filter's taps are not priced)"}
            print(json.dumps({"config": c, "width": W, "height": H, "jbf_half_size": half, "temporal_half_size": 3,
                              "gbuffer_ms": round(float(np.median(gms)), 3), "denoise_ms": round(float(np.median(dms)), 3),
                              "frame_ms": round(float(np.median(gms)) + float(np.median(dms)), 3),
                              "jbf_taps_per_s": round(taps / dn_s / 1e9, 2), "roofline": roof}), flush=True)
            ctx.close()
            continue
        ctx = rt.Context(0)
        kw = {}
        if c == "C1":
            ctx.upload(rt.Scene.two_spheres())
            W, H, spp = 640, 480, 1
            cam = rt.camera_two_spheres(W, H)
            kw = dict(whitted=True)
        elif c in ("C2", "C4"):
            ctx.upload(rt.Scene.cornell())
            W, H, spp = (784, 784, 256) if c == "C2" else (1920, 1080, 1024)
            cam, _, _ = rt.camera_default(W, H)
            kw = dict(exact=not args.fast)
        elif c == "C3":
            ctx.upload(rt.Scene.bvh_tracer(bvh["raw_bunny"], bvh["raw_teapot"]))
            W, H, spp = 1280, 960, 64
            cam = rt.camera_bvh_tracer(W, H)
            kw = dict(whitted=True)
        elif c == "C5":
            ctx.upload(rt.Scene.cornell_c5(bvh["raw_bunny"]))
            W, H, spp = 3840, 2160, args.c5_spp
            cam, _, _ = rt.camera_default(W, H)
            kw = dict(exact=not args.fast)
        else:
            raise SystemExit(f"unknown config {c}")
        ms = run(ctx, cam, W, H, spp, args.reps, full_warmup=args.full_warmup, **kw)
        st = ctx.stats()
        samples = W * H * spp
        rate = samples / (ms / 1e3)
        fps = flops_per_sample(c)
        roof = None if fps is None else {"bound": "valu", "flops_per_sample": round(fps, 1), "achieved_tflops": round(fps * rate / 1e12, 3),
                                         "peak_tflops": VALU_PEAK_TFLOPS, "frac": round(fps * rate / 1e12 / VALU_PEAK_TFLOPS, 4)}
        mode = "whitted" if c in ("C1", "C3") else ("fast" if args.fast else "exact")
        if roof is not None:
            roof["counters"] = counters_for(rt.KERNEL_NAMES.get(st.kernel, str(st.kernel)), W, H, spp, mode, st.n_passes)
        line = {"config": c, "width": W, "height": H, "spp": spp, "kernel_ms": round(ms, 3),
                "msamples_per_s": round(rate / 1e6, 2), "grid": st.grid, "passes": st.n_passes,
                "prepass_ms": round(st.last_prepass_ms, 3), "path_ms": round(st.last_main_ms, 3), "roofline": roof,
                "mode": mode}
        if c == "C5" and not args.fast:
            line["parity"] = c5_parity(ctx, W, H, spp)   # the last timed render's accumulation (seed 0, RR 0.8, frames 1..spp)
        print(json.dumps(line), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
