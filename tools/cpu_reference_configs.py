#!/usr/bin/env python3
"""The reference renderers on this host's CPU cores, per configuration (the CPU side of
tools/bench_configs.py): each harness under oracle/_ref/ runs the reference's own compiled geometry,
material, camera (and, for the Denoiser, filter) code with the shading glue restated (oracle/ref/).
The Monte Carlo configurations (C2, C4, C5) run `ref_harness bench_mt`: the reference's SHIPPED random
stream (thread_local mt19937, MSVC distribution; WN/Random.h:27-30,47-48) on a persistent thread pool,
not the injected-RNG parity mode (3-4x slower per sample).  C1 / C3 are deterministic (no RNG); the
Denoiser's cost is its filters.  Bounded samples (a few seconds each); one JSON line per configuration,
with the per-thread rate scaled to one thread per physical core of one socket (`socket_estimate`).

    python tools/cpu_reference_configs.py [--threads N]     (default: this job's CPU share)
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
REF = os.path.join(REPO, "oracle", "_ref")


def timed(cmd):
    t0 = time.perf_counter()
    subprocess.run(cmd, check=True, capture_output=True)
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=0)
    args = ap.parse_args()
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    cpu = bench.host_cpu()
    if args.threads <= 0:
        args.threads = cpu["usable_cpus"]
    T = str(args.threads)
    import _oracle as O
    from _rt import rt
    tmp = tempfile.mkdtemp(prefix="rt_cpuref_")
    out = [os.path.join(tmp, x) for x in ("a", "r", "s")]
    # the Cornell meshes (and the C5 bunny) as OBJ files for the harnesses
    for (name, raw, _, _) in O.cornell_meshes():
        rt.write_obj(os.path.join(tmp, name + ".obj"), raw)
    bunny = np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz"))
    rt.write_obj(os.path.join(tmp, "c5_bunny.obj"), rt.c5_mesh(bunny["raw_bunny"]))
    bvdir = os.path.join(tmp, "bv")
    os.makedirs(bvdir)
    rt.write_obj(os.path.join(bvdir, "bunny.obj"), bunny["raw_bunny"])
    rt.write_obj(os.path.join(bvdir, "teapot.obj"), bunny["raw_teapot"])
    lines = []
    # C1: the Whitted world, 640x480, 50 frames (identical: deterministic)
    dt = timed([os.path.join(REF, "ref_whitted_spheres"), "image", "640", "480", "50", T] + out)
    # (the harness traces each pixel once and accumulates that color 50 times -- the frames are identical --
    # so one frame's pixels are the traced samples)
    lines.append({"config": "C1", "samples": 640 * 480, "seconds": dt, "note": "one traced frame (50 identical frames accumulated)"})
    # C2 / C4: Cornell MC at reduced spp (frames are i.i.d., time is linear in spp), shipped RNG
    def bench_mt(extra, W, H, spp):
        r = subprocess.run([os.path.join(REF, "ref_harness"), "bench_mt", tmp, extra, str(W), str(H), str(spp), "0.8", T],
                           check=True, capture_output=True, text=True)
        tok = r.stdout.split()
        return float(tok[4])   # the frames only (scene build excluded)
    for c, (W, H, spp) in (("C2", (784, 784, 64)), ("C4", (1920, 1080, 16))):
        lines.append({"config": c, "samples": W * H * spp, "seconds": bench_mt("", W, H, spp), "rng": "shipped"})
    # C3: the BVH Ray Tracer, 1280x960, one frame (deterministic: every frame costs the same)
    dt = timed([os.path.join(REF, "ref_whitted_bvh"), "image", os.path.join(bvdir, "bunny.obj"), os.path.join(bvdir, "teapot.obj"),
                "1280", "960", "1", T] + out)
    lines.append({"config": "C3", "samples": 1280 * 960, "seconds": dt, "note": "includes the OBJ load + BVH build"})
    # C5: Cornell + 79,488-triangle bunny at 1920x1080, 2 spp, shipped RNG (scene build excluded)
    lines.append({"config": "C5", "samples": 1920 * 1080 * 8, "seconds": bench_mt(os.path.join(tmp, "c5_bunny.obj"), 1920, 1080, 8),
                  "rng": "shipped", "note": "1920x1080x8 (same framing as 3840x2160; time is linear in pixels x spp)"})
    # the Denoiser project: 480x270, 2 frames, joint bilateral 65 px (half 32) + temporal
    dt = timed([os.path.join(REF, "ref_denoiser"), "frames", tmp, "480", "270", "2", "0", "0.05", "32", "3", "1.0", "0.2", "1", T,
                os.path.join(tmp, "dn.bin")])
    lines.append({"config": "DN65", "samples": 480 * 270 * 2, "seconds": dt, "note": "480x270, 2 frames; per-frame cost scales with W*H"})
    for d in lines:
        d["threads"] = args.threads
        d["cpu_model"] = cpu["model"]
        d["msamples_per_s"] = round(d["samples"] / d["seconds"] / 1e6, 4)
        d["socket_estimate"] = round(d["msamples_per_s"] / args.threads * cpu["physical_cores_per_socket"], 3)
        d["physical_cores_per_socket"] = cpu["physical_cores_per_socket"]
        d["seconds"] = round(d["seconds"], 3)
        print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
