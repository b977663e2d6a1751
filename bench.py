#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: Msamples/s of the Cornell-box Monte Carlo path tracer on N MI355X.

Workload (one "step"): the C4 configuration -- the reference's Cornell box at 1920x1080, 1024 spp
(one sample = one camera path of one pixel in one frame, MC/Renderer.cpp:91-134), accumulated from
frame 1, packed to RGBA8 and gathered to rank 0.  The image is dealt to the N ranks in 8-row bands
(round-robin); each rank renders its bands in one persistent megakernel launch; RCCL all-gathers the
RGBA8 bands (the only collective).  Total work is fixed as N grows ("scaling": "strong").

    python bench.py                       # N=1, defaults finish in about a minute
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

Prints ONE JSON line on rank 0 (value = whole-job Msamples/s), with the roofline of the megakernel
(HIP events on the kernel's own stream) and the reference CPU baseline timed on this host.
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))

# Algorithmic bytes per sample for the C4 Cornell workload (DESIGN.md
# "Measurement"): reference work per sample = 3.645 rays x (24.61 node tests x 32 B + 3.57 triangle
# tests x 36 B + 16 B shading fetch).
REF_WORK = {"rays_per_sample": 3.645, "node_tests_per_ray": 24.61, "tri_tests_per_ray": 3.57}
BYTES_PER_SAMPLE = REF_WORK["rays_per_sample"] * (REF_WORK["node_tests_per_ray"] * 32 + REF_WORK["tri_tests_per_ray"] * 36 + 16)
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def load_pkg():
    import importlib.util
    spec = importlib.util.spec_from_file_location("rt_amd", os.path.join(REPO, "cpu-based-ray-tracer_amd", "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def load_dist():
    import importlib.util
    spec = importlib.util.spec_from_file_location("rt_dist", os.path.join(REPO, "cpu-based-ray-tracer_amd", "dist.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def cpu_baseline(W, H, seconds, threads):
    """The reference renderer (oracle/_ref: the reference's BVH/triangle/material/camera code compiled
    from /root/reference, integrator glue restated) on this host's cores, bounded to ~`seconds`;
    falls back to the oracle restatement ("port") if the harness binary is absent."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle as O
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if os.path.exists(harness):
        tmp = tempfile.mkdtemp(prefix="rt_cpu_")
        try:
            for (name, raw, _, _) in O.cornell_meshes():   # the fixture's objl positions, written back as OBJ
                with open(os.path.join(tmp, name + ".obj"), "w") as f:
                    for v in raw.reshape(-1, 3):
                        f.write("v %r %r %r\n" % tuple(float(c) for c in v))
                    for i in range(raw.shape[0]):
                        f.write("f %d %d %d\n" % (3 * i + 1, 3 * i + 2, 3 * i + 3))

            def run(spp):
                out = [os.path.join(tmp, x) for x in ("a", "r", "s")]
                t0 = time.perf_counter()
                subprocess.run([harness, "image", tmp, "", str(W), str(H), str(spp), "0", "0.8", str(threads)] + out,
                               check=True, capture_output=True)
                return time.perf_counter() - t0

            t1 = run(1)
            spp = max(1, int(seconds / max(t1, 1e-3)))
            dt = run(spp)
            return {"value": W * H * spp / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "reference",
                    "sample": f"oracle/_ref/ref_harness: reference MC/ BVH+triangle+material+camera code (compiled from "
                              f"/root/reference), integrator glue restated; Cornell {W}x{H} x {spp} spp = "
                              f"{W * H * spp} samples in {dt:.1f} s, {threads} threads, RR 0.8"}
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
    sc = O.Scene()
    t0 = time.perf_counter()
    sc.render(W, H, 1, threads=threads)
    t1 = time.perf_counter() - t0
    spp = max(1, int(seconds / max(t1, 1e-3)))
    t0 = time.perf_counter()
    sc.render(W, H, spp, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": W * H * spp / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle restatement, Cornell {W}x{H} x {spp} spp in {dt:.1f} s, {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--band", type=int, default=8)
    ap.add_argument("--fast", action="store_true", help="forward accumulation instead of the exact inner-first fold")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    # a dedicated (non-null) stream shared by the megakernel, the copies, RCCL and the torch ops,
    # so every step is ordered on ONE stream and torch.cuda.Event sees the kernel
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    assert stream.cuda_stream != 0

    rt = load_pkg()
    W, H, spp = args.width, args.height, args.spp
    ctx = rt.Context(dev.index, stream.cuda_stream)
    scene = rt.Scene.cornell()
    ctx.upload(scene)
    ctx.resize(W, H, args.band, rank, world)
    cam, _, _ = rt.camera_default(W, H)

    rtdist = load_dist()
    gat = rtdist.ImageGather(W, H, args.band, rank, world, dev)
    assert gat.n_local == ctx.local_rows
    kernel_ms = []
    launch_info = {}

    def step():
        ctx.render(cam, spp, first_frame=1, seed=0, rr=0.8, exact=not args.fast, fetch=False)
        ctx.copy_rgba_to_device(gat.send.data_ptr())   # this rank's rows, on the shared stream
        gat.gather()                                    # RCCL all-gather + reassembly on rank 0
        st = ctx.stats()
        kernel_ms.append(st.last_kernel_ms)
        launch_info.update(passes=st.n_passes, chunks=st.n_chunks, kernel=rt.KERNEL_NAMES.get(st.kernel, str(st.kernel)))

    for _ in range(args.warmup):
        step()
    kernel_ms.clear()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_samples = W * H * spp * args.steps
    value = total_samples / elapsed / 1e6

    # roofline of the megakernel on this rank: algorithmic bytes per launch / mean launch time.  A step
    # is `passes` launches over consecutive frame ranges (each followed by the in-order finalize of its
    # frame chunks, included in the HIP-event time); per launch = per step / passes.
    local_samples = gat.n_local * W * spp
    passes = max(1, int(launch_info.get("passes", 1)))
    k_s = float(np.mean(kernel_ms)) / 1e3 / passes if kernel_ms else float("nan")
    per_launch = local_samples / passes
    achieved = BYTES_PER_SAMPLE * per_launch / k_s / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": launch_info.get("kernel", "?"), "kernel_ms": round(k_s * 1e3, 3),
            "bytes_per_sample": round(BYTES_PER_SAMPLE, 1), "samples_per_launch": int(per_launch),
            "launches_per_step": passes, "frame_chunks": int(launch_info.get("chunks", 1)),
            "gsamples_per_s_kernel": round(per_launch / k_s / 1e9, 4)}
    prof = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(prof):
        try:
            pm = json.load(open(prof))
            key = f"{roof['kernel']}:{W}x{H}x{spp}_{'fast' if args.fast else 'exact'}_n{world}_p{passes}"
            if key in pm:
                roof["traffic"] = pm[key]["hbm_bytes_per_launch"]
        except Exception:
            pass

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        threads = min(threads, 16)
        cpu = cpu_baseline(W, H, args.cpu_seconds, threads)

    if rank == 0:
        line = {
            "metric": "Msamples/s Cornell box 1024spp @1/2/4/8 MI355X; per-pixel RMSE vs CPU ref",
            "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32+f64", "data": "synthetic (reference Cornell box scene, Philox RNG seed 0)",
            "config": {"workload": f"C4 cornell {W}x{H} {spp}spp", "width": W, "height": H, "spp": spp, "rr": 0.8,
                       "seed": 0, "band_rows": args.band, "accumulation": "fast" if args.fast else "exact",
                       "parallelism": f"row-bands x{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
