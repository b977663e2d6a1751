#!/usr/bin/env python3
"""One warm-up + one measured C4-shaped render with a given library build, for rocprofv3 PMC passes
comparing builds (profiles/run_rocprof.sh profiles bench.py itself).

    rocprofv3 --pmc SQ_INSTS_VALU -- python3 tools/prof_one.py librt_hip.so --spp 64
"""
import argparse
import json
import importlib.util
import os

os.environ.setdefault("RT_DEBUG_KNOBS", "1")   # the library reads its A/B knobs only behind this gate (csrc/rt_knobs.h)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "cpu-based-ray-tracer_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--fast", action="store_true")
    ap.add_argument("--sections", action="store_true", help="print the wave-cycle split of an RT_SECTIONS build")
    ap.add_argument("--scene", default="cornell", choices=["cornell", "c5", "c3"])
    ap.add_argument("--hist", action="store_true", help="print the candidate histograms of an RT_SECTIONS=3 build")
    ap.add_argument("--reps", type=int, default=1, help="measured renders after the warm-up")
    ap.add_argument("--nranks", type=int, default=1, help="render rank --rank's row bands of an N-rank frame")
    ap.add_argument("--rank", type=int, default=0)
    args = ap.parse_args()
    spec = importlib.util.spec_from_file_location("rt_amd", os.path.join(PKG, "__init__.py"))
    rt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rt)
    rt.LIB_PATH = os.path.join(PKG, args.lib)
    c = rt.Context(0)
    kw = dict(exact=not args.fast)
    if args.scene in ("c5", "c3"):
        import numpy as np
        bvh = np.load(os.path.join(REPO, "tests", "golden", "bvh_scene.npz"))
    if args.scene == "c5":
        c.upload(rt.Scene.cornell_c5(bvh["raw_bunny"]))
    elif args.scene == "c3":   # the BVH Ray Tracer's bunny + teapot, Whitted shading (BV/Renderer.cpp:121-233)
        c.upload(rt.Scene.bvh_tracer(bvh["raw_bunny"], bvh["raw_teapot"]))
        kw = dict(whitted=True)
    else:
        c.upload(rt.Scene.cornell())
    c.resize(args.width, args.height, 8, args.rank, args.nranks)
    cam = rt.camera_bvh_tracer(args.width, args.height) if args.scene == "c3" else rt.camera_default(args.width, args.height)[0]
    for _ in range(1 + args.reps):
        c.render(cam, args.spp, fetch=False, **kw)
    st = c.stats()
    print(f"{args.lib}: {st.last_kernel_ms:.2f} ms (path kernel {st.last_main_ms:.2f}), {c.local_rows * args.width * args.spp / st.last_kernel_ms / 1e3:.1f} Msamples/s")
    if args.sections:
        cyc = c.debug_counters(24)[16:24]
        # rt_coherent.hip SEC_MARK: [0] top (path ends, fold drain, work / camera records), [1] path end (fold set-up,
        # parked sample), [3] service (shadow verdict, fold level), [4] vertex shading (and the BVH variant's camera
        # ray), [5] box loop (leaf boxes) or BVH rounds, [6] Moller-Trumbore
        names = ["top: drain + records", "path end", "(unused; BVH: split phase)", "service", "vertex", "box loop (BVH: rounds)", "moller-trumbore", "(entry)"]
        tot = float(sum(cyc)) or 1.0
        print({n: round(v / tot, 4) for n, v in zip(names, cyc)})
        n = c.debug_counters(44)[24:44]
        it = max(n[0], 1)
        samples = c.local_rows * args.width * args.spp
        print({"wave_iterations": n[0], "lanes_on_path/it": round(n[1] / it, 2), "vertex/it": round(n[2] / it, 2),
               "finish/it": round(n[3] / it, 2), "camera/it": round(n[4] / it, 2),
               "mt_iters/it": round(n[5] / it, 2), "mt_lane_util": round(n[6] / max(n[5], 1) / 64, 3),
               "pairs/it": round(n[7] / it, 2), "compacted_chunks/it": round(n[8] / it, 2),
               "pairsA/it": round(n[13] / it, 2), "mt_lanesA/it": round(n[12] / it, 2), "mt_hits/it": round(n[14] / it, 2),
               "fin_iters_with_drain/it": round(n[9] / it, 3), "fin_lanes_with_drain/it": round(n[10] / it, 3),
               "drain_lanes_top/it": round(n[11] / it, 2),
               "union_tris_A/it": round(n[16] / it, 2), "union_tris_B/it": round(n[17] / it, 2), "union_tris_AB/it": round(n[18] / it, 2), "mt_open/it": round(n[19] / it, 4),
               "lane_iterations_per_sample": round(n[0] * 64 / samples, 3)})
    if args.sections and not args.hist:
        # the launch's timeline (rt_coherent.hip, RT_SECTIONS builds; wall_clock64 ticks at 100 MHz): how long the
        # waves run after their work queue ran dry (the launch's tail) -- meaningful for one render (--reps 0)
        t = c.debug_counters(448)[440:448]
        inv = lambda v: (~v) & 0xFFFFFFFFFFFFFFFF
        first_entry, last_entry, first_dry, last_dry, last_exit = inv(t[0]), t[1], inv(t[2]), t[3], t[4]
        waves = max(t[6], 1)
        ms = lambda ticks: round(ticks / 1e5, 3)
        print(json.dumps({"timeline_ms": {"entry_spread": ms(last_entry - first_entry), "first_dry_queue": ms(first_dry - first_entry),
                                          "last_dry_queue": ms(last_dry - first_entry), "last_exit": ms(last_exit - first_entry),
                                          "mean_wave_tail_after_dry_queue": ms(t[5] / waves), "mean_wave_busy_until_dry": ms(t[7] / waves)},
                          "waves": t[6], "reps": args.reps,
                          "segments_by_records_256": c.debug_counters(465)[448:465],
                          "waves_by_exit_minus_dry_0p1ms": c.debug_counters(488)[466:488]}))
    if args.hist:
        h = c.debug_counters(512)
        tot = lambda a, b: sum(h[a:b])
        out = {"A_candidates_hist": h[64:128], "B_candidates_hist": h[128:192], "wave_max_hist": h[192:256],
               "A_cand_by_tri": h[256:288], "B_cand_by_tri": h[288:320], "A_closest_by_tri": h[320:352], "B_blocked": h[352],
               "A_rays": tot(64, 128), "B_rays": tot(128, 192),
               "wave_union_A": h[400] / max(h[403], 1), "wave_union_B": h[401] / max(h[403], 1), "wave_union_AB": h[402] / max(h[403], 1)}
        print(json.dumps(out))
    c.close()


if __name__ == "__main__":
    main()
