#!/usr/bin/env python3
"""Summarize a profiles/run_rocprof.sh output directory (gpurun_out/prof_TAG) into the JSON kept under
profiles/<round>/: per-launch PMC counters of the megakernel, HBM bytes per launch (FETCH_SIZE x 1024
x 2, the gfx950 correction of MI355X_MICROARCH.md, + WRITE_SIZE x 1024), the kernel-trace statistics,
and derived ratios (VALU issue fraction, lane utilization).  The summary records the sha-256 of the
librt_hip.so it profiled and the bench shape key; bench.py reports `traffic` and the counter ratios only
from a summary whose build and shape match its own run.

    python profiles/summarize_pmc.py gpurun_out/prof_r02 profiles/r02/c4 --key 1920x1080x1024_exact_n1_p1 --samples 2123366400 --kernel pt_coherent_kernel
"""
import argparse
import collections
import csv
import glob
import hashlib
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# a wave64 VALU instruction occupies its SIMD-32 for 2 cycles (MI355X_MICROARCH.md); 256 CUs x 4 SIMDs
SIMDS = 1024
XCDS = 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--key", required=True, help="bench.py traffic key (WxHxSPP_mode_nN_pP; stored as KERNEL:key)")
    ap.add_argument("--samples", type=float, required=True, help="samples per megakernel launch")
    ap.add_argument("--kernel", default="pt_megakernel")
    args = ap.parse_args()
    os.makedirs(args.dst, exist_ok=True)
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(args.src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if args.kernel in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, name), v in per.items():
            agg[name].append(v)
    counters = {k: sum(v) / len(v) for k, v in agg.items()}
    stats = None
    for f in glob.glob(os.path.join(args.src, "trace", "**", "*kernel_stats.csv"), recursive=True):
        stats = list(csv.DictReader(open(f)))
    lib = os.path.join(REPO, "cpu-based-ray-tracer_amd", "librt_hip.so")
    out = {"kernel": args.kernel, "key": args.kernel + ":" + args.key, "per_launch_counters": counters, "samples_per_launch": args.samples,
           "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16] if os.path.exists(lib) else None}
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        hbm = counters["FETCH_SIZE"] * 1024 * 2 + counters["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = hbm
        out["hbm_correction"] = "FETCH_SIZE (KB) x1024 x2 (gfx950 reports half of a wide coalesced read, MI355X_MICROARCH.md HBM) + WRITE_SIZE (KB) x1024"
        out["hbm_bytes_per_sample"] = hbm / args.samples
    for name in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
        if name in counters:
            out[name.lower().replace("sq_insts_", "") + "_wave_insts_per_sample"] = counters[name] / args.samples
    if "SQ_THREAD_CYCLES_VALU" in counters and "SQ_INSTS_VALU" in counters:
        out["valu_lane_utilization"] = counters["SQ_THREAD_CYCLES_VALU"] / (64 * counters["SQ_INSTS_VALU"])
    if "SQ_INSTS_VALU" in counters and "GRBM_GUI_ACTIVE" in counters:
        # VALU issue slots used: wave-instructions x 2 cycles over all SIMDs' cycles (GRBM_GUI_ACTIVE is
        # summed over the 8 XCDs)
        out["valu_issue_frac"] = counters["SQ_INSTS_VALU"] * 2 / (SIMDS * counters["GRBM_GUI_ACTIVE"] / XCDS)
    if stats:
        out["kernel_stats"] = [{k: r[k] for k in ("Name", "Calls", "AverageNs", "Percentage")} for r in stats]
        for r in stats:
            if args.kernel in r["Name"]:
                out["kernel_avg_ms"] = out["kernel_ms"] = float(r["AverageNs"]) / 1e6
                if "GRBM_GUI_ACTIVE" in counters:
                    out["effective_clock_ghz"] = counters["GRBM_GUI_ACTIVE"] / 8 / (float(r["AverageNs"]) * 1e-9) / 1e9
    json.dump(out, open(os.path.join(args.dst, "pmc_summary.json"), "w"), indent=1)
    if stats:
        with open(os.path.join(args.dst, "bench_kernel_stats.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(stats[0].keys()))
            w.writeheader()
            w.writerows(stats)
    print(json.dumps({k: v for k, v in out.items() if k != "kernel_stats"}, indent=1))


if __name__ == "__main__":
    main()
