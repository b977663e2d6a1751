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


def split_bytes(c):
    """L2 -> fabric bytes from the per-size request counters, or None when the passes are absent"""
    need = ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum")
    if not all(k in c for k in need):
        return None
    rd = 32 * c["TCC_EA0_RDREQ_32B_sum"] + 64 * c["TCC_EA0_RDREQ_64B_sum"] + 128 * c["TCC_EA0_RDREQ_128B_sum"]
    wr = 64 * c["TCC_EA0_WRREQ_64B_sum"] + 32 * (c["TCC_EA0_WRREQ_sum"] - c["TCC_EA0_WRREQ_64B_sum"])
    return {"read_bytes": rd, "write_bytes": wr,
            "read_requests_unsized": c["TCC_EA0_RDREQ_sum"] - c["TCC_EA0_RDREQ_32B_sum"] - c["TCC_EA0_RDREQ_64B_sum"] - c["TCC_EA0_RDREQ_128B_sum"],
            "rdreq_dram": c.get("TCC_EA0_RDREQ_DRAM_sum"), "wrreq_dram": c.get("TCC_EA0_WRREQ_DRAM_sum")}


# known bytes per dispatch of tools/calib_traffic.hip: (kernel name, occurrence) -> (label, read, write)
CALIB = {("k_stream_copy", 0): ("stream copy 16 B/lane", 1 << 30, 1 << 30)}
CALIB.update({("k_park12", f): ("park 12 B, lanes at one frame, f%d" % f, 0, (1 << 24) * 12) for f in range(4)})
CALIB.update({("k_park12", 4 + f): ("park 12 B, lanes at staggered frames, launch %d" % f, 0, (1 << 24) * 12) for f in range(4)})
CALIB[("k_read48", 0)] = ("read 48-byte blocks, one per lane", (1 << 24) * 48, 0)
CALIB[("k_ring16", 0)] = ("ring: 16 B read + 16 B write per lane, 3 KiB lane stride", (1 << 20) * 16, (1 << 20) * 16)


def calibrate(src):
    """counted / known bytes per calibration dispatch: FETCH_SIZE, WRITE_SIZE and the size-split bytes"""
    per = collections.defaultdict(dict)   # (kernel, occurrence) -> counter -> value
    for f in glob.glob(os.path.join(src, "calib_*", "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        order = {}
        for d in sorted({(int(r["Dispatch_Id"]), r["Kernel_Name"]) for r in rows}):
            name = next((k for k, _ in CALIB if k in d[1]), None)
            if name is not None:
                order[d[0]] = (name, sum(1 for v in order.values() if v[0] == name))
        for r in rows:
            key = order.get(int(r["Dispatch_Id"]))
            if key is not None:
                per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if not per:
        return None
    out = []
    for key, (label, rd, wr) in CALIB.items():
        c = per.get(key, {})
        e = {"kernel": key[0], "shape": label, "known_read_bytes": rd, "known_write_bytes": wr}
        if "FETCH_SIZE" in c and rd:
            e["fetch_size_over_known"] = c["FETCH_SIZE"] * 1024 / rd
        if "WRITE_SIZE" in c and wr:
            e["write_size_over_known"] = c["WRITE_SIZE"] * 1024 / wr
        sz = split_bytes(c)
        if sz:
            if rd:
                e["split_read_over_known"] = sz["read_bytes"] / rd
            if wr:
                e["split_write_over_known"] = sz["write_bytes"] / wr
        e["requests"] = {k: v for k, v in c.items() if k.startswith("TCC_")}
        out.append(e)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--key", required=True, help="bench.py traffic key (WxHxSPP_mode_nN_pP; stored as KERNEL:key)")
    ap.add_argument("--samples", type=float, required=True, help="samples per megakernel launch")
    ap.add_argument("--kernel", default="pt_megakernel", help="substring of the profiled kernel's name (e.g. 'pt_coherent_kernel<true')")
    ap.add_argument("--key-kernel", default=None, help="kernel name in the stored key (bench.py's KERNEL_NAMES); default --kernel")
    ap.add_argument("--sha", default=None, help="lib_sha256 of the profiled build (bench line); default: the in-tree librt_hip.so")
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
    out = {"kernel": args.kernel, "key": (args.key_kernel or args.kernel) + ":" + args.key, "per_launch_counters": counters, "samples_per_launch": args.samples,
           "lib_sha256": args.sha or (hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16] if os.path.exists(lib) else None)}
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        hbm = counters["FETCH_SIZE"] * 1024 * 2 + counters["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = hbm
        out["hbm_correction"] = "FETCH_SIZE (KB) x1024 x2 (gfx950 reports half of a wide coalesced read, MI355X_MICROARCH.md HBM) + WRITE_SIZE (KB) x1024"
        out["hbm_bytes_per_sample"] = hbm / args.samples
    # request-size splits (run_rocprof.sh passes pmc_rdsz / pmc_wrsz): bytes = size x count per size class,
    # with no FETCH_SIZE factor (FETCH_SIZE prices 128-byte requests through TCC_BUBBLE)
    sz = split_bytes(counters)
    if sz:
        out.update({"split_" + k: v for k, v in sz.items()})
        out["split_read_bytes_per_sample"] = sz["read_bytes"] / args.samples
        out["split_write_bytes_per_sample"] = sz["write_bytes"] / args.samples
        out["split_bytes_per_sample"] = (sz["read_bytes"] + sz["write_bytes"]) / args.samples
        out["hbm_bytes_per_launch"] = sz["read_bytes"] + sz["write_bytes"]
        out["hbm_bytes_per_sample"] = out["split_bytes_per_sample"]
        out["hbm_correction"] = ("TCC_EA0_RDREQ_{32B,64B,128B} x {32,64,128} + TCC_EA0_WRREQ_64B x 64 + (TCC_EA0_WRREQ - _64B) x 32: "
                                 "L2 -> fabric bytes by request size (Infinity Cache hits included); calibration in calib_traffic.json")
    cal = calibrate(args.src)
    if cal:
        json.dump(cal, open(os.path.join(args.dst, "calib_traffic.json"), "w"), indent=1)
        out["calibration"] = "calib_traffic.json"
    for name in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
        if name in counters:
            out[name.lower().replace("sq_insts_", "") + "_wave_insts_per_sample"] = counters[name] / args.samples
    if "SQ_THREAD_CYCLES_VALU" in counters and "SQ_INSTS_VALU" in counters:
        out["valu_lane_utilization"] = counters["SQ_THREAD_CYCLES_VALU"] / (64 * counters["SQ_INSTS_VALU"])
    if "SQ_WAIT_ANY" in counters and "SQ_WAVE_CYCLES" in counters and counters["SQ_WAVE_CYCLES"]:
        out["wait_any_frac"] = counters["SQ_WAIT_ANY"] / counters["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in counters and "TCC_MISS_sum" in counters and (counters["TCC_HIT_sum"] + counters["TCC_MISS_sum"]):
        out["l2_hit_rate"] = counters["TCC_HIT_sum"] / (counters["TCC_HIT_sum"] + counters["TCC_MISS_sum"])
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
