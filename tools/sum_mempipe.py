#!/usr/bin/env python3
"""Summarize tools/prof_mempipe.sh passes: per counter, the mean over the measured dispatches of one kernel (the
last dispatches of the run: prof_one.py renders a warm-up, then the measured launch), and the ratios that say which
stage of the vector memory pipeline is busy.

    python tools/sum_mempipe.py gpurun_out/mem_r06g_c3 --kernel whitted_kernel > profiles/r06/.../mempipe.json
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", required=True)
    args = ap.parse_args()
    tot = {}
    for f in sorted(glob.glob(os.path.join(args.dir, "**", "*counter_collection*.csv"), recursive=True)):
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f)):
            if args.kernel in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        if not per:
            continue
        last = per[max(per)]   # the measured launch
        for k, v in last.items():
            tot.setdefault(k, v)
    g = tot.get("GRBM_GUI_ACTIVE")
    out = {"kernel": args.kernel, "counters": tot}
    if g:
        # GRBM_GUI_ACTIVE is reported summed over the 8 XCDs (profiles/summarize_pmc.py: XCDS), so the kernel's clocks
        # are a eighth of it; TA_BUSY_avr is per TA instance (one per CU); the TD/TCP sums add all CUs
        g = g / 8.0
        out["kernel_clocks"] = g
        ncu = 256
        r = {}
        if "TA_BUSY_avr" in tot:
            r["ta_busy_frac"] = tot["TA_BUSY_avr"] / g
        if "TD_TD_BUSY_sum" in tot:
            r["td_busy_frac"] = tot["TD_TD_BUSY_sum"] / (g * ncu)
        for k in ("TCP_PENDING_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum",
                  "TCP_TCP_TA_DATA_STALL_CYCLES_sum", "TCP_TD_TCP_STALL_CYCLES_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum",
                  "TA_DATA_STALLED_BY_TC_CYCLES_sum", "TD_TC_STALL_sum"):
            if k in tot:
                r[k.lower().replace("_sum", "_frac")] = tot[k] / (g * ncu)
        if "TA_FLAT_READ_WAVEFRONTS_sum" in tot:
            r["flat_read_wavefronts_per_cu_clock"] = tot["TA_FLAT_READ_WAVEFRONTS_sum"] / (g * ncu)
        if "TCP_TOTAL_CACHE_ACCESSES_sum" in tot:
            r["tcp_accesses_per_cu_clock"] = tot["TCP_TOTAL_CACHE_ACCESSES_sum"] / (g * ncu)
            if "TCP_TCC_READ_REQ_sum" in tot:
                r["tcp_miss_to_l2_frac"] = tot["TCP_TCC_READ_REQ_sum"] / max(1.0, tot["TCP_TOTAL_CACHE_ACCESSES_sum"])
        if "TCP_TCC_READ_REQ_LATENCY_sum" in tot and tot.get("TCP_TCC_READ_REQ_sum"):
            r["l2_read_latency_cycles"] = tot["TCP_TCC_READ_REQ_LATENCY_sum"] / tot["TCP_TCC_READ_REQ_sum"]
        if "SQ_WAVE_CYCLES" in tot:
            r["wait_any_frac"] = tot.get("SQ_WAIT_ANY", 0.0) / tot["SQ_WAVE_CYCLES"]
            r["active_inst_any_frac"] = tot.get("SQ_ACTIVE_INST_ANY", 0.0) / tot["SQ_WAVE_CYCLES"]
        out["ratios"] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
