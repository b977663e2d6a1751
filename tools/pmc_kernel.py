#!/usr/bin/env python3
"""Per-dispatch PMC averages of one kernel (name substring) over a rocprofv3 output directory tree, with
the usual ratios.   python tools/pmc_kernel.py gpurun_out/dn_b jbf_lds [--units N]"""
import collections
import csv
import glob
import sys

src, name = sys.argv[1], sys.argv[2]
units = float(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[3] == "--units" else None
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in glob.glob(f"{src}/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if name in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
c = {k: v / len(disp[k]) for k, v in tot.items()}
for k, v in sorted(c.items()):
    print(f"{k:32s} {v:.4g}")
g = c.get
if g("SQ_WAVE_CYCLES"):
    print("wait_any/wave_cycles", round(g("SQ_WAIT_ANY", 0) / g("SQ_WAVE_CYCLES"), 3))
if g("SQ_ACTIVE_INST_VALU"):
    print("valu lane util", round(g("SQ_THREAD_CYCLES_VALU", 0) / (g("SQ_ACTIVE_INST_VALU") * 64), 3))
if g("TCC_HIT_sum") is not None:
    print("L2 hit", round(g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")), 3))
if g("GRBM_GUI_ACTIVE") and g("SQ_INSTS_VALU"):
    # GRBM_GUI_ACTIVE is summed over XCDs by rocprofv3 (8 per dispatch); VALU issue = wave-insts x 2 cycles / SIMD-cycles
    cyc = g("GRBM_GUI_ACTIVE") / 8
    print("valu issue frac", round(g("SQ_INSTS_VALU") * 2 / (1024 * cyc), 3), "kernel cycles", f"{cyc:.4g}")
if units and g("SQ_INSTS_VALU"):
    print("valu lane-slots per unit", round(g("SQ_INSTS_VALU") * 64 / units, 2), "lds insts per unit", round(g("SQ_INSTS_LDS", 0) * 64 / units, 2))
