#!/usr/bin/env python3
"""Keep only what the VALU roofline reads from rocprofv3 output directories
(tools/pmc_valu.py): rows of the product's kernels (names with "nh::") in the
counter-collection and kernel-trace CSVs, and the kernel stats; everything else
is deleted.  The torch kernels' multi-KB names otherwise blow gpurun_out/ past
its copy-back limit.   Usage: trim_prof.py DIR [DIR ...]"""
import csv
import glob
import os
import sys

csv.field_size_limit(1 << 30)
for d in sys.argv[1:]:
    for p in glob.glob(os.path.join(d, "**", "*"), recursive=True):
        if not os.path.isfile(p):
            continue
        base = os.path.basename(p)
        if base.endswith("kernel_stats.csv"):
            rows = list(csv.reader(open(p)))
            keep = [rows[0]] + [r for r in rows[1:] if "nh::" in r[0]]
        elif base.endswith(("counter_collection.csv", "kernel_trace.csv")):
            rows = list(csv.reader(open(p)))
            ki = rows[0].index("Kernel_Name")
            keep = [rows[0]] + [r for r in rows[1:] if "nh::" in r[ki]]
        else:
            os.remove(p)
            continue
        with open(p, "w", newline="") as f:
            csv.writer(f).writerows(keep)
