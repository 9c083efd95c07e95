#!/usr/bin/env python3
"""Print name / calls / average of the fattn kernels in rocprofv3 kernel
statistics (kernel names contain commas: parsed as CSV).

  kstats.py run_kernel_stats.csv          per kernel name (rocprofv3's own summary)
  kstats.py run_kernel_trace.csv          per (kernel name, grid): one launch shape per line, so the
                                          bench's config-3 split kernel and the same instantiation on the
                                          64-sequence side line (another grid) are averaged apart
"""
import csv
import statistics
import sys
from collections import defaultdict


def short(n):
    return n.replace("void fattn::", "").replace("(fattn::SplitArgs)", "")


for path in sys.argv[1:]:
    print("==", path)
    rows = list(csv.DictReader(open(path)))
    if rows and "AverageNs" in rows[0]:
        for r in rows:
            if "fattn" in r["Name"]:
                print(f"   {short(r['Name']):60s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1000:8.2f} us")
        continue
    by = defaultdict(list)
    for r in rows:
        if "fattn" not in r["Kernel_Name"]:
            continue
        grid = tuple(int(r[f"Grid_Size_{a}"]) // max(1, int(r[f"Workgroup_Size_{a}"])) for a in "XYZ")
        by[(short(r["Kernel_Name"]), grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    for (name, grid), v in sorted(by.items(), key=lambda kv: -len(kv[1])):
        print(f"   {name:60s} grid {str(grid):16s} calls {len(v):5d} avg {statistics.fmean(v):8.2f} us "
              f"median {statistics.median(v):8.2f}")
