#!/usr/bin/env python3
"""Print name / calls / average ns of the fattn kernels in rocprofv3
kernel_stats.csv files (kernel names contain commas: parsed as CSV)."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        if "fattn" in r["Name"]:
            name = r["Name"].replace("void fattn::", "").replace("(fattn::SplitArgs)", "")
            print(f"   {name:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1000:8.2f} us")
