"""HBM traffic per launch of the decode kernel from two rocprofv3 PMC passes
(FETCH_SIZE, WRITE_SIZE), corrected as MI355X_MICROARCH.md's HBM section says:
KB units, and gfx950's FETCH_SIZE counting half of 16-B/lane streaming reads.

usage: python tools/traffic.py <fetch.csv> <write.csv> <workload> <alg_bytes> > profiles/traffic_r01.json
"""
import csv
import json
import sys


def per_dispatch(path, counter, kname="fattn_split_kernel"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kname in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return vals, r_kernel(path, kname)


def r_kernel(path, kname):
    for r in csv.DictReader(open(path)):
        if kname in r["Kernel_Name"]:
            return r["Kernel_Name"].replace("void fattn::", "").replace("(fattn::SplitArgs)", "")
    return None


def main():
    fetch_csv, write_csv, workload, alg = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    f, kern = per_dispatch(fetch_csv, "FETCH_SIZE")
    w, _ = per_dispatch(write_csv, "WRITE_SIZE")
    stat = lambda v: {"dispatches": len(v), "mean_kb": sum(v) / len(v), "min_kb": min(v), "max_kb": max(v)}
    fetch_b = sum(f) / len(f) * 1024 * 2
    write_b = sum(w) / len(w) * 1024
    out = {
        "workload": workload,
        "kernel": kern,
        "command": "rocprofv3 --pmc FETCH_SIZE (and separately WRITE_SIZE) -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline",
        "counters": {"FETCH_SIZE": stat(f), "WRITE_SIZE": stat(w)},
        "fetch_bytes_corrected": fetch_b,
        "write_bytes": write_b,
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": round((fetch_b + write_b) / alg, 4),
        "correction": "FETCH_SIZE x 1024 x 2 (gfx950 reports 1/2 of 16-B/lane streaming reads); WRITE_SIZE x 1024",
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
