#!/usr/bin/env python3
"""Summarise rocprofv3 counter-collection CSVs for one kernel.

  pmc_summary.py --kernel fattn_split_kernel a.csv [b.csv ...]
      per counter: dispatches, mean / min / max value per dispatch
  --traffic OUT.json --bench-line BENCH.log
      HBM bytes per launch from FETCH_SIZE and WRITE_SIZE, corrected as
      MI355X_MICROARCH.md prescribes (FETCH_SIZE is KiB and reports 1/2 of
      16-B/lane streaming reads on gfx950: x 1024 x 2; WRITE_SIZE x 1024),
      tagged with the workload, the plan (describe string) and the kernel
      source hash of the bench.py JSON line of the same command (bench.py
      reads a traffic file back only when all three match)
  --kernel a,b,c --sum-kernels
      several kernels of one launch (the staged prefill: kv_stage_f16,
      pf_mask_flags_kernel, the prefill body): per counter the sum over the
      kernels of each one's mean per dispatch
  --mfma
      MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x CUs x cycles),
      cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs)
"""
import argparse
import csv
import json
import statistics
import sys
from collections import defaultdict


def load(paths, kernel, per_kernel=False):
    """counter -> per-dispatch values (per_kernel: (kernel name, counter) -> values)"""
    vals = defaultdict(list)
    names = set()
    pats = kernel.split(",")
    for p in paths:
        with open(p, newline="") as f:
            for row in csv.DictReader(f):
                if not any(k in row["Kernel_Name"] for k in pats):
                    continue
                names.add(row["Kernel_Name"])
                key = (row["Kernel_Name"], row["Counter_Name"]) if per_kernel else row["Counter_Name"]
                vals[key].append(float(row["Counter_Value"]))
    return vals, sorted(names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--traffic")
    ap.add_argument("--workload", default="")
    ap.add_argument("--alg-bytes", type=float, default=0.0)
    ap.add_argument("--bench-line", default="", help="log holding the bench.py JSON line of the profiled command")
    ap.add_argument("--command", default="")
    ap.add_argument("--mfma", action="store_true")
    ap.add_argument("--sum-kernels", action="store_true", help="sum the per-kernel means (several kernels per launch)")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("csv", nargs="+")
    a = ap.parse_args()
    vals, names = load(a.csv, a.kernel, per_kernel=a.sum_kernels)
    if not vals:
        sys.exit(f"no dispatch of a kernel matching {a.kernel!r}")
    if a.sum_kernels:
        per = {}
        for (kn, c), v in sorted(vals.items()):
            print(f"  {kn[:70]:70s} {c:16s} n={len(v):4d} mean={statistics.fmean(v):.6g}")
            d = per.setdefault(c, {"dispatches": 0, "mean": 0.0, "min": 0.0, "max": 0.0})
            d["dispatches"] += len(v)
            d["mean"] += statistics.fmean(v)
            d["min"] += min(v)
            d["max"] += max(v)
        summ = per
    else:
        summ = {c: {"dispatches": len(v), "mean": statistics.fmean(v), "min": min(v), "max": max(v)}
                for c, v in sorted(vals.items())}
    print("kernels:", "; ".join(names))
    for c, s in summ.items():
        print(f"{c:32s} n={s['dispatches']:5d} mean={s['mean']:.6g} min={s['min']:.6g} max={s['max']:.6g}")
    if a.mfma:
        busy, gui = summ.get("SQ_VALU_MFMA_BUSY_CYCLES"), summ.get("GRBM_GUI_ACTIVE")
        if busy and gui:
            cyc = gui["mean"] / 8
            util = busy["mean"] / (4 * a.cus * cyc)
            print(f"MFMA busy / (4 x {a.cus} x GRBM_GUI_ACTIVE/8) = {util:.4f}  (kernel cycles {cyc:.0f})")
        if "SQ_INSTS_MFMA" in summ and "SQ_INSTS_VALU" in summ:
            print(f"VALU per MFMA instruction = {summ['SQ_INSTS_VALU']['mean'] / summ['SQ_INSTS_MFMA']['mean']:.3f}")
    plan, shash = "", ""
    if a.bench_line:
        for ln in open(a.bench_line):
            if ln.startswith('{"metric"'):
                bl = json.loads(ln)
                a.workload = a.workload or bl["config"]["workload"]
                a.alg_bytes = a.alg_bytes or float(bl["config"]["bytes_per_step"])
                plan, shash = bl["roofline"]["kernel"], bl["source_hash"]
    if a.traffic:
        fetch, write = summ["FETCH_SIZE"], summ["WRITE_SIZE"]
        fb = fetch["mean"] * 1024 * 2
        wb = write["mean"] * 1024
        out = {
            "workload": a.workload,
            "plan": plan,
            "source_hash": shash,
            "kernel": names[0] if len(names) == 1 else names,
            "command": a.command,
            "counters": {"FETCH_SIZE": {"dispatches": fetch["dispatches"], "mean_kb": fetch["mean"],
                                        "min_kb": fetch["min"], "max_kb": fetch["max"]},
                         "WRITE_SIZE": {"dispatches": write["dispatches"], "mean_kb": write["mean"],
                                        "min_kb": write["min"], "max_kb": write["max"]}},
            "fetch_bytes_corrected": fb,
            "write_bytes": wb,
            "hbm_bytes_per_launch": int(round(fb + wb)),
            "algorithmic_bytes_per_launch": int(a.alg_bytes),
            "traffic_over_algorithmic": round((fb + wb) / a.alg_bytes, 4) if a.alg_bytes else None,
            "correction": "FETCH_SIZE x 1024 x 2 (gfx950 reports 1/2 of 16-B/lane streaming reads); WRITE_SIZE x 1024",
        }
        with open(a.traffic, "w") as f:
            json.dump(out, f, indent=1)
        print("wrote", a.traffic, "hbm_bytes_per_launch", out["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main()
