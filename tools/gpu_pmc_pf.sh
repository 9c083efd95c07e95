#!/bin/bash
# PMC passes on the prefill kernel (no mask), one rocprofv3 run per pass
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="python3 bench.py --n-q 4096 --steps 3 --warmup 1 --rotate 2 --no-cpu-baseline --no-prefill"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $P1 -d $R/gpurun_out/pmc_pf1 -o run --output-format csv -- $B > $R/gpurun_out/pmc_pf1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $P2 -d $R/gpurun_out/pmc_pf2 -o run --output-format csv -- $B > $R/gpurun_out/pmc_pf2.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections, os
R = os.environ["GRAFT_REPO_ROOT"]
for d in ("pmc_pf1", "pmc_pf2"):
    for f in glob.glob(f"{R}/gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(list)
        for row in csv.DictReader(open(f)):
            if "pf_kernel" in row.get("Kernel_Name", ""):
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
        for k, v in sorted(acc.items()):
            print(d, k, "per-dispatch mean %.4g" % (sum(v) / len(v)), "n", len(v))
PY
