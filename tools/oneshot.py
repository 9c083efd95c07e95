#!/usr/bin/env python3
"""One-shot read ceiling of the config-3 launch shape (tools/hbm_copy.hip
hbm_oneshot): 256 workgroups each reading a 69,632-B slice of a K cache and of
a V cache (35.65 MB per launch), over 16 rotated cache pairs, LDS-DMA or
register loads, 4 / 8 / 16 waves, one step or all in flight; plus the same
bytes over 512 / 1024 workgroups.  Prints one line per variant and a JSON
summary.  (A measurement probe; never part of libfattn.)"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load():
    import torch  # noqa: F401  (one HIP runtime with torch)
    L = C.CDLL(os.path.join(ROOT, "ggml-cuda-experiments_amd", "lib", "libhbmcopy.so"))
    L.hbm_oneshot.restype = C.c_float
    L.hbm_oneshot.argtypes = [C.c_uint, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    return L


def main():
    L = load()
    per = 69632
    alg = 35692544  # config 3's algorithmic bytes (K + V + Q + O + mask)
    kv = 2 * 256 * per
    modes = {0: "ldsdma_all_in_flight", 1: "ldsdma_2steps_1_in_flight", 2: "vgpr_all_in_flight"}
    rows = []
    for wgs, pw in ((256, per), (512, per // 2), (1024, per // 4)):
        for waves in (4, 8, 16):
            for mode in (0, 1, 2):
                if pw // 1024 < waves:
                    continue
                reps = []
                for _ in range(3):
                    reps.append(L.hbm_oneshot(pw, wgs, waves, mode, 16, 200))
                us = min(reps)
                r = {"wgs": wgs, "waves": waves, "mode": modes[mode], "us": round(us, 3),
                     "reps_us": [round(x, 3) for x in reps],
                     "kv_TBps": round(kv / (us * 1e-6) / 1e12, 3) if us > 0 else None}
                rows.append(r)
                print(json.dumps(r), flush=True)
    best = min((r for r in rows if r["us"] > 0), key=lambda r: r["us"])
    print(json.dumps({"best": best, "alg_bytes": alg,
                      "peak_measured_oneshot_GBps": round(alg / (best["us"] * 1e-6) / 1e9, 1)}))


if __name__ == "__main__":
    sys.exit(main())
