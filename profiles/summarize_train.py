"""Summarise the training-step rocprofv3 collection (tools/gpu/profile_train.sh).

    python profiles/summarize_train.py gpurun_out/prof_train profiles/round2/train

The GEMM dispatches are grouped by grid (the three GEMM kinds of one net have
distinct grids: forward and backward-data [P/128, N/128, 1], weight gradients
[M/128, N/128, splits]); per group: dispatches per step, mean duration, and HBM
bytes per dispatch from the separate FETCH_SIZE / WRITE_SIZE passes (KiB;
FETCH_SIZE doubled for gfx950's 16-B-per-lane reads, MI355X_MICROARCH.md §HBM).
The trace covers 8 steps (2 warm-up, 5, 1 final), each PMC pass 5.
"""
from __future__ import annotations

import csv
import json
import os
import shutil
import sys


def grid_key(r, x="Grid_Size_X", y="Grid_Size_Y", z="Grid_Size_Z"):
    return f"{int(r[x]) // 256}x{r[y]}x{r[z]}"


def main(src, dest, trace_steps=8, pmc_steps=5):
    os.makedirs(dest, exist_ok=True)
    groups = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
        name = r["Kernel_Name"]
        key = f"{name} {grid_key(r)}" if "gemm" in name else name
        groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pmc = {}
    for c, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        for r in csv.DictReader(open(os.path.join(src, sub, "run_counter_collection.csv"))):
            if r["Counter_Name"] != c:
                continue
            # counter CSV: Grid_Size is the flattened total; group GEMMs by it and the workgroup
            key = f"{r['Kernel_Name']} grid{r['Grid_Size']}" if "gemm" in r["Kernel_Name"] else r["Kernel_Name"]
            pmc.setdefault(key, {}).setdefault(c, []).append(float(r["Counter_Value"]))
    out = {"source": os.path.relpath(dest), "command": "tools/train_profile.py (main.py config: 2048 rays, 64+128)",
           "kernels": {}, "hbm": {}}
    step_us = 0.0
    for k, v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        out["kernels"][k] = {"per_step": len(v) / trace_steps, "avg_us": sum(v) / len(v),
                             "us_per_step": sum(v) / trace_steps}
        step_us += sum(v) / trace_steps
    out["kernel_us_per_step"] = step_us
    for k, d in pmc.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            f, w = d["FETCH_SIZE"], d["WRITE_SIZE"]
            out["hbm"][k] = {"dispatches": len(f), "hbm_bytes_per_dispatch": (2 * sum(f) + sum(w)) * 1024 / len(f),
                             "fetch_kib_avg": sum(f) / len(f), "write_kib_avg": sum(w) / len(w)}
    json.dump(out, open(os.path.join(dest, "summary.json"), "w"), indent=1)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dest, "kernel_stats.csv"))
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
