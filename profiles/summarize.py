"""Summarise a rocprofv3 collection (profiles/collect.sh) into per-kernel numbers.

    python profiles/summarize.py gpurun_out/prof_r01 profiles/r01

Writes <dest>/summary.json and refreshes profiles/pmc_latest.json (read by
bench.py for the roofline's ``traffic`` field).  HBM bytes per launch follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE counts half the bytes of a wide (16 B/lane) coalesced read, so it is
doubled (the MLP kernel's reads are 16-B LDS-DMA weight pieces); WRITE_SIZE is
exact for 16-B-per-lane stores.
"""
from __future__ import annotations

import csv
import json
import os
import shutil
import sys


def per_kernel(path, counter, by_grid=False):
    acc = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        key = (r["Kernel_Name"], int(r["Grid_Size"])) if by_grid else r["Kernel_Name"]
        acc.setdefault(key, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def trace_by_grid(path):
    """Mean duration per (kernel, grid size) from the kernel trace."""
    acc = {}
    for r in csv.DictReader(open(path)):
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        acc.setdefault((r["Kernel_Name"], grid), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return {k: (len(v), sum(v) / len(v)) for k, v in acc.items()}


def main(src: str, dest: str) -> None:
    os.makedirs(dest, exist_ok=True)
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                            "pct": float(r["Percentage"])}
    fetch = per_kernel(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    for k in stats:
        f, w = fetch.get(k), write.get(k)
        if f is not None and w is not None:
            stats[k]["fetch_bytes_raw"] = f * 1024
            stats[k]["write_bytes"] = w * 1024
            stats[k]["hbm_bytes_per_launch"] = 2 * f * 1024 + w * 1024
    # per launch size (grid = threads): the same kernel runs several configurations
    # (e.g. the bf16 MLP on 128-, 64- and 192-sample passes); bench.py picks the
    # headline launch by its grid
    fg = per_kernel(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE", True)
    wg = per_kernel(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE", True)
    tg = trace_by_grid(os.path.join(src, "trace", "run_kernel_trace.csv"))
    for (name, grid), (calls, ms) in tg.items():
        if name not in stats:
            continue
        e = {"calls": calls, "avg_ms": ms}
        f, w = fg.get((name, grid)), wg.get((name, grid))
        if f is not None and w is not None:
            e.update({"fetch_bytes_raw": f * 1024, "write_bytes": w * 1024, "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024})
        stats[name].setdefault("by_grid", {})[str(grid)] = e
    out = {"source": src, "kernels": stats}
    json.dump(out, open(os.path.join(dest, "summary.json"), "w"), indent=1)
    shutil.copy(os.path.join(dest, "summary.json"), os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                  "pmc_latest.json"))
    for name in ("run_kernel_stats.csv",):
        shutil.copy(os.path.join(src, "trace", name), os.path.join(dest, "kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
