"""Summarise a rocprofv3 collection (profiles/collect.sh) into per-kernel numbers.

    python profiles/summarize.py gpurun_out/prof_<tag> profiles/<round>/<tag>

Writes <dest>/summary.json, copies the trace's kernel_stats.csv and the JSON line
the profiled bench printed, and merges the MLP kernel's entry into
profiles/pmc_latest.json (read by bench.py for the roofline's ``traffic`` field).

The profiled command is the headline bench alone (collect.sh), so every MLP
dispatch in it is a headline launch.  HBM bytes per launch follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE counts half the bytes of a wide (16 B/lane) coalesced read, so it is
doubled (the MLP kernel's reads are 16-B LDS-DMA weight pieces); WRITE_SIZE is
exact for 16-B-per-lane stores (the MLP's float4 (sigma, rgb) stores).
"""
from __future__ import annotations

import csv
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


PRECISION = None      # the profiled command's --precision (set in main)


def kernel_key(name: str) -> str:
    """Short kernel names: the split kernels are one template (mlp_x3.h) that rocprofv3
    names `mlp_x3_kernel` either way; the profiled command's precision tells them apart
    (bench.py's roofline.kernel uses the same keys)."""
    if "mlp_x3_kernel" in name:
        f16 = "OpF16" in name or ("OpBf16" not in name and PRECISION == "f16x3")
        return "mlp_x3_kernel<OpF16>" if f16 else "mlp_x3_kernel<OpBf16>"
    for k in ("mlp_bf16_kernel", "mlp_fp8_kernel", "mlp_f32_kernel"):
        if k in name:
            return k
    return name


def per_kernel(path, counter):
    acc = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc.setdefault(kernel_key(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(src: str, dest: str) -> None:
    global PRECISION
    os.makedirs(dest, exist_ok=True)
    words = open(os.path.join(src, "command.txt")).read().split()
    PRECISION = words[words.index("--precision") + 1] if "--precision" in words else None
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        stats[kernel_key(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                            "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6,
                            "pct": float(r["Percentage"])}
    fetch = per_kernel(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    for k in stats:
        f, w = fetch.get(k), write.get(k)
        if f is not None and w is not None:
            stats[k]["fetch_size_kib"] = f
            stats[k]["write_size_kib"] = w
            stats[k]["hbm_bytes_per_launch"] = 2 * f * 1024 + w * 1024
    cmd = open(os.path.join(src, "command.txt")).read().strip()
    bench = open(os.path.join(src, "bench_under_rocprof.json")).read().strip()
    out = {"source": os.path.relpath(dest, os.path.dirname(HERE)), "command": "bench.py " + cmd,
           "bench_under_rocprof": json.loads(bench.splitlines()[-1]), "kernels": stats}
    # the profiled bench printed the traffic of the PREVIOUS collection (pmc_latest.json as it
    # stood); the summary carries this collection's own counters in its place and keeps the
    # printed value beside them, labelled
    roof = out["bench_under_rocprof"].get("roofline", {})
    k = roof.get("kernel")
    if k in stats and "hbm_bytes_per_launch" in stats[k]:
        roof["traffic_as_printed"] = roof.get("traffic")
        roof["traffic_as_printed_source"] = roof.get("traffic_source")
        roof["traffic"] = stats[k]["hbm_bytes_per_launch"]
        roof["traffic_source"] = (f"this collection's rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `{out['command']}` "
                                  f"({out['source']}); bytes/launch, FETCH_SIZE x2 (gfx950)")
    json.dump(out, open(os.path.join(dest, "summary.json"), "w"), indent=1)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dest, "kernel_stats.csv"))
    # merge the MLP kernels into pmc_latest.json (one entry per precision's kernel)
    latest_p = os.path.join(HERE, "pmc_latest.json")
    latest = json.load(open(latest_p)) if os.path.exists(latest_p) else {}
    latest = {"kernels": latest.get("kernels", {}) if "by_grid" not in json.dumps(latest) else {}}
    for k, v in stats.items():
        if k.startswith("mlp_") and "hbm_bytes_per_launch" in v:
            latest["kernels"][k] = dict(v, source=out["source"], command=out["command"])
    json.dump(latest, open(latest_p, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
