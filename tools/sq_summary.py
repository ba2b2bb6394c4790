"""Summarise tools/pmc_sq.sh passes into profiles/<round>/<precision>/sq_counters.json.

    python tools/sq_summary.py gpurun_out/sq_<precision> profiles/<round>/<precision> <precision>

Per-dispatch means of each counter; derived: the MFMA pipe's busy fraction
(SQ_VALU_MFMA_BUSY_CYCLES over the dispatch's cycles x 1,024 SIMDs; GRBM_GUI_ACTIVE
counts cycles summed over the 8 XCDs), MFMAs per wave per 32-sample column tile,
VALU and LDS instructions per MFMA, and the effective clock implied by the
kernel's rocprofv3 duration (summary.json beside it)."""
import csv
import json
import os
import sys


def _lab_ms(path):
    """median_ms from the kernel_lab.py JSON a counter pass printed, or None."""
    try:
        txt = open(path).read()
        return float(next(iter(json.loads(txt[txt.index("{"):txt.rindex("}") + 1]).values()))["median_ms"])
    except (OSError, ValueError, StopIteration, KeyError):
        return None


def main(src, dest, prec):
    cnt = {}
    for p in ("p1", "p2"):
        acc = {}
        for r in csv.DictReader(open(os.path.join(src, p, "run_counter_collection.csv"))):
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        cnt.update({k: sum(v) / len(v) for k, v in acc.items()})
    cycles_xcd = cnt["GRBM_GUI_ACTIVE"] / 8
    wave_tiles = 61.44e6 / 32                       # 800x600x128 samples in 32-sample column tiles
    d = {"kernel_cycles_per_xcd": cycles_xcd,
         "mfma_pipe_busy_frac": cnt["SQ_VALU_MFMA_BUSY_CYCLES"] / (cycles_xcd * 1024),
         "mfma_per_wave_tile": cnt["SQ_INSTS_MFMA"] / wave_tiles,
         "valu_insts_per_mfma": cnt["SQ_INSTS_VALU"] / cnt["SQ_INSTS_MFMA"],
         "lds_insts_per_mfma": cnt["SQ_INSTS_LDS"] / cnt["SQ_INSTS_MFMA"],
         "lds_bank_conflict_cycles": cnt["SQ_LDS_BANK_CONFLICT"]}
    summ = os.path.join(dest, "summary.json")
    lab = _lab_ms(os.path.join(src, "p2.log"))
    if lab:   # the counter pass's own kernel time (kernel_lab.py's HIP events, same dispatches)
        d["kernel_ms_counter_pass"] = lab
        d["effective_clock_ghz"] = cycles_xcd / (lab * 1e-3) / 1e9
    elif os.path.exists(summ):
        key = {"f16x3": "mlp_x3_kernel<OpF16>", "bf16x3": "mlp_x3_kernel<OpBf16>"}.get(prec, f"mlp_{prec}_kernel")
        k = json.load(open(summ))["kernels"].get(key)
        if k:
            d["effective_clock_ghz"] = cycles_xcd / (k["avg_ms"] * 1e-3) / 1e9
    os.makedirs(dest, exist_ok=True)
    out = {"source": f"tools/pmc_sq.sh {prec} (two rocprofv3 --pmc passes over tools/kernel_lab.py, 800x600x128, "
                     f"per-dispatch means)", "counters": cnt, "derived": d}
    json.dump(out, open(os.path.join(dest, "sq_counters.json"), "w"), indent=1)
    print(prec, json.dumps(d))


if __name__ == "__main__":
    main(*sys.argv[1:4])
