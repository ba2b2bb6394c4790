"""Summarise tools/gpu/sq_train.sh into profiles/<round>/train/sq_counters.json: per kernel
(and per launch shape), per-dispatch means of each SQ counter, the MFMA pipe's busy
fraction, the effective clock (GRBM_GUI_ACTIVE over the dispatch's duration) and VALU /
LDS instructions per MFMA.

    python tools/sq_train_summary.py gpurun_out/sq_train profiles/round2/train
"""
import csv
import json
import os
import sys


def main(src, dest):
    per = {}
    for p in ("p1", "p2"):
        for r in csv.DictReader(open(os.path.join(src, p, "run_counter_collection.csv"))):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].strip()
            key = (name, r.get("Grid_Size", r.get("Grid_Size_X", "")), r.get("LDS_Block_Size", ""))
            d = per.setdefault(key, {}).setdefault(r["Counter_Name"], [])
            d.append(float(r["Counter_Value"]))
    out = {}
    for (name, grid, lds), cnt in sorted(per.items()):
        c = {k: sum(v) / len(v) for k, v in cnt.items()}
        if "GRBM_GUI_ACTIVE" not in c or "SQ_INSTS_MFMA" not in c:
            continue
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        d = {"dispatches": len(cnt["SQ_INSTS_MFMA"]) if "SQ_INSTS_MFMA" in cnt else 0,
             "kernel_cycles_per_xcd": cyc,
             "mfma_pipe_busy_frac": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (cyc * 1024),
             "valu_insts_per_mfma": c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"],
             "lds_insts_per_mfma": c["SQ_INSTS_LDS"] / c["SQ_INSTS_MFMA"],
             "wait_inst_any_per_wave_cycle": c["SQ_WAIT_INST_ANY"] / max(c["SQ_WAVE_CYCLES"], 1),
             "wait_any_per_wave_cycle": c["SQ_WAIT_ANY"] / max(c["SQ_WAVE_CYCLES"], 1),
             "lds_bank_conflict_cycles": c.get("SQ_LDS_BANK_CONFLICT", 0)}
        out[f"{name} grid={grid} lds={lds}"] = {"derived": d, "counters": c}
    os.makedirs(dest, exist_ok=True)
    json.dump({"source": "tools/gpu/sq_train.sh (two rocprofv3 --pmc passes over tools/train_profile.py 2)",
               "kernels": out}, open(os.path.join(dest, "sq_counters.json"), "w"), indent=1)
    for k, v in out.items():
        print(k, json.dumps({a: round(b, 4) for a, b in v["derived"].items()}))


if __name__ == "__main__":
    main(*sys.argv[1:])
