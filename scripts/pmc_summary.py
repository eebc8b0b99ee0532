"""Summarise rocprofv3 --pmc counter CSVs of GEMM runs (scripts/gemm_one.py): per kernel, the mean
over its dispatches of each counter, plus MFMA-busy % = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8
XCDs x CUs x 4 SIMDs) and the effective clock (GRBM_GUI_ACTIVE / 8 / kernel time).

    python scripts/pmc_summary.py OUT.json LABEL=DIR [LABEL=DIR ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(d: str, n_cu: int = 256):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for r in rows:
        k = r["Kernel_Name"]
        if "gemm" not in k.lower() and "Cijk" not in k:
            continue
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        t = sum(dur[k].values()) / max(1, len(dur[k]))
        g = m.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            m["mfma_busy_pct"] = 100.0 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * n_cu * 4)
        if g and t > 0:
            m["eff_clock_ghz"] = g / 8 / t / 1e9
        m["kernel_s"] = t
        out[k[:90]] = {a: round(b, 4) for a, b in m.items()}
    return out


def main():
    res = {}
    for arg in sys.argv[2:]:
        label, d = arg.split("=", 1)
        res[label] = summarise(d)
        for k, m in res[label].items():
            print(label, k[:60], json.dumps({a: m[a] for a in ("mfma_busy_pct", "eff_clock_ghz", "kernel_s") if a in m}))
    with open(sys.argv[1], "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
