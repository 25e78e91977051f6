"""Summarise tools/experiments/sq_counters.sh output per kernel (sum over the kernel's dispatches).

    python tools/experiments/sq_summary.py gpurun_out/sq [--kernel nn_lds_kernel] [--json out.json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--kernel", default="nn_lds_kernel")
    ap.add_argument("--json")
    a = ap.parse_args()
    tot: dict[str, float] = {}
    disp: dict[str, set] = {}
    for path in glob.glob(os.path.join(a.d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if a.kernel not in row["Kernel_Name"]:
                continue
            k = row["Counter_Name"]
            tot[k] = tot.get(k, 0.0) + float(row["Counter_Value"])
            disp.setdefault(k, set()).add(row["Dispatch_Id"])
    n = max((len(v) for v in disp.values()), default=1)
    per = {k: v / n for k, v in sorted(tot.items())}
    out = {"kernel": a.kernel, "dispatches": n, "per_dispatch": per}
    if "SQ_WAVE_CYCLES" in per and per["SQ_WAVE_CYCLES"]:
        wc = per["SQ_WAVE_CYCLES"]
        out["wait_any_frac"] = per.get("SQ_WAIT_ANY", 0) / wc
        out["wait_inst_any_frac"] = per.get("SQ_WAIT_INST_ANY", 0) / wc
        out["active_inst_frac"] = per.get("SQ_ACTIVE_INST_ANY", 0) / wc
    if per.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_frac"] = per.get("SQ_LDS_BANK_CONFLICT", 0) / per["SQ_LDS_IDX_ACTIVE"]
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
