"""Per-dispatch PMC values of one kernel, grouped by ICP pass (rocprofv3 --pmc ... --kernel-trace output).

    python tools/experiments/pmc_dispatch.py --dir gpurun_out/prof_C3_write --counter WRITE_SIZE \
        --kernel nn_lds_kernel --per-reg 21

The launches of one registration come in a fixed order (C3, one pair group: 21 searches = 20 ICP passes
+ the fitness pass), so dispatch k of the kernel belongs to pass k mod per_reg.  Prints, per pass, the
mean counter value over the registrations (FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM; both in
MB) as JSON lines.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pmc_traffic import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--counter", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--per-reg", type=int, default=21)
    a = ap.parse_args()
    rows = []
    for path in sorted(glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") == a.counter and short(r.get("Kernel_Name", "")) == a.kernel:
                    rows.append((int(r.get("Dispatch_Id", 0)), float(r["Counter_Value"])))
    rows.sort()
    scale = (2.0 if a.counter == "FETCH_SIZE" else 1.0) * 1024 / 1e6  # KiB -> MB
    per = {}
    for k, (_, v) in enumerate(rows):
        per.setdefault(k % a.per_reg, []).append(v * scale)
    for k in sorted(per):
        vs = per[k]
        print(json.dumps({"kernel": a.kernel, "counter": a.counter, "pass": k + 1, "mean_mb": sum(vs) / len(vs),
                          "n": len(vs)}))
    allv = [v for vs in per.values() for v in vs]
    if allv:
        print(json.dumps({"kernel": a.kernel, "counter": a.counter, "pass": "all", "mean_mb": sum(allv) / len(allv),
                          "n": len(allv)}))


if __name__ == "__main__":
    main()
