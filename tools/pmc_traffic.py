"""Summarise rocprofv3 output into profiles/ (run on the dev box after gpurun merged gpurun_out/).

    python tools/pmc_traffic.py --stats gpurun_out/prof_stats --fetch gpurun_out/prof_fetch \
        --write gpurun_out/prof_write --pairs 1024 --points 8192 --tag r01

* kernel stats (--kernel-trace --stats): per-kernel calls / average duration -> profiles/kernel_stats_<tag>.csv
* HBM traffic of the NN kernel per launch from the PMC passes, corrected as MI355X_MICROARCH.md §HBM
  prescribes: FETCH_SIZE reports half the bytes of a wide coalesced streaming read on gfx950, so it
  is doubled; WRITE_SIZE is taken as-is.  Units: FETCH_SIZE / WRITE_SIZE are in KiB.
  -> profiles/pmc_traffic.json (read by bench.py for roofline.traffic), with a per-kernel table
  (`kernels`) for every kernel of --also (fold_update_kernel, index_kernel, ...): mean FETCH
  (doubled) + WRITE bytes per launch and the average duration
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(d: str, pattern: str) -> list[str]:
    return sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))


def counters(d: str, name: str, kernel_sub: str) -> list[float]:
    vals = []
    for path in find(d, "*counter_collection.csv"):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == name and kernel_sub in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--tag", default="round1", help="profiles/<tag>/ receives the kernel stats")
    ap.add_argument("--kernel", default="nn_lds_kernel", help="kernel name (substring match in the PMC CSV)")
    ap.add_argument("--also", default="fold_update_kernel,index_kernel,nn_cache_test_kernel,nn_order_kernel,init_kernel,"
                                      "fitness_prep_kernel,finish_kernel",
                    help="comma-separated kernels for the per-kernel traffic table")
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    out = {"pairs": a.pairs, "points": a.points, "kernel": a.kernel, "tag": a.tag}
    if a.stats:
        st = find(a.stats, "*kernel_stats.csv")
        if st:
            dst = os.path.join(ROOT, "profiles", a.tag, "kernel_stats.csv")
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            shutil.copy(st[0], dst)
            with open(st[0]) as f:
                for row in csv.DictReader(f):
                    if a.kernel in row["Name"]:
                        out.setdefault("stats", []).append({k: row[k] for k in ("Name", "Calls", "AverageNs", "Percentage")
                                                            if k in row})
    if a.fetch:
        fs = counters(a.fetch, "FETCH_SIZE", a.kernel)
        if fs:
            kib = statistics.fmean(fs)  # launches differ per ICP pass: the mean matches the avg launch time
            out["fetch_size_kib_mean"] = kib
            out["fetch_bytes_corrected"] = 2.0 * kib * 1024
            out["fetch_dispatches"] = len(fs)
    if a.write:
        ws = counters(a.write, "WRITE_SIZE", a.kernel)
        if ws:
            kib = statistics.fmean(ws)
            out["write_size_kib_mean"] = kib
            out["write_bytes"] = kib * 1024
            out["write_dispatches"] = len(ws)
    if "fetch_bytes_corrected" in out and "write_bytes" in out:
        out["hbm_bytes_per_nn_launch"] = out["fetch_bytes_corrected"] + out["write_bytes"]

    table = {}
    for k in [a.kernel] + [x for x in a.also.split(",") if x]:
        row = {}
        fs = counters(a.fetch, "FETCH_SIZE", k) if a.fetch else []
        ws = counters(a.write, "WRITE_SIZE", k) if a.write else []
        if fs:
            row["fetch_bytes_corrected"] = 2.0 * statistics.fmean(fs) * 1024
            row["dispatches"] = len(fs)
        if ws:
            row["write_bytes"] = statistics.fmean(ws) * 1024
        if fs and ws:
            row["hbm_bytes_per_launch"] = row["fetch_bytes_corrected"] + row["write_bytes"]
        if a.stats:
            for path in find(a.stats, "*kernel_stats.csv"):
                with open(path) as f:
                    for r in csv.DictReader(f):
                        if k in r["Name"]:
                            row["avg_ns"] = float(r["AverageNs"])
                            row["calls"] = int(r["Calls"])
        if "hbm_bytes_per_launch" in row and "avg_ns" in row:
            row["hbm_gbs"] = row["hbm_bytes_per_launch"] / row["avg_ns"]
        if row:
            table[k] = row
    out["kernels"] = table

    if a.fetch or a.write:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
