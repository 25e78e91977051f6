"""Summarise rocprofv3 output of one benchmark config into profiles/ (tools/profile_round.sh runs it).

    python tools/pmc_traffic.py --config C3 --stats DIR --fetch DIR --write DIR --tag round3

* kernel stats (--kernel-trace --stats): copied to profiles/<tag>/kernel_stats_<config>.csv
* HBM traffic per launch of every kernel of --kernels from the PMC passes, corrected as
  MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE reports half the bytes of a wide coalesced streaming
  read on gfx950, so it is doubled; WRITE_SIZE is taken as-is.  Units: FETCH_SIZE / WRITE_SIZE are
  in KiB.  Launches differ per ICP pass: the mean over the launches matches the average launch time.
  -> profiles/pmc_traffic.json, under configs[<config>][<kernel>], stamped with the sha256 of the
  library build that was profiled and of the ICP kernels' sources (tools/srchash.py): bench.py uses a
  row only when its own library, or failing that its ICP kernel sources, have that hash.
"""
from __future__ import annotations

import argparse
import csv
import glob
import hashlib
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "icp-4dradar_amd", "icp4r", "_lib", "libicp4r.so")
OUT = os.path.join(ROOT, "profiles", "pmc_traffic.json")
KERNELS = ("nn_lds_kernel,nn_tile_kernel,fold_update_kernel,fold_update_wide_kernel,fold_update_held_kernel,fold_update_res_kernel,index_kernel,src_order_kernel,index_refine_kernel,"
           "nn_seed_kernel,nn_cache_test_kernel,nn_order_kernel,init_kernel,fitness_prep_kernel,finish_kernel,"
           "solo_kernel,corr_kernel")


def find(d: str, pattern: str) -> list[str]:
    return sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))


def short(name: str) -> str:
    """'void icp4r::nn_lds_kernel<true>(icp4r::PairArgs, ...)' -> 'nn_lds_kernel'."""
    s = name.split("(")[0].split("<")[0]
    return s.rsplit("::", 1)[-1].replace("void ", "").strip()


def counters(d: str, name: str, kernel: str) -> list[float]:
    vals = []
    for path in find(d, "*counter_collection.csv"):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == name and short(row.get("Kernel_Name", "")) == kernel:
                    vals.append(float(row["Counter_Value"]))
    return vals


def stats(d: str) -> dict:
    out = {}
    for path in find(d, "*kernel_stats.csv"):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = short(r["Name"])
                out[k] = {"avg_ns": float(r["AverageNs"]), "calls": int(r["Calls"]),
                          "percentage": float(r.get("Percentage", "nan"))}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True, help="C1 / C2 / C3 / C5 (bench.py's config names)")
    ap.add_argument("--stats")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--tag", default="round3", help="profiles/<tag>/ receives the kernel stats")
    ap.add_argument("--kernels", default=KERNELS)
    ap.add_argument("--library", default=LIB)
    a = ap.parse_args()
    with open(a.library, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    try:
        with open(OUT) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        doc = {}
    from srchash import icp_sources_sha256

    src = icp_sources_sha256()
    if doc.get("library_sha256") != sha:  # rows of another build are stale: start over
        doc = {"library_sha256": sha, "configs": {}}
    doc["icp_sources_sha256"] = src  # (tools/srchash.py: the ICP kernels' sources, headers and flags)
    doc["tag"] = a.tag
    doc["note"] = ("HBM bytes per launch: FETCH_SIZE x 2 (gfx950: FETCH_SIZE reports half of a wide streaming "
                   "read) + WRITE_SIZE, KiB -> bytes, mean over the launches of the profiled run "
                   "(MI355X_MICROARCH.md §HBM); avg_ns from the separate --kernel-trace --stats run")
    st = stats(a.stats) if a.stats else {}
    if a.stats:
        src = find(a.stats, "*kernel_stats.csv")
        if src:
            dst = os.path.join(ROOT, "profiles", a.tag, f"kernel_stats_{a.config}.csv")
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            shutil.copy(src[0], dst)
    table = {}
    for k in [x for x in a.kernels.split(",") if x]:
        row = {}
        fs = counters(a.fetch, "FETCH_SIZE", k) if a.fetch else []
        ws = counters(a.write, "WRITE_SIZE", k) if a.write else []
        if fs:
            row["fetch_size_kib_mean"] = statistics.fmean(fs)
            row["fetch_bytes_corrected"] = 2.0 * row["fetch_size_kib_mean"] * 1024
            row["fetch_dispatches"] = len(fs)
        if ws:
            row["write_size_kib_mean"] = statistics.fmean(ws)
            row["write_bytes"] = row["write_size_kib_mean"] * 1024
            row["write_dispatches"] = len(ws)
        if fs and ws:
            row["hbm_bytes_per_launch"] = row["fetch_bytes_corrected"] + row["write_bytes"]
        if k in st:
            row.update(st[k])
        if "hbm_bytes_per_launch" in row and "avg_ns" in row:
            row["hbm_gbs"] = row["hbm_bytes_per_launch"] / row["avg_ns"]
        if row:
            table[k] = row
    doc.setdefault("configs", {})[a.config] = table
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps({a.config: table}, indent=1))


if __name__ == "__main__":
    main()
