"""Per-kernel statistics from a rocprofv3 rocpd database (the image's rocprofv3 writes SQLite).

    python tools/experiments/rocpd_stats.py gpurun_out/prof_c3/run_results.db [--csv profiles/kernel_stats_<tag>.csv]

Prints name, calls, total/avg/min/max duration (ns) and share of GPU kernel time, like rocprofv3's
--stats kernel_stats.csv (same column names), sorted by total time.
"""
from __future__ import annotations

import argparse
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name)  # drop the argument list
    return name.replace("icp4r::", "")


def stats(db_path: str) -> list[dict]:
    db = sqlite3.connect(db_path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = db.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg: dict[str, list[int]] = {}
    for name, s, e in rows:
        agg.setdefault(short(name), []).append(int(e) - int(s))
    total = sum(sum(v) for v in agg.values()) or 1
    out = []
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        out.append({"Name": k, "Calls": len(v), "TotalDurationNs": sum(v), "AverageNs": sum(v) / len(v),
                    "Percentage": 100.0 * sum(v) / total, "MinNs": min(v), "MaxNs": max(v)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    a = ap.parse_args()
    st = stats(a.db)
    w = csv.DictWriter(sys.stdout, fieldnames=list(st[0].keys()))
    w.writeheader()
    w.writerows(st)
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(st[0].keys()))
            w.writeheader()
            w.writerows(st)


if __name__ == "__main__":
    main()
