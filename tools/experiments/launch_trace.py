"""Ordered kernel launches from a rocprofv3 rocpd database (per-launch durations, e.g. of the NN pass
of every ICP iteration).

    python tools/experiments/launch_trace.py gpurun_out/prof/run_results.db [--last 48] [--match nn_]
"""
from __future__ import annotations

import argparse
import glob
import os
import sqlite3

from rocpd_stats import short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=48)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    path = a.db
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))[-1]
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = db.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
    rows = [(short(n), int(e) - int(s)) for n, s, e in rows if a.match in short(n)]
    for k, (n, d) in enumerate(rows[-a.last:]):
        print(f"{k:4d} {d / 1000.0:10.1f} us  {n}")


if __name__ == "__main__":
    main()
