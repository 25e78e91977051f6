"""Per-kernel durations and the idle gap before each, from a rocprofv3 kernel trace of
tools/experiments/c1_loop.py: registrations are cut at each init_kernel; the first few are dropped.

    python3 tools/experiments/trace_gaps.py <dir with *kernel_trace.csv> [skip]
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

d = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = []
for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").rsplit("::", 1)[-1]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
regs, cur = [], []
for r in rows:
    if r[2] == "init_kernel" and cur:
        regs.append(cur)
        cur = []
    cur.append(r)
regs.append(cur)
regs = [g for g in regs if g and g[0][2] == "init_kernel"][skip:]
dur, gap = defaultdict(list), defaultdict(list)
spans = []
for g in regs:
    spans.append((g[-1][1] - g[0][0]) / 1e3)
    for k, (s, e, nme) in enumerate(g):
        dur[nme].append((e - s) / 1e3)
        if k:
            gap[nme].append((s - g[k - 1][1]) / 1e3)
print(f"registrations {len(regs)}, span first start -> last end: median {statistics.median(spans):.1f} us")
tot_d = tot_g = 0.0
for nme in dur:
    per = len(dur[nme]) / len(regs)
    md = statistics.fmean(dur[nme])
    mg = statistics.fmean(gap[nme]) if gap[nme] else 0.0
    tot_d += md * per
    tot_g += mg * len(gap[nme]) / len(regs)
    print(f"{nme:28s} x{per:5.1f}  dur {md:7.2f} us (median {statistics.median(dur[nme]):6.2f}, min "
          f"{min(dur[nme]):6.2f})  gap before {mg:5.2f} us")
print(f"sum of durations {tot_d:.1f} us, of gaps {tot_g:.1f} us per registration")
