"""Timeline of the last single-pair registration in a rocprofv3 kernel trace (diagnostic):
    python tools/experiments/trace_pair.py gpurun_out/tc_<name>
Per launch: start (us from the registration's first kernel), duration, gap before it, kernel; then
per-kernel totals and the summed gaps (device idle between launches)."""
import csv
import glob
import sys
from collections import defaultdict


def short(n):
    return n.split("(")[0].replace("void ", "").replace("icp4r::", "").split("<")[0]


f = sorted(glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True))[-1]
rows = [r for r in csv.DictReader(open(f)) if "icp4r::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
inits = [i for i, r in enumerate(rows) if "init_kernel" in r["Kernel_Name"]]
last = rows[inits[-2]:inits[-1]] if len(inits) > 1 else rows[inits[-1]:]
t0 = int(last[0]["Start_Timestamp"])
prev_end = t0
tot = defaultdict(float)
gaps = 0.0
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = max(0, s - prev_end)
    gaps += g
    tot[short(r["Kernel_Name"])] += (e - s) / 1e3
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap {g / 1e3:5.1f}  {short(r['Kernel_Name'])}")
    prev_end = max(prev_end, e)
print(f"span {(prev_end - t0) / 1e3:.1f} us, gaps {gaps / 1e3:.1f} us")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {k:28s} {v:8.1f} us")
