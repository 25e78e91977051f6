"""Per-dispatch durations of one benchmark batch, grouped by ICP pass (diagnostic).

    rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --check 0
    python tools/experiments/pass_trace.py gpurun_out/trace

Prints, for the last batch in the trace, every icp4r kernel dispatch in order with its duration (us),
so the cost of each NN pass (test / order / search) and update is visible per iteration.
"""
from __future__ import annotations

import csv
import glob
import sys


def main():
    root = sys.argv[1]
    f = sorted(glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True))[-1]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if "icp4r::" in r["Kernel_Name"]]
    starts = [i for i, r in enumerate(ks) if "init_kernel" in r["Kernel_Name"]]
    last = ks[starts[-1]:]
    t0 = int(last[0]["Start_Timestamp"])
    tot = {}
    for r in last:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("icp4r::", "")
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[name] = tot.get(name, 0.0) + d
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:10.1f} {d:9.1f}  {name}")
    end = max(int(r["End_Timestamp"]) for r in last)
    print(f"batch span {(end - t0) / 1e3:.1f} us")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"  {k:40s} {v:9.1f} us")


if __name__ == "__main__":
    main()
