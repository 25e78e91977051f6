"""Timeline of one grouped batch from a rocprofv3 kernel trace (diagnostic): per queue, the kernels of
the last registration in order with start / duration, and how much of the batch span each queue was
busy and both were busy together.

    python tools/experiments/overlap.py gpurun_out/<trace dir>
"""
from __future__ import annotations

import csv
import glob
import sys
from collections import defaultdict


def main():
    f = sorted(glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True))[-1]
    rows = [r for r in csv.DictReader(open(f)) if "icp4r::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    inits = [i for i, r in enumerate(rows) if "init_kernel" in r["Kernel_Name"]]
    # the last grouped batch: its group inits run on different queues; it ends before the next init
    k = max(j for j in range(1, len(inits)) if rows[inits[j]]["Queue_Id"] != rows[inits[j - 1]]["Queue_Id"])
    stop = inits[k + 1] if k + 1 < len(inits) else len(rows)
    last = rows[inits[k - 1]:stop]
    t0 = int(last[0]["Start_Timestamp"])
    end = max(int(r["End_Timestamp"]) for r in last)
    busy = defaultdict(list)
    for r in last:
        busy[r["Queue_Id"]].append((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Kernel_Name"]))
    span = end - t0
    print(f"batch span {span / 1e3:.1f} us, queues {sorted(busy)}")
    cover = [0] * (span // 1000 + 1)
    for q, iv in busy.items():
        tot = sum(e - s for s, e, _ in iv)
        per = defaultdict(float)
        for s, e, n in iv:
            per[n.split("(")[0].replace("void ", "").replace("icp4r::", "")] += (e - s) / 1e3
        print(f"queue {q}: busy {tot / 1e3:.1f} us ({100 * tot / span:.0f} %)  " +
              "  ".join(f"{k} {v:.0f}" for k, v in sorted(per.items(), key=lambda kv: -kv[1])))
        for s, e, _ in iv:
            for us in range(s // 1000, e // 1000 + 1):
                if us < len(cover):
                    cover[us] += 1
    both = sum(1 for c in cover if c >= 2)
    none = sum(1 for c in cover if c == 0)
    print(f"us with >= 2 queues busy: {both} ({100 * both / len(cover):.0f} %), idle: {none}")


if __name__ == "__main__":
    main()
