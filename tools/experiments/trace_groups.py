"""Per-queue timeline of the last grouped C3 batch in a rocprofv3 kernel trace (diagnostic).

    python tools/experiments/trace_groups.py gpurun_out/tv_<name> [--list]

Prints the batch span, per queue the summed duration of each kernel and the mean launch duration of
the search and the update, the share of the span in which 0 / 1 / 2+ queues ran a kernel, and, for
every pair of queues, how long a search on one overlapped an update on the other (the overlap the
pair groups exist for).  --list prints every launch (queue, start, duration, kernel).
"""
from __future__ import annotations

import csv
import glob
import sys
from collections import defaultdict


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "").replace("icp4r::", "").split("<")[0]


def main():
    d = sys.argv[1]
    f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[-1]
    rows = [r for r in csv.DictReader(open(f)) if "icp4r::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    inits = [i for i, r in enumerate(rows) if "init_kernel" in r["Kernel_Name"]]
    # batches: runs of init launches; the last one with inits on >= 2 queues
    groups = []
    i = 0
    while i < len(inits):
        j = i
        while j + 1 < len(inits) and inits[j + 1] - inits[j] <= 4:
            j += 1
        groups.append(inits[i:j + 1])
        i = j + 1
    multi = [g for g in groups if len({rows[k]["Queue_Id"] for k in g}) >= 2]
    if not multi:
        multi = groups
    g = multi[-1]
    nxt = [gg[0] for gg in groups if gg[0] > g[-1]]
    stop = nxt[0] if nxt else len(rows)
    last = rows[g[0]:stop]
    t0 = min(int(r["Start_Timestamp"]) for r in last)
    end = max(int(r["End_Timestamp"]) for r in last)
    span = end - t0
    ivs = defaultdict(list)
    for r in last:
        ivs[r["Queue_Id"]].append((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, short(r["Kernel_Name"])))
    print(f"{d}: batch span {span / 1e3:.1f} us, {len(last)} launches, queues {sorted(ivs)}")
    for q, iv in sorted(ivs.items()):
        per = defaultdict(list)
        for s, e, n in iv:
            per[n].append((e - s) / 1e3)
        tot = sum(e - s for s, e, _ in iv)
        print(f"  queue {q}: busy {tot / 1e3:.0f} us ({100 * tot / span:.0f} %)")
        for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            print(f"    {n:28s} {len(v):3d} x {sum(v) / len(v):7.1f} us = {sum(v):8.1f} us")
    cover = [0] * (span // 100 + 1)  # 0.1-us bins
    for iv in ivs.values():
        for s, e, _ in iv:
            for b in range(s // 100, e // 100):
                cover[b] += 1
    n0 = sum(1 for c in cover if c == 0)
    n1 = sum(1 for c in cover if c == 1)
    n2 = sum(1 for c in cover if c >= 2)
    print(f"  time with 0 / 1 / 2+ queues busy: {n0 / 10:.0f} / {n1 / 10:.0f} / {n2 / 10:.0f} us")
    qs = sorted(ivs)
    for a in qs:
        for b in qs:
            if a == b:
                continue
            ov = 0
            for s1, e1, n1_ in ivs[a]:
                if "nn_lds" not in n1_:
                    continue
                for s2, e2, n2_ in ivs[b]:
                    if "fold_update" in n2_:
                        ov += max(0, min(e1, e2) - max(s1, s2))
            print(f"  search on {a} beside update on {b}: {ov / 1e3:.0f} us")
    if "--list" in sys.argv:
        for r in last:
            print(f"{r['Queue_Id']:>4} {(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} "
                  f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:7.1f}  {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
