"""Per-pass event counts and per-run clocks of the persistent batched search (diagnostic;
ICP4R_PHASE_TICKS=1, ICP4R_GROUPS=1).

    python tools/nn_events.py [--pairs 1024] [--iters 20]

For pass k (a run of k iterations minus a run of k-1), summed over every wave of nn_lds_kernel:
runs (one wave's ≤64-query slice of an item), queries, superblock visits (candidates of the run's
coarse test), visits that passed the per-query test, candidate blocks, block pushes with at least
one lane, drains, drained work items; and the wave clocks (s_memtime) of run setup, traversal and
result writes.  Lines are JSON, one per pass, then the total.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))

NAMES = ["runs", "queries", "sb_visits", "sb_passed", "blk_cands", "pushes", "drains", "items",
         "ck_setup", "ck_traverse", "ck_write"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    os.environ["ICP4R_PHASE_TICKS"] = "1"
    os.environ["ICP4R_GROUPS"] = "1"
    import icp4r
    from icp4r import synth

    P, n = a.pairs, a.points
    pairs = [synth.make_pair(1000 + k, n) for k in range(P)]
    src = np.concatenate([p.src_xyzi() for p in pairs])
    tgt = np.concatenate([p.tgt_xyzi() for p in pairs])
    cnt = np.full(P, n, np.int32)
    off = np.arange(P, dtype=np.int64) * n
    ctx = icp4r.Context(0)
    lib = icp4r.load()
    lib.icp4r__debug_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]

    def ticks():
        buf = (C.c_uint64 * 32)()
        return np.array(list(buf), np.float64) if lib.icp4r__debug_ticks(ctx._h, buf, 32) == 0 else None

    prev = np.zeros(11)
    prev_it = np.zeros(4)
    total = np.zeros(11)
    tot_ms = 0.0
    for k in range(1, a.iters + 2):  # the last one: the iterations + the fitness pass
        fit = k == a.iters + 1
        p = icp4r.default_params(max_iterations=min(k, a.iters), mse_threshold_absolute=-1.0,
                                 transformation_epsilon=-1.0, compute_fitness=1 if fit else 0)
        t0 = ticks()
        ctx.reset_timers()
        ctx.align_batch_host(src, off, cnt, tgt, off, cnt, params=p)
        t1 = ticks()
        if t0 is None:
            t0 = np.zeros(32)
        d = (t1 - t0)[16:27]
        last = d - prev
        prev = d
        it = (t1 - t0)[8:12]  # per-item wall (100 MHz): compaction, staging, search (all waves), items
        it_last = it - prev_it
        prev_it = it
        total += last
        ms, _ = ctx.kernel_time_ms()
        r = {"pass": "fitness" if fit else k}
        r.update({nm: int(v) for nm, v in zip(NAMES, last)})
        runs = max(last[0], 1)
        r["per_run"] = {"queries": last[1] / runs, "sb_visits": last[2] / runs, "blk_cands": last[4] / runs,
                        "pushes": last[5] / runs, "drains": last[6] / runs,
                        "cyc_setup": last[8] / runs, "cyc_traverse": last[9] / runs, "cyc_write": last[10] / runs}
        r["cyc_per_sb_visit"] = last[9] / max(last[2], 1)
        ni = max(it_last[3], 1)
        r["items"] = {"n": int(it_last[3]), "compact_us": it_last[0] / ni / 100, "stage_us": it_last[1] / ni / 100,
                      "search_wall_us": it_last[2] / ni / 100,
                      # wave clocks inside runs / (search wall x 16 waves): the waves' busy share of it
                      "run_cyc_per_item": (last[8] + last[9] + last[10]) / ni}
        r["registration_kernel_ms"] = ms
        print(json.dumps(r), flush=True)
    runs = max(total[0], 1)
    print(json.dumps({"pass": "total", **{nm: int(v) for nm, v in zip(NAMES, total)},
                      "per_run": {nm: total[i] / runs for i, nm in enumerate(NAMES) if i}}), flush=True)


if __name__ == "__main__":
    main()
