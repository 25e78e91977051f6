"""Per-pass event counts and per-run clocks of the persistent batched search (diagnostic;
ICP4R_PHASE_TICKS=1, ICP4R_GROUPS=1).

    python tools/experiments/nn_events.py [--pairs 1024] [--iters 20]

For every NN pass of one registration (each pass adds into its own tick slots), summed over every
wave of nn_lds_kernel:
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

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    ctx = icp4r.Context(0, plan=icp4r.env_plan())
    ctx.set_kernel_timing(True)
    lib = icp4r.load()
    lib.icp4r__debug_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]

    def ticks(k):
        buf = (C.c_uint64 * k)()
        return np.array(list(buf), np.float64) if lib.icp4r__debug_ticks(ctx._h, buf, k) == 0 else None

    # one registration: every NN pass adds into its own slots (pass_tick_base(P) + pass * 16)
    base, slots, npass = 32 + 20 * P, 16, a.iters + 1
    t0 = ticks(base + slots * npass)
    ctx.reset_timers()
    p = icp4r.default_params(max_iterations=a.iters, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0,
                             compute_fitness=1)
    ctx.align_batch_host(src, off, cnt, tgt, off, cnt, params=p)
    t1 = ticks(base + slots * npass)
    if t0 is None:
        t0 = np.zeros_like(t1)
    ms, _ = ctx.kernel_time_ms()
    total = np.zeros(11)
    for k in range(npass):
        d = (t1 - t0)[base + k * slots: base + (k + 1) * slots]
        last, it = d[:11], d[11:15]  # per-item walls (100 MHz): compaction, staging, search, items
        total += last
        r = {"pass": "fitness" if k == a.iters else k + 1}
        r.update({nm: int(v) for nm, v in zip(NAMES, last)})
        runs = max(last[0], 1)
        r["per_run"] = {"queries": last[1] / runs, "sb_visits": last[2] / runs, "blk_cands": last[4] / runs,
                        "pushes": last[5] / runs, "drains": last[6] / runs,
                        "cyc_setup": last[8] / runs, "cyc_traverse": last[9] / runs, "cyc_write": last[10] / runs}
        r["cyc_per_sb_visit"] = last[9] / max(last[2], 1)
        ni = max(it[3], 1)
        r["items"] = {"n": int(it[3]), "compact_us": it[0] / ni / 100, "stage_us": it[1] / ni / 100,
                      "search_wall_us": it[2] / ni / 100, "run_cyc_per_item": (last[8] + last[9] + last[10]) / ni}
        print(json.dumps(r), flush=True)
    runs = max(total[0], 1)
    print(json.dumps({"pass": "total", "registration_kernel_ms": ms, **{nm: int(v) for nm, v in zip(NAMES, total)},
                      "per_run": {nm: total[i] / runs for i, nm in enumerate(NAMES) if i}}), flush=True)


if __name__ == "__main__":
    main()
