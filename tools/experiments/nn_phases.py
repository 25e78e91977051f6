"""Per-pass phase times of the persistent batched search (diagnostic; ICP4R_PHASE_TICKS=1).

    python tools/experiments/nn_phases.py [--pairs 1024] [--iters 20]

For pass k (a run of k iterations minus a run of k-1): pairs searched, and per searched pair the
wall time of compaction, target staging and the search itself (workgroup thread 0's clock).
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    os.environ["ICP4R_PHASE_TICKS"] = "1"
    import icp4r
    from icp4r import synth

    P, n = a.pairs, a.points
    pairs = [synth.make_pair(1000 + k, n) for k in range(P)]
    src = np.concatenate([p.src_xyzi() for p in pairs])
    tgt = np.concatenate([p.tgt_xyzi() for p in pairs])
    cnt = np.full(P, n, np.int32)
    off = np.arange(P, dtype=np.int64) * n
    ctx = icp4r.Context(0, plan=icp4r.env_plan())
    lib = icp4r.load()
    lib.icp4r__debug_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]

    def ticks():
        buf = (C.c_uint64 * 32)()
        return np.array(list(buf), np.float64) if lib.icp4r__debug_ticks(ctx._h, buf, 32) == 0 else None

    prev = None
    for k in range(1, a.iters + 1):
        p = icp4r.default_params(max_iterations=k, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0,
                                 compute_fitness=0)
        t0 = ticks()
        ctx.reset_timers()
        ctx.align_batch_host(src, off, cnt, tgt, off, cnt, params=p)
        t1 = ticks()
        ms, _ = ctx.kernel_time_ms()
        if t0 is None:
            t0 = np.zeros(32)
        d = t1 - t0
        last = d - prev if prev is not None else d
        prev = d
        pr = max(last[11], 1)
        runs = max(last[27], 1)
        print(f"pass {k:2d}: items {int(last[11]):5d}  per item: compact {last[8] / pr * 0.01:6.1f} us  "
              f"stage {last[9] / pr * 0.01:6.1f} us  search {last[10] / pr * 0.01:7.1f} us | runs {int(last[27]):6d} "
              f"per run: setup {last[24] / runs * 0.01:5.1f} us  traverse {last[25] / runs * 0.01:6.1f} us  "
              f"write {last[26] / runs * 0.01:5.1f} us (drains {last[28] / runs * 0.01:5.1f} us)   (avg search launch {ms:.3f} ms)")


if __name__ == "__main__":
    main()
