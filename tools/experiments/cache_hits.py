"""Per-pass hit rate of the cached-neighbour test on the benchmark workload (diagnostic).

    python tools/experiments/cache_hits.py [--pairs 256] [--iters 20]

Runs the batch with max_iterations = 1..iters (fitness pass off) and differences the device hit
counter, so row k is the share of queries whose NN pass k resolved without a search; the last row
is the fitness pass.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import icp4r
    from icp4r import synth

    P, n = a.pairs, a.points
    pairs = [synth.make_pair(1000 + k, n) for k in range(P)]
    src = np.concatenate([p.src_xyzi() for p in pairs])
    tgt = np.concatenate([p.tgt_xyzi() for p in pairs])
    cnt = np.full(P, n, np.int32)
    off = np.arange(P, dtype=np.int64) * n
    ctx = icp4r.Context(0, plan=icp4r.env_plan())

    prev_h = prev_e = 0
    for k in range(1, a.iters + 2):
        fit = k == a.iters + 1
        p = icp4r.default_params(max_iterations=min(k, a.iters), mse_threshold_absolute=-1.0,
                                 transformation_epsilon=-1.0, compute_fitness=1 if fit else 0)
        ctx.reset_timers()
        ctx.align_batch_host(src, off, cnt, tgt, off, cnt, params=p)
        h = ctx.nn_cache_hits()
        e, t = ctx.nn_counters()
        ms, launches = ctx.kernel_time_ms()
        dh, de = h - prev_h, e - prev_e
        print(f"pass {k:2d}{' (fitness)' if fit else '          '}: hits {dh / (P * n):6.3f}  "
              f"evals/query {de / (P * n):8.1f}  avg NN pass {ms:7.3f} ms over {launches}", end="")
        print()
        prev_h, prev_e = h, e


if __name__ == "__main__":
    main()
