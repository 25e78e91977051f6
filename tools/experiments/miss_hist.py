"""Per-pass distribution of cached-neighbour misses over the pairs of the benchmark batch
(diagnostic; ICP4R_PHASE_TICKS=1 makes nn_order_kernel record each pair's work of the last pass).

    python tools/experiments/miss_hist.py [--pairs 1024] [--iters 20]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    os.environ["ICP4R_PHASE_TICKS"] = "1"
    os.environ.setdefault("ICP4R_FUSE_ORDER", "0")  # (nn_order_kernel records the per-pair work)
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
    for k in range(1, a.iters + 1):
        p = icp4r.default_params(max_iterations=k, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0,
                                 compute_fitness=0)
        ctx.align_batch_host(src, off, cnt, tgt, off, cnt, params=p)
        buf = (C.c_uint64 * (32 + P))()
        lib.icp4r__debug_ticks(ctx._h, buf, 32 + P)
        m = np.array(list(buf), np.int64)[32:32 + P]
        s = np.sort(m)[::-1]
        print(json.dumps({"pass": k, "pairs": int((m > 0).sum()), "misses": int(m.sum()),
                          "top": s[:8].tolist(), "p50": int(np.median(m[m > 0])) if (m > 0).any() else 0,
                          "over1024": int((m > 1024).sum()), "work_over1024": int(m[m > 1024].sum()),
                          "le": {str(t): [int(((m > 0) & (m <= t)).sum()), int(m[(m > 0) & (m <= t)].sum())]
                                 for t in (16, 64, 128, 256, 512)}}), flush=True)


if __name__ == "__main__":
    main()
