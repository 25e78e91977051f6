"""Phase timing of index_kernel's kd build for pair 0's target (diagnostic; ICP4R_PHASE_TICKS=1).

    python tools/experiments/index_ticks.py [--pairs 1024]

s_memrealtime (100 MHz) at: start, after the counting sorts, after the levels, after the scatter and
boxes — for a single pair and for pair 0 of a batch (where 2 clouds per CU-slot queue up).
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
    a = ap.parse_args()
    os.environ["ICP4R_PHASE_TICKS"] = "1"
    import icp4r
    from icp4r import synth

    lib = icp4r.load()
    lib.icp4r__debug_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]
    for P in (1, a.pairs):
        pairs = [synth.make_pair(1000 + k, a.points) for k in range(min(P, 64))]
        pairs = [pairs[k % len(pairs)] for k in range(P)]
        src = np.concatenate([p.src_xyzi() for p in pairs])
        tgt = np.concatenate([p.tgt_xyzi() for p in pairs])
        cnt = np.full(P, a.points, np.int32)
        off = np.arange(P, dtype=np.int64) * a.points
        ctx = icp4r.Context(0, plan=icp4r.env_plan())
        p = icp4r.default_params(max_iterations=1, compute_fitness=0)
        for _ in range(2):
            ctx.align_batch_host(src, off, cnt, tgt, off, cnt, params=p)
        buf = (C.c_uint64 * 16)()
        lib.icp4r__debug_ticks(ctx._h, buf, 16)
        t = np.array(list(buf), np.float64)[12:16]
        d = np.diff(t) * 0.01
        print(json.dumps({"pairs": P, "sort_us": d[0], "levels_us": d[1], "scatter_boxes_us": d[2]}), flush=True)


if __name__ == "__main__":
    main()
