"""Phase timing of fold_update_kernel on the GPU (s_memrealtime, 100 MHz = 10 ns ticks), pair 0.

    ICP4R_PHASE_TICKS is set by this script; prints pass A / pass B / solve / transform in µs for a
    single pair of each size and for pair 0 of a 1024-pair batch (the last iteration's update).
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

os.environ["ICP4R_PHASE_TICKS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))

import numpy as np  # noqa: E402

import icp4r  # noqa: E402
from icp4r import synth  # noqa: E402


def ticks(ctx) -> list[float]:
    buf = (C.c_uint64 * 32)()
    lib = icp4r.load()
    lib.icp4r__debug_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]
    rc = lib.icp4r__debug_ticks(ctx._h, buf, 32)
    if rc:
        raise RuntimeError(lib.icp4r_last_error())
    t = [int(v) for v in buf]
    names = ["passA", "passB", "solve", "transform"]
    out = {names[k]: (t[k + 1] - t[k]) * 0.01 for k in range(4)}  # µs
    if t[12] and t[15] and t[12] >= t[1]:  # the wide update's pass B (PAR): setup, first fill, folds, tail
        out["passB_parts"] = {"setup": (t[12] - t[1]) * 0.01, "fill0": (t[13] - t[12]) * 0.01,
                              "chunks": (t[14] - t[13]) * 0.01, "end": (t[15] - t[14]) * 0.01}
        if t[31] and t[30] and t[27]:  # finer: entry, after the first barrier, the chunk folds
            out["passB_fine"] = {"entry": (t[31] - t[1]) * 0.01, "to_barrier": (t[30] - t[31]) * 0.01,
                                 "to_fill": (t[12] - t[30]) * 0.01, "fold0": (t[27] - t[13]) * 0.01,
                                 "wait1": (t[28] - t[27]) * 0.01 if t[28] else None,
                                 "fold1": (t[29] - t[28]) * 0.01 if t[29] else None}
    if t[5] and t[6] and t[5] < 100000:  # ICP4R_SOLVE_PROBE builds: the rotation twice, back to back
        out["rotation_x2"] = [t[5] * 0.01, t[6] * 0.01]
    return out


def main():
    ctx = icp4r.Context(0, plan=icp4r.env_plan())
    p = icp4r.default_params(max_iterations=5, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0,
                             eigen_l1_bytes=int(os.environ.get("EIGEN_L1", "0")))
    for n in (2048, 8192):
        pr = synth.make_pair(7, n)
        ctx.align(pr.src_xyzi(), pr.tgt_xyzi(), p)
        print(json.dumps({"case": f"single {n}", **ticks(ctx)}), flush=True)
    for rep in range(3):  # C1: pair 0 at 2048, PCL defaults (the MSE criterion live)
        pr = synth.make_pair(0, 2048)
        ctx.align(pr.src_xyzi(), pr.tgt_xyzi(), icp4r.default_params())
        print(json.dumps({"case": f"C1 pcl defaults rep {rep}", **ticks(ctx)}), flush=True)
    P, n = 1024, 8192
    src = np.stack([synth.make_pair(k, n).src_xyzi() for k in range(P)]).reshape(-1, 4)
    tgt = np.stack([synth.make_pair(k, n).tgt_xyzi() for k in range(P)]).reshape(-1, 4)
    off = np.arange(P, dtype=np.int64) * n
    cnt = np.full(P, n, np.int32)
    ctx.align_batch_host(src, off, cnt, tgt, off, cnt, params=p)
    print(json.dumps({"case": f"batch {P}x{n} pair 0", **ticks(ctx)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
