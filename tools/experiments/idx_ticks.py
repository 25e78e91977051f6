"""Per-cloud timeline of index_kernel in the C3 batch (diagnostic build).

    tools/experiments/ab_build.sh wgticks "-DICP4R_WG_TICKS=1"
    ICP4R_LIBRARY=_var/ab/wgticks/libicp4r.so python tools/experiments/idx_ticks.py [--pairs 1024]

Every cloud's kd build stamps s_memrealtime (100 MHz) at its start and end, with the CU it ran on.
Prints the launch span, per-cloud build times (targets / sources) and how many builds each CU ran.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

os.environ["ICP4R_PHASE_TICKS"] = "1"
os.environ["ICP4R_GROUPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--points", type=int, default=8192)
    args = ap.parse_args()
    import torch

    import icp4r
    from bench import make_shard

    P, n = args.pairs, args.points
    src_h, tgt_h = make_shard(0, P, n)
    dev = torch.device("cuda", 0)
    src = torch.from_numpy(src_h.reshape(-1, 4)).to(dev)
    tgt = torch.from_numpy(tgt_h.reshape(-1, 4)).to(dev)
    off = torch.arange(P, dtype=torch.int64, device=dev) * n
    cnt = torch.full((P,), n, dtype=torch.int32, device=dev)
    results = torch.zeros((P, 96), dtype=torch.uint8, device=dev)
    ctx = icp4r.Context(0, plan=icp4r.env_plan())
    params = icp4r.default_params(max_iterations=20, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
    batch = icp4r.Batch(src=src.data_ptr(), tgt=tgt.data_ptr(), src_off=off.data_ptr(), src_n=cnt.data_ptr(),
                        tgt_off=off.data_ptr(), tgt_n=cnt.data_ptr(), guess=None, aligned=None, npairs=P,
                        max_src_n=n, max_tgt_n=n)
    for _ in range(2):
        ctx.align_batch_device(batch, params, results.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    k = 32 + 20 * P
    buf = (C.c_uint64 * k)()
    lib = icp4r.load()
    lib.icp4r__debug_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]
    if lib.icp4r__debug_ticks(ctx._h, buf, k):
        raise RuntimeError(lib.icp4r_last_error())
    raw = np.array(buf[32 + 12 * P:], dtype=np.uint64).reshape(P, 2, 4)  # [pair][tgt, src][start, end, hw, -]
    have = raw[:, :, 0] > 0  # (clouds built elsewhere, e.g. sources ordered by src_order_kernel, have no stamps)
    t0 = raw[:, :, 0][have].astype(np.int64).min()
    st = ((raw[:, :, 0].astype(np.int64) - t0) * 0.01)[have]
    du = (raw[:, :, 1].astype(np.int64) - raw[:, :, 0].astype(np.int64)) * 0.01
    hw = raw[:, :, 2][have]
    hid = (hw & np.uint64(0xffffffff)).astype(np.int64)
    xcc = (hw >> np.uint64(32)).astype(np.int64) & 0xf
    cu = (xcc << 16) | (((hid >> 13) & 7) << 8) | (((hid >> 12) & 1) << 4) | ((hid >> 8) & 0xf)
    pct = lambda v: {f"p{q}": round(float(np.percentile(v, q)), 1) for q in (0, 10, 50, 90, 100)}
    per_cu = {}
    for c in cu.tolist():
        per_cu[c] = per_cu.get(c, 0) + 1
    cnts = list(per_cu.values())
    out = {"span_us": round(float((raw[:, :, 1][have].astype(np.int64).max() - t0) * 0.01), 1),
           "target_build_us": pct(du[:, 0][have[:, 0]]),
           "source_build_us": pct(du[:, 1][have[:, 1]]) if have[:, 1].any() else None,
           "start_us": pct(st), "cus": len(per_cu),
           "builds_per_cu": {str(v): cnts.count(v) for v in sorted(set(cnts))}}
    ph = (raw[:, 1, 3].astype(np.int64) - raw[:, 1, 0].astype(np.int64)) * 0.01  # src_order: descent + histogram
    if have[:, 1].any() and (raw[:, 1, 3] > 0).any():
        out["src_order_phase1_us"] = pct(ph[raw[:, 1, 3] > 0])
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
