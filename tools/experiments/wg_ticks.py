"""Per-workgroup phase timeline of fold_update_kernel in the C3 batch (diagnostic build).

    tools/experiments/ab_build.sh wgticks "-DICP4R_WG_TICKS=1"
    ICP4R_LIBRARY=_var/ab/wgticks/libicp4r.so python tools/experiments/wg_ticks.py [--pairs 1024]

Every pair's workgroup stamps s_memrealtime (100 MHz) at its start, after pass A, pass B, the solve
and the fused test, in its 10th update (single pair group).  Prints the launch span, the start
spread (do all workgroups start at once?) and the phase durations' percentiles in µs.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

os.environ["ICP4R_PHASE_TICKS"] = "1"
os.environ.setdefault("ICP4R_GROUPS", "1")  # (group 0's pairs are the ones stamped)
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
    G = max(1, int(os.environ["ICP4R_GROUPS"]))
    Pg = P // G  # pair group 0 (the stamped one)
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
    k = 32 + 12 * Pg + 64
    buf = (C.c_uint64 * k)()
    lib = icp4r.load()
    lib.icp4r__debug_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]
    if lib.icp4r__debug_ticks(ctx._h, buf, k):
        raise RuntimeError(lib.icp4r_last_error())
    raw = np.array(buf[32 + 4 * Pg:32 + 12 * Pg], dtype=np.uint64).reshape(Pg, 8)
    fine = np.array(buf[32 + 12 * Pg:], dtype=np.uint64).astype(np.int64)
    hw = raw[:, 5] if os.environ.get("ICP4R_RES_UPDATE", "0") == "0" else np.zeros(Pg, np.uint64)
    if hw.any():  # fold-wave placement: per CU, how many fold waves share each SIMD
        hid = (hw & 0xffffffff).astype(np.int64)
        xcc = (hw >> np.uint64(32)).astype(np.int64) & 0xf
        simd = (hid >> 4) & 3
        cu = (xcc << 16) | (((hid >> 13) & 7) << 8) | (((hid >> 12) & 1) << 4) | ((hid >> 8) & 0xf)
        per = {}
        for c, s_ in zip(cu.tolist(), simd.tolist()):
            per.setdefault(c, [0, 0, 0, 0])[s_] += 1
        worst = [max(v) for v in per.values()]
        print(json.dumps({"cus": len(per), "fold_waves_max_per_simd_hist": {str(k): worst.count(k) for k in sorted(set(worst))},
                          "example": list(per.items())[:4]}))
    t = raw[:, :5].astype(np.int64).astype(np.float64) * 0.01  # µs
    ok = (t > 0).all(axis=1)
    t = t[ok]
    t0 = t[:, 0].min()
    out = {"groups": G, "env": {k: v for k, v in os.environ.items() if k.startswith("ICP4R_")},
           "pairs_stamped": int(ok.sum()), "span_us": float(t[:, 4].max() - t0),
           "start_spread_us": float(t[:, 0].max() - t0)}
    pct = lambda v: {f"p{q}": round(float(np.percentile(v, q)), 1) for q in (0, 10, 50, 90, 100)}
    out["start"] = pct(t[:, 0] - t0)
    for j, name in enumerate(["passA", "passB", "solve", "tail"]):
        out[name] = pct(t[:, j + 1] - t[:, j])
    t6 = raw[ok, 6].astype(np.int64).astype(np.float64) * 0.01
    if (t6 > 0).all():  # the tail split at the test's end: the test, then the misses' rank placement
        out["tail_test"] = pct(t6 - t[:, 3])
        out["tail_place"] = pct(t[:, 4] - t6)
    t5 = raw[ok, 5].astype(np.int64).astype(np.float64) * 0.01
    if not hw.any() and (t5 > 0).all():  # fold_update_res_kernel: pass B split after its prologue
        out["passB_prologue"] = pct(t5 - t[:, 1])
        out["passB_chunks"] = pct(t[:, 2] - t5)
    t7 = raw[ok, 7].astype(np.int64).astype(np.float64) * 0.01
    if (t7 > 0).all():  # fold_update_res_kernel: pass A split at the end of the pair's loads
        out["load"] = pct(t7 - t[:, 0])
        out["passA_folds"] = pct(t[:, 1] - t7)
    out["total"] = pct(t[:, 4] - t[:, 0])
    if fine[0] > 0:  # fold_update_res_kernel, pair 0: pass A per column, pass B per chunk (fill end, fold end)
        r0 = int(raw[0, 7]) if raw[0, 7] else int(raw[0, 0])
        colA = [f for f in fine[:32] if f > 0]
        out["pair0_passA_col_us"] = [round((b - a) * 0.01, 2) for a, b in zip([r0] + colA[:-1], colA)]
        pb = [f for f in fine[32:64]]
        t5 = int(raw[0, 5])
        seq = [t5] + [f for f in pb if f > 0]
        out["pair0_passB_fill_fold_us"] = [round((b - a) * 0.01, 2) for a, b in zip(seq[:-1], seq[1:])]
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
