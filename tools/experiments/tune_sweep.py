"""NN tuning on the GPU: search variants interleaved in ONE process (cdna_hip_programming.md §5.4
rule 24).  The library reads ICP4R_NN_Q / ICP4R_LEAF at plan time, so variants switch in-process.
Prints one JSON line per variant and round: NN kernel average launch time, whole-batch device time,
distance evaluations per launch, the FP32 roofline fraction, and whether the results are
bit-identical to the brute-force reference run.

    python tools/experiments/tune_sweep.py [--pairs 1024 --points 8192 --rounds 2 --variants pruned:2:16,brute:4:0]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_VARIANTS = "brute:4:0,pruned:1:16,pruned:2:16,pruned:4:16,pruned:1:32,pruned:2:32,pruned:4:32"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variants", default=DEFAULT_VARIANTS, help="mode:Q:leaf,...  (mode = brute|packed|pruned)")
    args = ap.parse_args()
    sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))
    sys.path.insert(0, ROOT)
    import torch

    import icp4r
    from bench import make_shard

    n, P = args.points, args.pairs
    src_h, tgt_h = make_shard(0, P, n)
    dev = torch.device("cuda", 0)
    src = torch.from_numpy(src_h.reshape(-1, 4)).to(dev)
    tgt = torch.from_numpy(tgt_h.reshape(-1, 4)).to(dev)
    off = torch.arange(P, dtype=torch.int64, device=dev) * n
    cnt = torch.full((P,), n, dtype=torch.int32, device=dev)
    res = torch.zeros((P, 96), dtype=torch.uint8, device=dev)
    ctx = icp4r.Context(0, plan=icp4r.env_plan())
    batch = icp4r.Batch(src=src.data_ptr(), tgt=tgt.data_ptr(), src_off=off.data_ptr(), src_n=cnt.data_ptr(),
                        tgt_off=off.data_ptr(), tgt_n=cnt.data_ptr(), npairs=P, max_src_n=n, max_tgt_n=n)
    stream = torch.cuda.current_stream(dev).cuda_stream
    modes = {"brute": icp4r.NN_BRUTE, "packed": icp4r.NN_BRUTE_PACKED, "pruned": icp4r.NN_PRUNED}
    variants = [v.split(":") for v in args.variants.split(",")]
    ref = None
    for rnd in range(args.rounds):
        for mode, q, leaf in variants:
            os.environ["ICP4R_NN_Q"] = q
            os.environ["ICP4R_LEAF"] = leaf
            p = icp4r.default_params(max_iterations=args.iters, mse_threshold_absolute=-1.0,
                                     transformation_epsilon=-1.0, nn_mode=modes[mode])
            ctx.align_batch_device(batch, p, res.data_ptr(), stream)  # warm-up
            torch.cuda.synchronize()
            ctx.reset_timers()
            ctx.align_batch_device(batch, p, res.data_ptr(), stream)
            torch.cuda.synchronize()
            nn_ms, k = ctx.kernel_time_ms()
            b_ms, _ = ctx.batch_time_ms()
            ev = ctx.nn_counters()[0] / max(k, 1)
            if ref is None:
                ref = res.clone()
            tf = ev * 8 / (nn_ms * 1e-3) / 1e12
            print(json.dumps({"round": rnd, "mode": mode, "Q": int(q), "leaf": int(leaf), "nn_ms": nn_ms,
                              "batch_ms": b_ms, "pairs_per_s": P / (b_ms * 1e-3), "evals_per_launch": ev,
                              "evaluated_fraction": ev / (P * n * n), "tflops": tf, "frac": tf / 157.3,
                              "identical_to_first": bool(torch.equal(ref, res)),
                              "plan": icp4r.plan(P, n, n, modes[mode])}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
