"""NN-sweep tuning on the GPU: scalar vs packed FP32 and queries-per-lane Q, interleaved in one process
(cdna_hip_programming.md §5.4 rule 24).  Prints one JSON line per variant with the NN kernel's average
launch time and the FP32 roofline fraction on the benchmark workload.

    python tools/tune_sweep.py [--pairs 1024 --points 8192 --rounds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(args):
    sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))
    sys.path.insert(0, ROOT)
    import numpy as np
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
    ctx = icp4r.Context(0)
    batch = icp4r.Batch(src=src.data_ptr(), tgt=tgt.data_ptr(), src_off=off.data_ptr(), src_n=cnt.data_ptr(),
                        tgt_off=off.data_ptr(), tgt_n=cnt.data_ptr(), npairs=P, max_src_n=n, max_tgt_n=n)
    stream = torch.cuda.current_stream(dev).cuda_stream
    out = {}
    for mode in (icp4r.NN_BRUTE, icp4r.NN_BRUTE_PACKED):
        p = icp4r.default_params(max_iterations=args.iters, mse_threshold_absolute=-1.0, nn_mode=mode)
        ctx.align_batch_device(batch, p, res.data_ptr(), stream)  # warm-up
        torch.cuda.synchronize()
        ref = res.clone()
        ctx.reset_timers()
        for _ in range(args.rounds):
            ctx.align_batch_device(batch, p, res.data_ptr(), stream)
        torch.cuda.synchronize()
        nn_ms, k = ctx.kernel_time_ms()
        b_ms, _ = ctx.batch_time_ms()
        same = bool(torch.equal(ref, res))
        tf = P * n * n * 8 / (nn_ms * 1e-3) / 1e12
        out[mode] = res.clone()
        print(json.dumps({"Q": os.environ.get("ICP4R_NN_Q", "auto"), "mode": "packed" if mode == 2 else "scalar",
                          "nn_ms": nn_ms, "batch_ms": b_ms, "pairs_per_s": P / (b_ms * 1e-3), "tflops": tf,
                          "frac": tf / 157.3, "repeatable": same, "plan": icp4r.plan(P, n, n)}), flush=True)
    print(json.dumps({"Q": os.environ.get("ICP4R_NN_Q", "auto"),
                      "scalar_equals_packed": bool(torch.equal(out[1], out[2]))}), flush=True)
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--qs", default="8,4,2,1")
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        child(args)
        return
    for q in args.qs.split(","):
        env = dict(os.environ, ICP4R_NN_Q=q)
        cmd = [sys.executable, __file__, "--child", "--pairs", str(args.pairs), "--points", str(args.points),
               "--iters", str(args.iters), "--rounds", str(args.rounds)]
        r = subprocess.run(cmd, env=env, timeout=600)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
