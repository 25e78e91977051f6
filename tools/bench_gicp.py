"""Generalized ICP throughput / latency with per-stage device times, next to
the oracle on one host core.

    python tools/bench_gicp.py [--case map|scan|batch] [--steps 3]

Cases:
  map    the reference node's call (radar_odometry.cpp:399-405): one 8k-point scan, associated to the map
         frame with a slightly wrong odometry prediction, against a 64k-point submap
         (synth.make_map_pair), k = 5 (setCorrespondenceRandomness(5))
  scan   one 8k/8k scan pair, fast_gicp defaults (k = 20)
  batch  --pairs independent 8k/8k pairs, k = 5, one device batch (throughput mode)

Stage times are HIP events on the launch stream: covariances (ICP4R_STAGE_GICP_COV), NN passes
(ICP4R_STAGE_NN), Gauss-Newton / LM iterations (ICP4R_STAGE_UPDATE), whole registration
(ICP4R_STAGE_BATCH).  The CPU line is oracle/gicp_oracle.c (single thread, brute-force k-NN) on a
reduced pair (--cpu-points) and scales as stated in its `sample`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "icp-4dradar_amd"), os.path.join(ROOT, "oracle")]


def _pad4(x):
    out = np.zeros((len(x), 4), np.float32)
    out[:, :3] = x[:, :3]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="map", choices=["map", "scan", "batch"])
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--cpu-points", type=int, default=2048)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--k", type=int, default=0, help="override k_correspondences")
    ap.add_argument("--reg", type=int, default=-1, help="override the regularization (icp4r_gicp_regularization)")
    ap.add_argument("--max-iterations", type=int, default=-1)
    ap.add_argument("--no-stages", action="store_true",
                    help="no per-stage events (each costs device time between kernels): the call's time alone")
    a = ap.parse_args()
    import torch

    import icp4r
    from icp4r import gicp, synth

    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    if a.case == "map":
        # as the node calls it: the scan already associated to the map frame with the odometry's
        # prediction (pointAssociateToMap, radar_odometry.cpp:382-385) — here the true pose composed
        # with a 0.3 m / 1 degree prediction error
        pr = synth.make_map_pair(0, n_src=a.points)
        yaw = np.deg2rad(1.0)
        err = np.array([[np.cos(yaw), -np.sin(yaw), 0.0, 0.3], [np.sin(yaw), np.cos(yaw), 0.0, -0.2],
                        [0.0, 0.0, 1.0, 0.05], [0.0, 0.0, 0.0, 1.0]])
        Tp = pr.T_gt @ err
        src_map = pr.src.copy()
        src_map[:, :3] = (pr.src[:, :3].astype(np.float64) @ Tp[:3, :3].T + Tp[:3, 3]).astype(np.float32)
        pairs = [(src_map, pr.tgt)]
        k = 5
    elif a.case == "scan":
        pr = synth.make_pair(0, a.points)
        pairs = [(pr.src, pr.tgt)]
        k = 20
    else:
        pairs = []
        for i in range(a.pairs):
            pr = synth.make_pair(i % 64, a.points)
            pairs.append((pr.src, pr.tgt))
        k = 5
    src = np.concatenate([_pad4(s) for s, _ in pairs])
    tgt = np.concatenate([_pad4(t) for _, t in pairs])
    sn = np.array([len(s) for s, _ in pairs], np.int32)
    tn = np.array([len(t) for _, t in pairs], np.int32)
    so = np.concatenate([[0], np.cumsum(sn)[:-1]]).astype(np.int64)
    to = np.concatenate([[0], np.cumsum(tn)[:-1]]).astype(np.int64)
    ts = {n: torch.from_numpy(v).to(dev) for n, v in dict(src=src, tgt=tgt, sn=sn, tn=tn, so=so, to=to).items()}
    res = torch.zeros(len(pairs) * icp4r.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    b = icp4r.Batch()
    b.src, b.tgt = ts["src"].data_ptr(), ts["tgt"].data_ptr()
    b.src_off, b.src_n, b.tgt_off, b.tgt_n = ts["so"].data_ptr(), ts["sn"].data_ptr(), ts["to"].data_ptr(), ts["tn"].data_ptr()
    b.npairs, b.max_src_n, b.max_tgt_n = len(pairs), int(sn.max()), int(tn.max())
    ctx = icp4r.Context(0, plan=icp4r.env_plan())
    ctx.set_kernel_timing(not a.no_stages)  # (per-stage times, unless --no-stages)
    k = a.k or k
    p = gicp.default_params(k_correspondences=k)
    if a.reg >= 0:
        p.regularization = a.reg
    if a.max_iterations >= 0:
        p.max_iterations = a.max_iterations
    side = torch.cuda.Stream(dev)

    def step():
        gicp.align_batch_device(b, p, res.data_ptr(), stream=side.cuda_stream, ctx=ctx)

    step()
    torch.cuda.synchronize()
    ctx.reset_timers()
    t = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - t) * 1e3 / a.steps
    stages = {}
    for name, st in (("cov", icp4r.STAGE_GICP_COV), ("nn", icp4r.STAGE_NN), ("iter", icp4r.STAGE_UPDATE),
                     ("batch", icp4r.STAGE_BATCH)):
        ms, n = ctx.stage_time_ms(st)
        stages[name] = {"avg_ms": ms, "launches": n}
    out = np.frombuffer(res.cpu().numpy().tobytes(), icp4r.RESULT_DTYPE)
    iters = out["iterations"] + 1
    line = {
        "measurement": f"gicp_{a.case}", "pairs": len(pairs), "src_points": int(sn.max()), "tgt_points": int(tn.max()),
        "k": k, "regularization": p.regularization, "max_iterations": p.max_iterations, "wall_ms_per_call": wall_ms, "device_ms_per_call": stages["batch"]["avg_ms"],
        "pairs_per_s": len(pairs) / (wall_ms * 1e-3), "stages": stages,
        "iterations_mean": float(iters.mean()), "converged": int(out["converged"].sum()),
    }
    if not a.no_cpu:
        import oracle  # CPU baseline only

        s, t_ = pairs[0]
        ncpu = min(a.cpu_points, len(s))
        mcpu = min(len(t_), ncpu * len(t_) // len(s))
        t = time.perf_counter()
        r = oracle.gicp_align(s[:ncpu], t_[:mcpu], k=k)
        cpu_s = time.perf_counter() - t
        line["cpu_baseline"] = {"seconds_per_pair": cpu_s, "cores": 1, "kind": "port",
                                "sample": f"oracle/gicp_oracle.c on the first {ncpu} source / {mcpu} target points "
                                          f"of pair 0 ({r['iterations'] + 1} iterations, brute-force k-NN)"}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
