"""Radar ego-velocity throughput: a device batch of scans vs the oracle on one
host core.

    python tools/bench_ego.py [--scans 1024] [--points 8192] [--steps 5]

The node's cost is fitSineRansac: (int)(0.2 N) hypotheses, each scored against all N points
(0.2 N² inlier tests, a double cos each) — 13.4 M tests per 8k-point scan.  roofline: the inlier
test is 2 FP64 FMA = 4 FLOP (A cos(a+b) = (A cos b) cos a - (A sin b) sin a; the compare and count
not counted) against the FP64 vector peak (78.6 TFLOP/s, AMD MI355X spec).
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
PEAK_FP64_TFLOPS = 78.6
FLOP_PER_TEST = 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=1024)
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-scans", type=int, default=3)
    a = ap.parse_args()
    import torch

    from icp4r import Context, ego, synth

    base, v = synth.make_sequence(0, frames=32, n=a.points)
    recs = np.stack([base[k % len(base)] for k in range(a.scans)])  # scan s draws its own hypotheses
    dev = torch.device("cuda", 0)
    rec_d = torch.from_numpy(recs.reshape(-1, 5)).to(dev)
    cnt = torch.full((a.scans,), a.points, dtype=torch.int32, device=dev)
    off = torch.arange(a.scans, dtype=torch.int64, device=dev) * a.points
    res = torch.zeros((a.scans, 72), dtype=torch.uint8, device=dev)
    ctx = Context(0)
    p = ego.default_params()
    side = torch.cuda.Stream(dev)  # a real stream handle: the null handle would select the context's stream
    stream = side.cuda_stream

    def step():
        ego.ego_velocity_batch_device(rec_d.data_ptr(), off.data_ptr(), cnt.data_ptr(), a.scans, a.points,
                                      res.data_ptr(), params=p, ctx=ctx, stream=stream)

    step()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record(side)
    for _ in range(a.steps):
        step()
    t1.record(side)
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / a.steps
    out = np.frombuffer(res.cpu().numpy().tobytes(), dtype=ego.EGO_RESULT_DTYPE)
    H = int(a.points * 0.2)
    tests = a.scans * H * a.points
    achieved = tests * FLOP_PER_TEST / (ms * 1e-3) / 1e12
    import oracle  # CPU baseline only

    t = time.perf_counter()
    for k in range(a.cpu_scans):
        f = oracle.ego_features(recs[k])
        A, b, *_ = oracle.ego_ransac(f)
        oracle.ego_split_lsq(f, A, b)
    cpu_s = (time.perf_counter() - t) / a.cpu_scans
    line = {
        "measurement": "ego_velocity_batch", "scans": a.scans, "points": a.points, "hypotheses_per_scan": H,
        "device_ms_per_batch": ms, "scans_per_s": a.scans / (ms * 1e-3),
        "roofline": {"bound": "fp64-valu", "achieved": achieved, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_FP64_TFLOPS, "inlier_tests_per_batch": tests,
                     "note": "whole batch time (features + RANSAC + select); 2 FP64 FMA (4 FLOP) per inlier test"},
        "cpu_baseline": {"value": 1.0 / cpu_s, "unit": "scans/s", "cores": 1, "kind": "port",
                         "sample": f"{a.cpu_scans} scans of the same batch, oracle/ego_oracle.c (-O2, glibc cos)"},
        "speedup_vs_cpu": (a.scans / (ms * 1e-3)) * cpu_s,
        "status_nonzero": int((out["status"] != 0).sum()),
        "velocity_xy_error_max": float(np.abs(out["v"][:, :2] - (-v[:2])).max()),
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
