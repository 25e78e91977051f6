"""Scan-to-map path on one GPU: map store + Sector_Search, and the
radar_odometry loop body (radar_odometry.cpp:382-396) with the submap registered by icp4r.

  * map: K synthetic radar scans of 6,554 points (SURVEY.md C5's scan size) posed along a trajectory
    (pointAssociateToMap on the device), default K = 1500 -> 9.8 M points (a long drive);
  * Sector_Search(p_now, 80 m, heading): device time (HIP events) of the count / scan / write
    kernels, HBM roofline (algorithmic bytes = 16 B/point read twice + 16 B per kept point written),
    and the single-thread CPU oracle (map_oracle.c, the full-traversal restatement) on the same map;
  * loop body: add_scan + sector search into device memory + 20-iteration ICP of the next scan
    against the submap (count stays on the device as tgt_n).  Checked against the oracle.

One JSON line per measurement.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("icp-4dradar_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402

import icp4r  # noqa: E402
import oracle  # noqa: E402  (checker / CPU baseline only)
from icp4r import synth  # noqa: E402
from icp4r.mapstore import KD_TREE, RADAR_RADIUS  # noqa: E402

PEAK_HBM_GBS = 8000.0


def pose(k: int):
    yaw = 0.02 * k
    R = np.array([[math.cos(yaw), -math.sin(yaw), 0.0], [math.sin(yaw), math.cos(yaw), 0.0], [0.0, 0.0, 1.0]])
    t = np.array([1.5 * k * math.cos(0.01 * k), 1.5 * k * math.sin(0.01 * k), 0.0])
    deg = math.degrees(math.atan2(math.sin(yaw), math.cos(yaw)))  # R2rpy's yaw: (-180, 180]
    return R, t, deg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=1500)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    ctx = icp4r.Context(0, plan=icp4r.env_plan())
    tree = KD_TREE(0.3, 0.6, 0.5, ctx=ctx)
    base = [synth.make_pair(7000 + i, 6554).src_xyzi() for i in range(64)]
    t0 = time.perf_counter()
    for k in range(a.scans):
        R, t, _ = pose(k)
        tree.add_scan(base[k % len(base)], R, t)
    add_s = time.perf_counter() - t0
    n = tree.size()
    R, t, heading = pose(a.scans - 1)
    center = t.astype(np.float32)
    dev = torch.device("cuda", 0)
    d_out = torch.empty((n + 8 * 6554, 4), dtype=torch.float32, device=dev)  # room for the loop's scans
    d_cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    tree.sector_search_device(center, RADAR_RADIUS, heading, d_out.data_ptr(), d_cnt.data_ptr())  # warm-up
    ctx.synchronize()
    tree.reset_timers()
    for _ in range(a.reps):
        tree.sector_search_device(center, RADAR_RADIUS, heading, d_out.data_ptr(), d_cnt.data_ptr())
    ctx.synchronize()
    ms, calls = tree.time_ms()
    kept = int(d_cnt.item())
    algo_bytes = 2 * 16 * n + 16 * kept
    # CPU oracle on the same map: the world-frame scans restated on the host, one full traversal
    world = []
    for k in range(a.scans):
        Rk, tk, _ = pose(k)
        world.append(oracle.associate_to_map(base[k % len(base)], Rk, tk))
    hm = np.concatenate(world)
    t1 = time.perf_counter()
    ref = oracle.sector_search(hm, center, RADAR_RADIUS, heading)
    cpu_s = time.perf_counter() - t1
    got = d_out[:kept].cpu().numpy()
    exact = kept == len(ref) and bool((got == hm[ref]).all())
    print(json.dumps({
        "measurement": "sector_search", "map_points": n, "kept": kept, "device_ms": ms, "launches": calls,
        "points_per_s": n / (ms * 1e-3), "roofline": {"bound": "hbm", "achieved": algo_bytes / (ms * 1e-3) / 1e9,
                                                      "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                                      "frac": algo_bytes / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                                                      "algorithmic_bytes": algo_bytes},
        "cpu_baseline": {"ms": cpu_s * 1e3, "cores": 1, "kind": "port",
                         "sample": f"map_oracle.c full traversal of the same {n}-point map"},
        "speedup_vs_cpu": cpu_s * 1e3 / ms, "identical_to_oracle": exact,
        "build_s_incl_host_upload": add_s}), flush=True)

    # radar_odometry loop body on the device, registered with icp4r (the node uses fast_gicp here)
    scan = synth.make_pair(9999, 6554).src_xyzi()
    src = torch.from_numpy(scan).to(dev)
    zero = torch.zeros(1, dtype=torch.int64, device=dev)
    sn = torch.tensor([len(scan)], dtype=torch.int32, device=dev)
    res = torch.zeros((1, 96), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    p = icp4r.default_params(max_iterations=20, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
    ctx.reset_timers()
    walls = []
    for rep in range(5):
        t2 = time.perf_counter()
        tree.add_scan(scan, R, t)
        tree.sector_search_device(center, RADAR_RADIUS, heading, d_out.data_ptr(), d_cnt.data_ptr())
        # the submap's size sizes the registration's plan (its tiles, index and workspace strides): read
        # back once per frame, as the node's host loop would; sizing the plan for the whole map (the
        # sector search's worst case) had launched ~1,200 mostly empty target tiles per NN pass
        ctx.synchronize()  # (the search runs on the context's stream)
        m_sub = int(d_cnt.item())
        batch = icp4r.Batch(src=src.data_ptr(), tgt=d_out.data_ptr(), src_off=zero.data_ptr(), src_n=sn.data_ptr(),
                            tgt_off=zero.data_ptr(), tgt_n=d_cnt.data_ptr(), npairs=1, max_src_n=len(scan),
                            max_tgt_n=m_sub)
        ctx.align_batch_device(batch, p, res.data_ptr(), None)
        ctx.synchronize()
        walls.append(time.perf_counter() - t2)
    bms, _ = ctx.batch_time_ms()
    r = np.frombuffer(res.cpu().numpy().tobytes(), dtype=icp4r.RESULT_DTYPE)[0]
    sub = d_out[: int(d_cnt.item())].cpu().numpy()
    o = oracle.align(scan, sub, numerics=oracle.NUM_F32, max_iterations=20, mse_threshold_absolute=-1.0,
                     transformation_epsilon=-1.0)
    print(json.dumps({"measurement": "scan_to_map_loop_body", "map_points": tree.size(), "submap": int(d_cnt.item()),
                      "wall_ms_median_add_search_icp": 1e3 * float(np.median(walls)),
                      "icp_device_ms_avg": bms, "iterations": int(r["iterations"]), "status": int(r["status"]),
                      "icp_bit_exact_vs_oracle": bool((r["T"].reshape(4, 4).T == o["T"]).all())}), flush=True)
    tree.close()
    ctx.close()


if __name__ == "__main__":
    main()
