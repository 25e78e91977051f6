"""Report every BASELINE.json config on one GPU (bench.py is the C3 headline line; this adds the rest).

  C1  1 pair 2k/2k, PCL defaults (10 iters, early stop live)        GPU latency vs the CPU oracle
  C2  1 pair 8k/8k, 20 iters fixed                                   single-pair latency (target split)
  C3  (bench.py)                                                     batched throughput
  C5  scan 8192 vs map 65540 (10 accumulated scans), 20 iters fixed  scan-to-map latency

Latencies are device time of the whole registration (library HIP events around it, no per-kernel
events inside) and host wall time of the synchronous icp4r_align call (includes the PCIe upload of
both clouds and the result download); one more call with per-kernel events gives the NN kernel's
time and work counters.
Each GPU result is checked bit-for-bit against the oracle.  One JSON line per config.
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("icp-4dradar_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402

import icp4r  # noqa: E402
import oracle  # noqa: E402
from icp4r import synth  # noqa: E402


def run(name, src, tgt, params, oparams, reps=5):
    ctx = icp4r.Context(0, plan=icp4r.env_plan())
    # the timed calls without per-kernel events, then (after a warm-up call that creates them) one
    # call with them for the NN kernel's time and work counters
    ctx.set_kernel_timing(False)
    r, _ = ctx.align(src, tgt, params)  # warm-up
    ctx.reset_timers()
    walls = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r, _ = ctx.align(src, tgt, params)
        walls.append(time.perf_counter() - t0)
    dev_ms, k = ctx.batch_time_ms()
    ctx.set_kernel_timing(True)
    ctx.align(src, tgt, params)
    ctx.reset_timers()
    ctx.align(src, tgt, params)
    dev_ev_ms, _ = ctx.batch_time_ms()
    nn_ms, nk = ctx.kernel_time_ms()
    k = 1
    evals = ctx.nn_counters()[0] / max(nk, 1)
    t0 = time.perf_counter()
    o = oracle.align(src, tgt, **oparams)
    cpu_s = time.perf_counter() - t0
    bit_exact = bool((r.matrix() == o["T"]).all() and r.iterations == o["iterations"] and r.fitness == o["fitness"])
    line = {"config": name, "n": len(src), "m": len(tgt), "iterations": r.iterations,
            "gpu_device_ms": dev_ms, "gpu_wall_ms_incl_pcie": 1e3 * float(np.median(walls)),
            "gpu_device_ms_with_kernel_events": dev_ev_ms,
            "nn_kernel_avg_ms": nn_ms, "nn_launches_per_call": nk // max(k, 1),
            "nn_evals_per_launch": evals, "nn_evaluated_fraction": evals / (len(src) * len(tgt)),
            "plan": icp4r.plan(1, len(src), len(tgt)),
            "cpu_oracle_ms_1thread": 1e3 * cpu_s, "speedup_device_vs_cpu": 1e3 * cpu_s / dev_ms,
            "bit_exact_vs_oracle": bit_exact}
    print(json.dumps(line), flush=True)
    ctx.close()


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="C1,C2,C5")
    only = ap.parse_args().only.split(",")
    # C1: the reference-default CPU config (PCL defaults, 10 iterations, early stop live)
    p = synth.make_pair(0, 2048)
    if "C1" in only:
        run("C1", p.src_xyzi(), p.tgt_xyzi(), icp4r.default_params(), {"numerics": oracle.NUM_F32})
    fixed = dict(max_iterations=20, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
    # C2: single 8k pair, 20 iterations
    p = synth.make_pair(1, 8192)
    if "C2" in only:
        run("C2", p.src_xyzi(), p.tgt_xyzi(), icp4r.default_params(**fixed), dict(numerics=oracle.NUM_F32, **fixed))
    # C5: 8k scan vs 64k map (10 accumulated scans)
    p = synth.make_map_pair(0)
    if "C5" in only:
        run("C5", p.src_xyzi(), p.tgt_xyzi(), icp4r.default_params(**fixed), dict(numerics=oracle.NUM_F32, **fixed),
            reps=3)


if __name__ == "__main__":
    main()
