#!/usr/bin/env python3
"""Does pass A's MSE chain (PCL's default MSE criteria live) set the single-pair update's pace?
C1's pair with PCL defaults vs the same with both MSE criteria off (need_mse = 0): update time per
launch (per-kernel events) and the registration's device time.  Prints one JSON line per variant."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))
import icp4r  # noqa: E402
from icp4r import synth  # noqa: E402

ctx = icp4r.Context(0, plan=icp4r.env_plan())
for name, n in (("C1", 2048), ("C2", 8192)):
    p = synth.make_pair(0 if name == "C1" else 1, n)
    s, t = p.src_xyzi(), p.tgt_xyzi()
    for label, kw in (("mse_live", {}), ("mse_off", dict(mse_threshold_absolute=-1.0, euclidean_fitness_epsilon=-1.0))):
        params = icp4r.default_params(**kw)
        r, _ = ctx.align(s, t, params)
        ctx.reset_timers()
        for _ in range(30):
            r, _ = ctx.align(s, t, params)
        dev_ms, calls = ctx.batch_time_ms()
        ctx.set_kernel_timing(True)
        ctx.reset_timers()
        for _ in range(10):
            r, _ = ctx.align(s, t, params)
        upd_ms, upd_n = ctx.stage_time_ms(icp4r.STAGE_UPDATE)
        ctx.set_kernel_timing(False)
        print(json.dumps({"config": name, "variant": label, "iterations": int(r.iterations),
                          "device_ms": dev_ms, "update_us_per_launch": 1e3 * upd_ms, "update_launches": upd_n}))
