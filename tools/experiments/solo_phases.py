#!/usr/bin/env python3
"""Phase walls of solo_kernel (diagnostic; ICP4R_PHASE_TICKS=1): pair 0 of one registration of C1 and
C2, summed per phase by its thread 0 (s_memrealtime, 100 MHz), printed in us — total and per
iteration.  Slots (icp4r_kernels.hip, solo_kernel): staging, test, search, pass A, pass B, solve,
fitness test, fitness search, fitness sum, iterations.

    python tools/experiments/solo_phases.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))
NAMES = ["stage", "test", "search", "pass_a", "pass_b", "solve", "fit_test", "fit_search", "fit_sum"]


def main():
    os.environ["ICP4R_PHASE_TICKS"] = "1"
    import icp4r
    from icp4r import synth

    lib = icp4r.load()
    lib.icp4r__debug_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]
    fixed = dict(max_iterations=20, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
    os.environ.setdefault("ICP4R_SOLO", "1")  # (C2's 8192 sources are past the default solo size)
    for name, pair, params in (("C1", synth.make_pair(0, 2048), icp4r.default_params()),
                               ("C2", synth.make_pair(1, 8192), icp4r.default_params(**fixed))):
        ctx = icp4r.Context(0, plan=icp4r.env_plan())
        ctx.set_kernel_timing(True)
        s, t = pair.src_xyzi(), pair.tgt_xyzi()
        ctx.align(s, t, params)  # warm-up (allocates the tick slots)

        def ticks():
            buf = (C.c_uint64 * 32)()
            if lib.icp4r__debug_ticks(ctx._h, buf, 32) != 0:
                raise RuntimeError(icp4r.load().icp4r_last_error())
            return np.array(list(buf), np.float64)

        t0 = ticks()
        ctx.reset_timers()
        r, _ = ctx.align(s, t, params)
        d = ticks() - t0
        ms, _ = ctx.kernel_time_ms()
        it = max(d[9], 1)
        out = {"config": name, "iterations": int(r.iterations), "solo_kernel_ms": ms,
               "phases_us": {k: d[i] / 100.0 for i, k in enumerate(NAMES)},
               "per_iteration_us": {k: d[i] / 100.0 / it for i, k in enumerate(NAMES[1:6], 1)},
               "test_core_us_per_pass": d[27] / 100.0 / max(it - 1, 1), "test_overflow_passes": int(d[28]),
               "misses_per_pass": d[29] / max(it - 1, 1)}
        print(json.dumps(out), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
