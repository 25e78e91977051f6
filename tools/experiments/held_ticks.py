"""fold_update_held_kernel's stamps against fold_update_wide_kernel's (plan option phase_ticks = 1,
pair 0 of a single pair, the registration's last update, 10 ns ticks), relative to the kernel's
ticks[0]: 1 pass A end, 2 pass B end, 3 solve end; held only: 20.. the fold wave's pass-A chunk
starts, 26 its end, 6 the first filler's pass-B chunk offsets done, 28 / 29 pass B's first two chunk
starts, 30 its fold end, 32..45 each filler wave's first pass-B chunk staged.

    python3 tools/experiments/held_ticks.py [n] [fixed]   (fixed: 20 iterations, no early stops)
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))
import icp4r  # noqa: E402
from icp4r import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
fixed = len(sys.argv) > 2
ctx = icp4r.Context(0, plan=icp4r.env_plan())
ctx.set_plan_option("phase_ticks", 1)
lib = icp4r.load()
lib.icp4r__debug_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]
p = (icp4r.default_params(max_iterations=20, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0) if fixed
     else icp4r.default_params())
for held in (1, 0):
    ctx.set_plan_option("held_update", held)
    for rep in range(3):
        pr = synth.make_pair(0, n)
        ctx.align(pr.src_xyzi(), pr.tgt_xyzi(), p)
        buf = (C.c_uint64 * 48)()
        lib.icp4r__debug_ticks(ctx._h, buf, 48)
        t = [int(v) for v in buf]
        keys = [1, 2, 3] + ([9] if held else []) + (list(range(20, 27)) + [6, 28, 29, 30] + list(range(32, 46)) if held else [])
        rel = {k: round((t[k] - t[0]) * 0.01, 2) for k in keys if t[k] > t[0] or k == 9}
        print(json.dumps({"n": n, "held": held, "rep": rep, "rel_us": rel}), flush=True)
