"""fold_update_held_kernel's pass A stamps (plan option phase_ticks = 1, pair 0, 10 ns ticks): the fold
wave's chunk starts (slots 20..23), its end (24), the first filler's chunk-0 store (25), the means (26);
relative to the kernel's ticks[0]."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))
import icp4r  # noqa: E402
from icp4r import synth  # noqa: E402

ctx = icp4r.Context(0, plan=icp4r.env_plan())
ctx.set_plan_option("phase_ticks", 1)
lib = icp4r.load()
lib.icp4r__debug_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]
for held in (1, 0):
    ctx.set_plan_option("held_update", held)
    for rep in range(3):
        pr = synth.make_pair(0, 2048)
        ctx.align(pr.src_xyzi(), pr.tgt_xyzi(), icp4r.default_params())
        buf = (C.c_uint64 * 32)()
        lib.icp4r__debug_ticks(ctx._h, buf, 32)
        t = [int(v) for v in buf]
        rel = {k: round((t[k] - t[0]) * 0.01, 2) for k in list(range(1, 9)) + list(range(20, 31)) if t[k] > t[0]}
        print(json.dumps({"held": held, "rep": rep, "rel_us": rel}), flush=True)
