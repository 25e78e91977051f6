"""nn_tile_kernel's phases per NN pass of one C1 registration (s_memrealtime, 10 ns ticks), with
plan option phase_ticks = 1 on a fresh context: workgroup (0, 0, 0) — staging to the barrier, the
seed, the traversal, the writes — and the launch's first start to last end over every workgroup;
then the update's phases (pass A, pass B, solve) of the last iteration.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))

import icp4r  # noqa: E402
from icp4r import synth  # noqa: E402

M64 = (1 << 64) - 1


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    for rep in range(3):
        ctx = icp4r.Context(0, plan=icp4r.env_plan())
        ctx.set_plan_option("phase_ticks", 1)
        pr = synth.make_pair(0, n)
        p = icp4r.default_params() if n == 2048 else icp4r.default_params(max_iterations=20,
                                                                          mse_threshold_absolute=-1.0,
                                                                          transformation_epsilon=-1.0)
        ctx.align(pr.src_xyzi(), pr.tgt_xyzi(), p)
        lib = icp4r.load()
        base = 32 + 20 * 1
        k = base + 64 * 16
        buf = (C.c_uint64 * k)()
        lib.icp4r__debug_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]
        if lib.icp4r__debug_ticks(ctx._h, buf, k):
            raise RuntimeError(lib.icp4r_last_error())
        t = [int(v) for v in buf]
        rows = []
        for ps in range(24):
            s = t[base + 16 * ps: base + 16 * ps + 16]
            if not s[0]:
                break
            first = M64 - s[6] if s[6] else 0
            # (round 6: the seed chain runs before the staging barrier — "seed" is then the chain's
            # end from the start, "stage" the barrier's; the traversal starts at the barrier)
            seed_first = s[2] < s[1]
            rows.append({"pass": ps, "stage": (s[1] - s[0]) * 0.01,
                         "seed": ((s[2] - s[0]) if seed_first else (s[2] - s[1])) * 0.01,
                         "traverse": (s[3] - max(s[1], s[2])) * 0.01, "write": (s[4] - s[3]) * 0.01,
                         "wg0": (s[4] - s[0]) * 0.01, "launch_span": (s[5] - first) * 0.01 if first else None,
                         "wg0_start_lag": (s[0] - first) * 0.01 if first else None,
                         "entry_to_start": (s[0] - s[7]) * 0.01 if s[7] else None})
        keys = ["stage", "seed", "traverse", "write", "wg0", "launch_span", "wg0_start_lag", "entry_to_start"]
        mean = {kk: round(sum(r[kk] for r in rows[1:]) / max(1, len(rows) - 1), 2) for kk in keys}
        print(json.dumps({"n": n, "rep": rep, "pass0": rows[0] if rows else None, "later_mean": mean}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
