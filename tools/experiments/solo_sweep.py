#!/usr/bin/env python3
"""Single-pair registration device time vs cloud size for the unbatched plans (diagnostic, GPU):
the solo plan (solo_kernel, ICP4R_SOLO=1), the multi-launch plan (ICP4R_SOLO=0) and the batched
LDS plan forced on one pair (ICP4R_NN_LDS=1).  Every mode's result is checked bit-identical to the
multi-launch plan's.  Prints one JSON line per (size, iteration setting).

    python tools/experiments/solo_sweep.py [--sizes 1024,2048,4096,6144,8192] [--reps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))

MODES = {"solo": {"ICP4R_SOLO": "1"}, "multi": {"ICP4R_SOLO": "0"}, "lds1": {"ICP4R_SOLO": "0", "ICP4R_NN_LDS": "1"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,2048,4096,6144,8192")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import icp4r
    from icp4r import synth

    ctx = icp4r.Context(0, plan=icp4r.env_plan())
    settings = {"pcl_defaults": icp4r.default_params(),
                "fixed20": icp4r.default_params(max_iterations=20, mse_threshold_absolute=-1.0,
                                                transformation_epsilon=-1.0)}
    for n in [int(x) for x in a.sizes.split(",")]:
        p = synth.make_pair(7, n)
        s, t = p.src_xyzi(), p.tgt_xyzi()
        for sname, params in settings.items():
            row = {"n": n, "params": sname}
            ref = None
            for mode, env in MODES.items():
                for k in ("ICP4R_SOLO", "ICP4R_NN_LDS"):
                    os.environ.pop(k, None)
                os.environ.update(env)
                r, _ = ctx.align(s, t, params)  # warm-up
                ctx.reset_timers()
                for _ in range(a.reps):
                    r, _ = ctx.align(s, t, params)
                ms, calls = ctx.batch_time_ms()
                row[mode + "_ms"] = ms
                if ref is None:
                    ref = bytes(r)
                row[mode + "_identical"] = bytes(r) == ref
                row["iterations"] = int(r.iterations)
            print(json.dumps(row), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
