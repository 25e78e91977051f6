import json, sys
sys.path.insert(0, "icp-4dradar_amd")
import icp4r
from icp4r import synth
ctx = icp4r.Context(0, plan=icp4r.env_plan())
for n in (300, 700, 1024):
    p = synth.make_pair(50 + n, n)
    s, t = p.src_xyzi(), p.tgt_xyzi()
    params = icp4r.default_params()
    solo = icp4r.plan(1, n, n)["solo"]
    r, _ = ctx.align(s, t, params)
    ctx.reset_timers()
    for _ in range(50):
        r, _ = ctx.align(s, t, params)
    ms, k = ctx.batch_time_ms()
    print(json.dumps({"n": n, "device_ms": ms, "iterations": int(r.iterations), "solo": bool(solo)}))
