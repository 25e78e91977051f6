"""Device time of one single-pair registration (HIP events, no profiler): python3 c1_time.py [n] [reps]
(20 iterations, no early stops: the same launches for any library build, diagnostic ones included)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))
import icp4r  # noqa: E402
from icp4r import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ctx = icp4r.Context(0, plan=icp4r.env_plan())
pr = synth.make_pair(0, n)
p = icp4r.default_params(max_iterations=20, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
ctx.align(pr.src_xyzi(), pr.tgt_xyzi(), p)
ctx.reset_timers()
for _ in range(reps):
    r, _ = ctx.align(pr.src_xyzi(), pr.tgt_xyzi(), p)
ms, k = ctx.batch_time_ms()
print(f"{os.environ.get('ICP4R_LIBRARY', 'default')}: n {n} device {ms:.4f} ms per registration ({k} calls), iterations {r.iterations}")
