"""Per-iteration GPU-vs-oracle comparison (ULP distance of T) for debugging bit-exactness."""
import sys, os, json
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("icp-4dradar_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import icp4r, oracle
from helpers import load_case_clouds

def ulps(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return int(np.abs(a - b).max())

g = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))
src, tgt = load_case_clouds(g["cases"][0])
ctx = icp4r.Context(0, plan=icp4r.env_plan())
for it in (1, 2, 3, 5, 10):
    r, out = ctx.align(src, tgt, icp4r.default_params(max_iterations=it), want_aligned=True)
    o = oracle.align(src, tgt, numerics=oracle.NUM_F32, max_iterations=it, trace=True, aligned=True)
    print(it, "T ulps", ulps(r.matrix(), o["T"]), "aligned ulps", ulps(out[:, :3], o["aligned"][:, :3]),
          "fit", r.fitness, o["fitness"], flush=True)
    if it == 1:
        print("gpu T\n", r.matrix(), "\noracle T\n", o["T"])
        print("oracle mu_src", o["trace"]["mu_src"][0], "mu_dst", o["trace"]["mu_dst"][0])
        print("oracle sigma", o["trace"]["sigma"][0].ravel())
# tiny case
rng = np.random.default_rng(1)
t = rng.uniform(-10, 10, (64, 4)).astype(np.float32)
s = t.copy(); s[:, 0] += 0.01
r, _ = ctx.align(s, t, icp4r.default_params(max_iterations=1))
o = oracle.align(s, t, numerics=oracle.NUM_F32, max_iterations=1, trace=True)
print("tiny ulps", ulps(r.matrix(), o["T"]))
print(r.matrix(), "\n", o["T"])
