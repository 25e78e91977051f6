"""NN work counters of a 256-pair 8k batch with the second chance off and on (diagnostic).

    python tools/sc_stats.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import icp4r
from icp4r import synth
pairs = [synth.make_pair(1000 + k, 8192) for k in range(256)]
ctx = icp4r.Context(0)
p = icp4r.default_params(max_iterations=20, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
from test_gpu_parity import _batch
args = _batch([(q.src_xyzi(), q.tgt_xyzi()) for q in pairs])
for sc in ("0", "1"):
    os.environ["ICP4R_SECOND_CHANCE"] = sc
    ctx.reset_timers()
    ctx.align_batch_host(*args, params=p)
    st = ctx.nn_stats()
    miss = st["cache_tested"] - st["cache_hits"]
    print(sc, st, "misses", miss, "sc frac of misses %.3f" % (st["second_chance_hits"] / max(miss, 1)))
