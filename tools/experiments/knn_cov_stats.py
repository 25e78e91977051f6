"""k-NN covariance work counters: distance evaluations per query of gicp_knn_cov_kernel on the
bench clouds (an 8k scan, the 65k submap), k = 5 and 20.  Tooling only."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "icp-4dradar_amd")]

import icp4r
from icp4r import gicp, synth


def main():
    torch.zeros(1, device="cuda:0")
    ctx = icp4r.Context(0)
    ctx.set_kernel_timing(True)
    pr = synth.make_map_pair(0, n_src=8192)
    clouds = {"scan8k": np.ascontiguousarray(pr.src[:, :3]), "map65k": np.ascontiguousarray(pr.tgt[:, :3]),
              "pair8k": np.ascontiguousarray(synth.make_pair(0, 8192).tgt[:, :3])}
    for name, c in clouds.items():
        for k in (5, 20):
            gicp.covariances(c, k, 3, ctx=ctx)
            ctx.reset_timers()
            gicp.covariances(c, k, 3, ctx=ctx)
            st = ctx.nn_stats()
            print(json.dumps({"cloud": name, "n": len(c), "k": k, "evals_per_query": st["evaluations"] / len(c),
                              "box_tests_per_query": st["box_tests"] / len(c)}), flush=True)


if __name__ == "__main__":
    main()
