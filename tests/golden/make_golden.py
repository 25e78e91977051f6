"""Generate the committed golden fixtures — TEST INFRASTRUCTURE (run by hand; output is committed).

    python tests/golden/make_golden.py

Inputs are seeded synthetic radar pairs in the reference's own scan format (raw float32 records
x, y, z, intensity, v_r: /root/reference/src/iterative_closest_point.cpp:64-82, :354-385).  Expected
outputs come from the independent numpy twin (tests/golden/numpy_twin.py), NOT from the C oracle or
the HIP product, so the fixtures pin both.  The reference itself cannot run here (PCL/ROS absent,
SURVEY.md §8c) — see DESIGN.md §Oracle for what that means for parity.

Known-answer tests are analytic: identity (src == tgt, the node's order-0 frame,
iterative_closest_point.cpp:306-310), a pure translation and a pure yaw with exact correspondences.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))

import numpy_twin as twin  # noqa: E402
from icp4r import synth  # noqa: E402


def nn_digest(idx: np.ndarray, d2: np.ndarray) -> str:
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(idx, np.int32).tobytes())
    h.update(np.ascontiguousarray(d2, np.float32).tobytes())
    return h.hexdigest()


def pair_case(name: str, index: int, n: int, iters: int, full_nn: bool) -> dict:
    pair = synth.make_pair(index, n)
    synth.write_bin(os.path.join(HERE, f"{name}_src.bin"), pair.src)
    synth.write_bin(os.path.join(HERE, f"{name}_tgt.bin"), pair.tgt)
    src, tgt = pair.src_xyzi(), pair.tgt_xyzi()
    r = twin.icp(src, tgt, max_iterations=iters)
    tr0 = r["trace"][0]
    idx0, d20 = tr0["nn_idx0"], tr0["nn_d20"]
    rng = np.random.default_rng(7)
    rows = np.sort(rng.choice(n, size=min(256, n), replace=False))
    case = {
        "name": name, "pair_index": index, "n": n, "m": n, "max_iterations": iters,
        "src_bin": f"{name}_src.bin", "tgt_bin": f"{name}_tgt.bin",
        "T_gt": pair.T_gt.tolist(),
        "nn0_sha256": nn_digest(idx0, d20),
        "nn0_rows": rows.tolist(),
        "nn0_idx_rows": idx0[rows].tolist(),
        "nn0_d2_rows": [float(v) for v in d20[rows]],
        "mu_src0": tr0["mu_src"].tolist(), "mu_dst0": tr0["mu_dst"].tolist(), "sigma0": tr0["sigma"].tolist(),
        "T_final_trace": [t["T_final"].astype(float).tolist() for t in r["trace"]],
        "mse_trace": [t["mse"] for t in r["trace"]],
        "T": r["T"].astype(float).tolist(),
        "iterations": r["iterations"], "converged": r["converged"], "convergence_state": r["state"],
        "fitness": r["fitness"],
    }
    if full_nn:
        case["nn0_idx"] = idx0.tolist()
        case["nn0_d2"] = [float(v) for v in d20]
    return case


def kat_cases() -> list[dict]:
    rng = np.random.default_rng(4242)
    base = np.concatenate([rng.uniform(-20, 20, (300, 2)), rng.uniform(-2, 2, (300, 1))], axis=1).astype(np.float32)
    base = np.concatenate([base, rng.uniform(0, 30, (300, 1)).astype(np.float32)], axis=1)
    out = []
    # identity: src == tgt -> T = I (order-0 frame of the node)
    out.append({"name": "kat_identity", "src": base.tolist(), "tgt": base.tolist(), "T_expect": np.eye(4).tolist(),
                "tol_t": 1e-5, "tol_r": 1e-5})
    # pure translation: tgt = src + t, small enough that every NN is the true partner
    t = np.array([0.05, -0.03, 0.01], np.float32)
    tgt = base.copy()
    src = base.copy()
    src[:, :3] = base[:, :3] - t
    T = np.eye(4)
    T[:3, 3] = t
    out.append({"name": "kat_translation", "src": src.tolist(), "tgt": tgt.tolist(), "T_expect": T.tolist(),
                "tol_t": 1e-5, "tol_r": 1e-5})
    # pure yaw of 0.2 degree about the origin
    a = np.deg2rad(0.2)
    R = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    src = base.copy()
    src[:, :3] = (base[:, :3].astype(np.float64) @ R).astype(np.float32)  # R^T p
    T = np.eye(4)
    T[:3, :3] = R
    out.append({"name": "kat_yaw", "src": src.tolist(), "tgt": base.tolist(), "T_expect": T.tolist(),
                "tol_t": 1e-5, "tol_r": 1e-5})
    return out


def main():
    cases = [pair_case("c1_pair0_2k", 0, 2048, 10, full_nn=True),
             pair_case("c2_pair1_8k", 1, 8192, 20, full_nn=False)]
    golden = {"generator": "tests/golden/make_golden.py (numpy twin, float64 Umeyama)", "cases": cases,
              "kat": kat_cases()}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(golden, f)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
