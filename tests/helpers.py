"""Shared test helpers (pose error metrics, fixture loading)."""
from __future__ import annotations

import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# north_star parity bar: <= 1e-4 m translation, <= 1e-4 rad rotation on identical inputs
TOL_T = 1e-4
TOL_R = 1e-4


def rot_angle(R1: np.ndarray, R2: np.ndarray) -> float:
    """Angle (rad) of R1ᵀR2, accurate for small angles (atan2 of the skew part)."""
    M = np.asarray(R1, np.float64).T @ np.asarray(R2, np.float64)
    v = np.array([M[2, 1] - M[1, 2], M[0, 2] - M[2, 0], M[1, 0] - M[0, 1]])
    return float(np.arctan2(np.linalg.norm(v) / 2.0, (np.trace(M) - 1.0) / 2.0))


def pose_err(T1, T2) -> tuple[float, float]:
    T1 = np.asarray(T1, np.float64)
    T2 = np.asarray(T2, np.float64)
    return float(np.abs(T1[:3, 3] - T2[:3, 3]).max()), rot_angle(T1[:3, :3], T2[:3, :3])


def load_case_clouds(case: dict):
    from icp4r import synth

    src = synth.records_to_xyzi(synth.read_bin(os.path.join(GOLDEN_DIR, case["src_bin"])))
    tgt = synth.records_to_xyzi(synth.read_bin(os.path.join(GOLDEN_DIR, case["tgt_bin"])))
    return src, tgt
