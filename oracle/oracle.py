"""ctypes loader for the C oracle (oracle/icp_oracle.c) — TEST INFRASTRUCTURE ONLY.

This is the checker and the CPU-baseline leg.  Only tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product path (icp4r) never does.
Parity status: unpinned by the reference (no reference tests exist; PCL is not vendored) —
pinned by analytic known-answer tests and an independent numpy/scipy twin.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libicp_oracle.so")

NUM_F32, NUM_F64 = 0, 1
NN_KDTREE, NN_BRUTE = 0, 1


class OracleParams(C.Structure):
    _fields_ = [
        ("max_iterations", C.c_int32),
        ("min_correspondences", C.c_int32),
        ("max_correspondence_distance", C.c_double),
        ("transformation_epsilon", C.c_double),
        ("transformation_rotation_epsilon", C.c_double),
        ("euclidean_fitness_epsilon", C.c_double),
        ("mse_threshold_absolute", C.c_double),
        ("max_iterations_similar_transforms", C.c_int32),
        ("numerics", C.c_int32),
        ("nn", C.c_int32),
        ("compute_fitness", C.c_int32),
        ("huber_delta", C.c_double),
        ("fitness_max_range", C.c_double),
        ("eigen_l1_bytes", C.c_int32),
        ("eigen_gebp_mr", C.c_int32),
    ]


class OracleResult(C.Structure):
    _fields_ = [
        ("T", C.c_float * 16),
        ("fitness", C.c_double),
        ("iterations", C.c_int32),
        ("converged", C.c_int32),
        ("status", C.c_int32),
        ("convergence_state", C.c_int32),
        ("n_correspondences", C.c_int32),
        ("reserved", C.c_int32),
    ]


class OracleTrace(C.Structure):
    _fields_ = [
        ("T_inc", C.c_void_p),
        ("T_final", C.c_void_p),
        ("mse", C.c_void_p),
        ("ncorr", C.c_void_p),
        ("sigma", C.c_void_p),
        ("mu_src", C.c_void_p),
        ("mu_dst", C.c_void_p),
    ]


class GicpOracleParams(C.Structure):
    _fields_ = [("k", C.c_int32), ("max_iterations", C.c_int32), ("rotation_epsilon", C.c_double),
                ("transformation_epsilon", C.c_double), ("max_correspondence_distance", C.c_double),
                ("regularization", C.c_int32), ("lm_max_iterations", C.c_int32), ("lm_init_lambda_factor", C.c_double)]


class GicpOracleResult(C.Structure):
    _fields_ = [("T", C.c_double * 16), ("iterations", C.c_int32), ("converged", C.c_int32),
                ("lm_failed", C.c_int32), ("n_valid", C.c_int32)]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_params_default.argtypes = [C.POINTER(OracleParams)]
        L.oracle_align.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_int32,
                                   C.c_void_p, C.POINTER(OracleParams), C.POINTER(OracleResult),
                                   C.c_void_p, C.POINTER(OracleTrace)]
        L.oracle_align.restype = C.c_int
        L.oracle_nearest.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_int32,
                                     C.c_int32, C.c_void_p, C.c_void_p]
        L.oracle_nearest.restype = C.c_int
        L.oracle_fitness.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_int32,
                                     C.c_void_p, C.c_double, C.c_int32]
        L.oracle_fitness.restype = C.c_double
        L.oracle_kdtree_leaf_visits.restype = C.c_int64
        L.oracle_rot_f32.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_rot_f32.restype = None
        L.oracle_calc_dist.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_calc_dist.restype = C.c_float
        L.oracle_calc_heading.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_calc_heading.restype = C.c_float
        L.oracle_sector_keep.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_float]
        L.oracle_sector_keep.restype = C.c_int
        L.oracle_sector_search.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_float, C.c_float,
                                           C.c_void_p]
        L.oracle_sector_search.restype = C.c_int64
        L.oracle_associate_to_map.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.ego_features.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
        L.ego_features.restype = None
        L.ego_hyp_index.argtypes = [C.c_uint64, C.c_int64, C.c_int32]
        L.ego_hyp_index.restype = C.c_int32
        L.ego_fit_sine_ransac.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_double, C.c_uint64,
                                          C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_void_p,
                                          C.POINTER(C.c_int32)]
        L.ego_fit_sine_ransac.restype = C.c_double
        L.ego_split_lsq.argtypes = [C.c_void_p, C.c_int32, C.c_double, C.c_double, C.c_double, C.c_void_p,
                                    C.c_void_p]
        L.ego_split_lsq.restype = C.c_int32
        L.gicp_oracle_params_default.argtypes = [C.POINTER(GicpOracleParams)]
        L.gicp_oracle_params_default.restype = None
        L.gicp_oracle_covariances.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]
        L.gicp_oracle_covariances.restype = None
        L.gicp_oracle_align.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p,
                                        C.POINTER(GicpOracleParams), C.POINTER(GicpOracleResult)]
        L.gicp_oracle_align.restype = C.c_int
        _lib = L
    return _lib


def default_params(**kw) -> OracleParams:
    p = OracleParams()
    lib().oracle_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _cloud(a: np.ndarray):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] < 3:
        raise ValueError("cloud must be (N, >=3) float32")
    return a, a.shape[0], a.shape[1]


def align(src: np.ndarray, tgt: np.ndarray, guess: np.ndarray | None = None, trace: bool = False,
          aligned: bool = False, **params):
    """Run the restated PCL ICP.  Returns a dict with T (4x4, float32), fitness, iterations, ..."""
    s, n, ss = _cloud(src)
    t, m, ts = _cloud(tgt)
    p = default_params(**params)
    r = OracleResult()
    g = None
    if guess is not None:
        g = np.ascontiguousarray(np.asarray(guess, np.float32).T.reshape(16))  # column-major
    tr = None
    bufs = {}
    if trace:
        it = max(1, p.max_iterations)
        bufs = {
            "T_inc": np.zeros((it, 16), np.float32), "T_final": np.zeros((it, 16), np.float32),
            "mse": np.zeros(it, np.float64), "ncorr": np.zeros(it, np.int32),
            "sigma": np.zeros((it, 9), np.float64), "mu_src": np.zeros((it, 3), np.float64),
            "mu_dst": np.zeros((it, 3), np.float64),
        }
        tr = OracleTrace(*[bufs[k].ctypes.data for k in ("T_inc", "T_final", "mse", "ncorr", "sigma", "mu_src", "mu_dst")])
    out = np.zeros((n, 4), np.float32) if aligned else None
    lib().oracle_align(s.ctypes.data if n else None, n, ss, t.ctypes.data if m else None, m, ts,
                       g.ctypes.data if g is not None else None, C.byref(p), C.byref(r),
                       out.ctypes.data if out is not None else None, C.byref(tr) if tr else None)
    res = {
        "T": np.array(r.T, np.float32).reshape(4, 4).T.copy(),
        "fitness": r.fitness, "iterations": r.iterations, "converged": bool(r.converged),
        "status": r.status, "convergence_state": r.convergence_state,
        "n_correspondences": r.n_correspondences,
    }
    if trace:
        k = r.iterations
        res["trace"] = {
            "T_inc": bufs["T_inc"][:k].reshape(k, 4, 4).transpose(0, 2, 1).copy(),
            "T_final": bufs["T_final"][:k].reshape(k, 4, 4).transpose(0, 2, 1).copy(),
            "mse": bufs["mse"][:k].copy(), "ncorr": bufs["ncorr"][:k].copy(),
            "sigma": bufs["sigma"][:k].reshape(k, 3, 3).copy(),
            "mu_src": bufs["mu_src"][:k].copy(), "mu_dst": bufs["mu_dst"][:k].copy(),
        }
    if aligned:
        res["aligned"] = out
    return res


def rot_f32(sigma: np.ndarray) -> np.ndarray:
    """PCL's float Umeyama rotation of a 3x3 sigma (row-major): Eigen's JacobiSVD<Matrix3f> + umeyama."""
    s = np.ascontiguousarray(np.asarray(sigma, np.float32).reshape(9))
    R = np.empty(9, np.float32)
    lib().oracle_rot_f32(s.ctypes.data, R.ctypes.data)
    return R.reshape(3, 3)


def nearest(query: np.ndarray, tgt: np.ndarray, nn: int = NN_BRUTE):
    q, n, qs = _cloud(query)
    t, m, ts = _cloud(tgt)
    idx = np.empty(n, np.int32)
    d2 = np.empty(n, np.float32)
    rc = lib().oracle_nearest(q.ctypes.data, n, qs, t.ctypes.data, m, ts, nn, idx.ctypes.data, d2.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"oracle_nearest failed: {rc}")
    return idx, d2


def fitness(src: np.ndarray, tgt: np.ndarray, T: np.ndarray, max_range: float = np.finfo(np.float64).max,
            nn: int = NN_KDTREE) -> float:
    s, n, ss = _cloud(src)
    t, m, ts = _cloud(tgt)
    Tc = np.ascontiguousarray(np.asarray(T, np.float32).T.reshape(16))
    return lib().oracle_fitness(s.ctypes.data, n, ss, t.ctypes.data, m, ts, Tc.ctypes.data, max_range, nn)


# ---------------------------------------------------------------------------------------------------
# Scan-to-map submap path (map_oracle.c): ikd-Tree map store + Sector_Search as radar_odometry uses it.

def calc_heading(a, b) -> float:
    a = np.ascontiguousarray(a, np.float32)[:3].copy()
    b = np.ascontiguousarray(b, np.float32)[:3].copy()
    return float(lib().oracle_calc_heading(a.ctypes.data, b.ctypes.data))


def sector_search(map_pts: np.ndarray, center, radius: float, heading: float) -> np.ndarray:
    """KD_TREE::Sector_Search over an append-only map: indices of the kept points, insertion order."""
    m, n, stride = _cloud(map_pts)
    c = np.ascontiguousarray(center, np.float32)[:3].copy()
    out = np.empty(max(n, 1), np.int64)
    k = lib().oracle_sector_search(m.ctypes.data, n, stride, c.ctypes.data, radius, heading, out.ctypes.data)
    return out[:k].copy()


def associate_to_map(pts: np.ndarray, R: np.ndarray, t: np.ndarray) -> np.ndarray:
    """pointAssociateToMap: (n, 4) float32 x, y, z, intensity -> world frame (double math, float out)."""
    p = np.ascontiguousarray(pts, np.float32).reshape(-1, 4)
    Rd = np.ascontiguousarray(R, np.float64).reshape(9)
    td = np.ascontiguousarray(t, np.float64).reshape(3)
    out = np.empty_like(p)
    lib().oracle_associate_to_map(p.ctypes.data, len(p), Rd.ctypes.data, td.ctypes.data, out.ctypes.data)
    return out


# ---- radar ego velocity (ego_oracle.c)
EGO_SEED = 0x1CB4D12A5EED  # icp4r_ego_params_default


def ego_features(records: np.ndarray) -> np.ndarray:
    """The node's parse (:373-384): (N, 4) float32 distance, arfa, beta [deg], v_r."""
    rec = np.ascontiguousarray(records, dtype=np.float32)
    feat = np.zeros((len(rec), 4), np.float32)
    if len(rec):
        lib().ego_features(rec.ctypes.data, len(rec), feat.ctypes.data)
    return feat


def ego_ransac(feat: np.ndarray, iterations: int | None = None, sigma: float = 0.5, seed: int = EGO_SEED):
    """fitSineRansac (:85-128) with the reproducible hypothesis stream: (A, b, best score, best index,
    per-hypothesis scores)."""
    feat = np.ascontiguousarray(feat, dtype=np.float32)
    n = len(feat)
    it = int(n * 0.2) if iterations is None or iterations <= 0 else int(iterations)
    A, b, bh = C.c_double(0.0), C.c_double(0.0), C.c_int32(-1)
    scores = np.zeros(max(it, 1), np.float64)
    best = lib().ego_fit_sine_ransac(feat.ctypes.data if n else None, n, it, sigma, seed, C.byref(A), C.byref(b),
                                     scores.ctypes.data, C.byref(bh))
    return A.value, b.value, best, bh.value, scores[:it]


def ego_split_lsq(feat: np.ndarray, A: float, b: float, dyn_threshold: float = 0.2):
    """Split + Vxyz (:391-431): (V (3,), static mask (N,) uint8, number of static points)."""
    feat = np.ascontiguousarray(feat, dtype=np.float32)
    n = len(feat)
    mask = np.zeros(n, np.uint8)
    V = np.zeros(3, np.float64)
    ns = lib().ego_split_lsq(feat.ctypes.data if n else None, n, A, b, dyn_threshold, mask.ctypes.data if n else None,
                             V.ctypes.data)
    return V, mask, ns


# ---- GICP (gicp_oracle.c)
GICP_REG_NONE, GICP_REG_MIN_EIG, GICP_REG_NORMALIZED_MIN_EIG, GICP_REG_PLANE, GICP_REG_FROBENIUS = 0, 1, 2, 3, 4


def gicp_params(**kw) -> GicpOracleParams:
    p = GicpOracleParams()
    lib().gicp_oracle_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _xyz4(a: np.ndarray) -> np.ndarray:
    a = np.asarray(a, np.float32)
    out = np.zeros((len(a), 4), np.float32)
    out[:, :3] = a[:, :3]
    return out


def gicp_covariances(cloud: np.ndarray, k: int = 20, regularization: int = GICP_REG_PLANE) -> np.ndarray:
    c = _xyz4(cloud)
    out = np.zeros((len(c), 9), np.float64)
    if len(c):
        lib().gicp_oracle_covariances(c.ctypes.data, len(c), k, regularization, out.ctypes.data)
    return out.reshape(-1, 3, 3)


def gicp_align(src: np.ndarray, tgt: np.ndarray, guess: np.ndarray | None = None, **params) -> dict:
    """FastGICPSingleThread restated: T (4x4 float64: the double x0; final_transformation_ is its
    float), iterations (nr_iterations_), converged, lm_failed, n_valid."""
    s, t = _xyz4(src), _xyz4(tgt)
    p = gicp_params(**params)
    r = GicpOracleResult()
    g = None if guess is None else np.ascontiguousarray(np.asarray(guess, np.float64).reshape(16))
    rc = lib().gicp_oracle_align(s.ctypes.data if len(s) else None, len(s), t.ctypes.data if len(t) else None,
                                 len(t), g.ctypes.data if g is not None else None, C.byref(p), C.byref(r))
    return {"rc": rc, "T": np.array(r.T, np.float64).reshape(4, 4), "iterations": r.iterations,
            "converged": bool(r.converged), "lm_failed": bool(r.lm_failed), "n_valid": r.n_valid}
