"""Radar ego velocity and the scan parse (include/icp4r/icp4r_ego.h), mirroring the reference node's
per-frame code around its ICP call (src/iterative_closest_point.cpp):

    fitSineRansac(points, A_best, b_best, iterations, sigma)        :85-128   -> fitSineRansac()
    parse of the 5-float records into RadarPoint_Info2               :354-385  -> radar_features()
    static / dynamic split, Vxyz = (KᵀK)⁻¹ Kᵀ Vr                     :391-431  -> ego_velocity()

GPU-only: there is no CPU fallback (the library raises if it is missing).  Hypothesis pairs are
drawn reproducibly (SplitMix64 of seed + k, mod n) — the reference's std::random_device draw with
an inclusive upper bound is one of the bugs this fixes (icp4r_ego.h).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import Context, _check, _ptr, default_context, load

SIGMA = 0.5              # fitSineRansac's default (:89)
DYNAMIC_THRESHOLD = 0.2  # :396


class EgoParams(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("reserved0", C.c_int32), ("sigma", C.c_double),
                ("dynamic_threshold", C.c_double), ("seed", C.c_uint64), ("reserved", C.c_int32 * 8)]


class EgoResult(C.Structure):
    _fields_ = [("A", C.c_double), ("b", C.c_double), ("v", C.c_double * 3), ("score", C.c_double),
                ("n", C.c_int32), ("n_static", C.c_int32), ("iterations", C.c_int32), ("best", C.c_int32),
                ("status", C.c_int32), ("reserved", C.c_int32)]

    def velocity(self) -> np.ndarray:
        return np.array(self.v, np.float64)


assert C.sizeof(EgoResult) == 72
EGO_RESULT_DTYPE = np.dtype([("A", np.float64), ("b", np.float64), ("v", np.float64, 3), ("score", np.float64),
                             ("n", np.int32), ("n_static", np.int32), ("iterations", np.int32), ("best", np.int32),
                             ("status", np.int32), ("reserved", np.int32)])
assert EGO_RESULT_DTYPE.itemsize == 72

_bound = False


def _lib():
    global _bound
    L = load()
    if not _bound:
        vp, i32 = C.c_void_p, C.c_int32
        L.icp4r_ego_params_default.restype = None
        L.icp4r_ego_params_default.argtypes = [C.POINTER(EgoParams)]
        L.icp4r_radar_features.restype = C.c_int
        L.icp4r_radar_features.argtypes = [vp, vp, i32, vp, vp]
        L.icp4r_ego_velocity.restype = C.c_int
        L.icp4r_ego_velocity.argtypes = [vp, vp, i32, C.POINTER(EgoParams), C.POINTER(EgoResult), vp, vp]
        L.icp4r_ego_velocity_batch_device.restype = C.c_int
        L.icp4r_ego_velocity_batch_device.argtypes = [vp, vp, vp, vp, i32, i32, C.POINTER(EgoParams), vp, vp, vp]
        _bound = True
    return L


def default_params(**kw) -> EgoParams:
    p = EgoParams()
    _lib().icp4r_ego_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _records(rec) -> np.ndarray:
    rec = np.ascontiguousarray(rec, dtype=np.float32)
    if rec.ndim != 2 or rec.shape[1] != 5:
        raise ValueError(f"records must be (N, 5) float32 [x, y, z, intensity, v_r], got {rec.shape}")
    return rec


def radar_features(records, ctx: Context | None = None) -> tuple[np.ndarray, np.ndarray]:
    """(xyzi (N, 4): the PointXYZI cloud, feat (N, 4): distance, arfa, beta [deg], v_r)."""
    rec = _records(records)
    n = len(rec)
    xyzi = np.zeros((n, 4), np.float32)
    feat = np.zeros((n, 4), np.float32)
    ctx = ctx or default_context()
    _check(_lib().icp4r_radar_features(ctx.handle, _ptr(rec), n, _ptr(xyzi), _ptr(feat)), "icp4r_radar_features")
    return xyzi, feat


def ego_velocity(records, params: EgoParams | None = None, ctx: Context | None = None, want_mask: bool = False,
                 want_scores: bool = False):
    """Ego velocity of one scan: (EgoResult, static mask or None, per-hypothesis scores or None)."""
    rec = _records(records)
    n = len(rec)
    p = params if params is not None else default_params()
    ctx = ctx or default_context()
    r = EgoResult()
    mask = np.zeros(n, np.uint8) if want_mask else None
    H = p.iterations if p.iterations > 0 else int(n * 0.2)
    scores = np.zeros(max(H, 0), np.float64) if want_scores else None
    rc = _lib().icp4r_ego_velocity(ctx.handle, _ptr(rec), n, C.byref(p), C.byref(r),
                                   _ptr(mask) if mask is not None else None,
                                   _ptr(scores) if scores is not None and scores.size else None)
    _check(rc, "icp4r_ego_velocity")
    return r, mask, scores


def ego_velocity_batch_device(records_ptr: int, off_ptr: int, cnt_ptr: int, nscans: int, max_n: int,
                              results_ptr: int, params: EgoParams | None = None, mask_ptr: int | None = None,
                              ctx: Context | None = None, stream: int | None = None):
    """Many scans already in HBM (device pointers); asynchronous on `stream`."""
    p = params if params is not None else default_params()
    ctx = ctx or default_context()
    _check(_lib().icp4r_ego_velocity_batch_device(ctx.handle, records_ptr, off_ptr, cnt_ptr, nscans, max_n,
                                                  C.byref(p), results_ptr, mask_ptr,
                                                  C.c_void_p(stream) if stream else None),
           "icp4r_ego_velocity_batch_device")


def fitSineRansac(points, A_best: float = 0.0, b_best: float = 0.0, iterations: int | None = None,  # noqa: N802
                  sigma: float = SIGMA, seed: int | None = None, ctx: Context | None = None):
    """The node's fitSineRansac (:85-128) on a scan's records: returns (A_best, b_best, best score).
    A_best / b_best keep the values passed in when no hypothesis scores > 0."""
    kw = {"sigma": sigma}
    if iterations is not None:
        kw["iterations"] = int(iterations)
    if seed is not None:
        kw["seed"] = seed
    r, _, _ = ego_velocity(points, default_params(**kw), ctx)
    if r.best < 0:
        return A_best, b_best, r.score
    return r.A, r.b, r.score
