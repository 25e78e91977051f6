"""Generalized ICP (include/icp4r/icp4r_gicp.h), mirroring fast_gicp as the reference's
radar_odometry node drives it on its scan-to-map path (src/radar_odometry.cpp:398-411):

    fast_gicp::FastGICPSingleThread<PointXYZI, PointXYZI> fgicp_st;      -> FastGICPSingleThread()
    fgicp_st.clearTarget(); fgicp_st.clearSource();                      -> clearTarget / clearSource
    fgicp_st.setInputTarget(SubMap); fgicp_st.setInputSource(scan_map);  -> setInputTarget / setInputSource
    fgicp_st.setCorrespondenceRandomness(5);                             -> setCorrespondenceRandomness
    fgicp_st.align(*Final);                                              -> align
    fgicp_st.getFitnessScore(); hasConverged(); getFinalTransformation() -> same names

GPU-only: there is no CPU fallback (the library raises if it is missing).  fast_gicp itself is not
in this image; the algorithm restated is described in icp4r_gicp.h and oracle/gicp_oracle.h.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import (DBL_MAX, E_EMPTY, E_INVALID, E_NONFINITE, OK, Batch, Context, ICP4RError, Result, _check, _cloud,
               _ptr, default_context, load)

REG_NONE, REG_MIN_EIG, REG_NORMALIZED_MIN_EIG, REG_PLANE, REG_FROBENIUS = 0, 1, 2, 3, 4
FLT_MAX = float(np.finfo(np.float32).max)


class GicpParams(C.Structure):
    _fields_ = [("k_correspondences", C.c_int32), ("max_iterations", C.c_int32), ("rotation_epsilon", C.c_double),
                ("transformation_epsilon", C.c_double), ("max_correspondence_distance", C.c_double),
                ("regularization", C.c_int32), ("lm_max_iterations", C.c_int32),
                ("lm_init_lambda_factor", C.c_double), ("compute_fitness", C.c_int32), ("reserved", C.c_int32 * 9)]


_bound = False


def _lib():
    global _bound
    L = load()
    if not _bound:
        vp, i32 = C.c_void_p, C.c_int32
        L.icp4r_gicp_params_default.restype = None
        L.icp4r_gicp_params_default.argtypes = [C.POINTER(GicpParams)]
        L.icp4r_gicp_align.restype = C.c_int
        L.icp4r_gicp_align.argtypes = [vp, vp, i32, i32, vp, i32, i32, vp, C.POINTER(GicpParams), C.POINTER(Result),
                                       vp, i32]
        L.icp4r_gicp_align_batch_device.restype = C.c_int
        L.icp4r_gicp_align_batch_device.argtypes = [vp, C.POINTER(Batch), C.POINTER(GicpParams), vp, vp]
        L.icp4r_gicp_covariances.restype = C.c_int
        L.icp4r_gicp_covariances.argtypes = [vp, vp, i32, i32, i32, i32, vp]
        _bound = True
    return L


def default_params(**kw) -> GicpParams:
    p = GicpParams()
    _lib().icp4r_gicp_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def align(src, tgt, params: GicpParams | None = None, guess=None, want_aligned: bool = False,
          ctx: Context | None = None) -> tuple[Result, np.ndarray | None]:
    """One pair from host arrays (N, >=3) float32; guess row-major 4x4 or None."""
    ctx = ctx or default_context()
    s, n, ss = _cloud(src)
    t, m, ts = _cloud(tgt)
    p = params if params is not None else default_params()
    g = None if guess is None else np.ascontiguousarray(np.asarray(guess, np.float32).T.reshape(16))
    out = np.zeros((n, 4), np.float32) if want_aligned else None
    r = Result()
    rc = _lib().icp4r_gicp_align(ctx.handle, _ptr(s), n, ss, _ptr(t), m, ts, _ptr(g) if g is not None else None,
                                 C.byref(p), C.byref(r), _ptr(out) if out is not None else None, 16)
    if rc not in (OK, E_EMPTY, E_NONFINITE):
        _check(rc, "icp4r_gicp_align")
    return r, out


def align_batch_device(batch: Batch, params: GicpParams, results_ptr: int, stream: int | None = None,
                       ctx: Context | None = None):
    """Device-resident batch (icp4r_batch of torch.cuda tensor pointers); asynchronous on `stream`."""
    ctx = ctx or default_context()
    _check(_lib().icp4r_gicp_align_batch_device(ctx.handle, C.byref(batch), C.byref(params), C.c_void_p(results_ptr),
                                                C.c_void_p(stream) if stream else None),
           "icp4r_gicp_align_batch_device")


def covariances(cloud, k: int = 20, regularization: int = REG_PLANE, ctx: Context | None = None) -> np.ndarray:
    """FastGICP::calculate_covariances of one cloud: (N, 3, 3) float64."""
    ctx = ctx or default_context()
    c, n, cs = _cloud(cloud)
    out = np.zeros((n, 3, 3), np.float64)
    _check(_lib().icp4r_gicp_covariances(ctx.handle, _ptr(c), n, cs, k, regularization, _ptr(out)),
           "icp4r_gicp_covariances")
    return out


class FastGICPSingleThread:
    """fast_gicp::FastGICPSingleThread<PointXYZI, PointXYZI> surface used by the reference node
    (defaults: k = 20, PLANE regularisation, 64 iterations, rotation / transformation epsilon 2e-3 /
    5e-4, LM with 10 trials)."""

    def __init__(self, context: Context | None = None):
        self._ctx = context
        self._p = default_params()
        self._src = None
        self._tgt = None
        self._result: Result | None = None

    # --- inputs ---
    def setInputSource(self, cloud):
        self._src = np.ascontiguousarray(cloud, np.float32)
        self._result = None

    def setInputTarget(self, cloud):
        self._tgt = np.ascontiguousarray(cloud, np.float32)
        self._result = None

    def clearSource(self):
        self._src = None
        self._result = None

    def clearTarget(self):
        self._tgt = None
        self._result = None

    # --- FastGICP / LsqRegistration setters ---
    def setCorrespondenceRandomness(self, k: int):
        self._p.k_correspondences = int(k)

    def setRegularizationMethod(self, method: int):
        self._p.regularization = int(method)

    def setMaxCorrespondenceDistance(self, distance_threshold: float):
        self._p.max_correspondence_distance = float(distance_threshold)

    def setMaximumIterations(self, nr_iterations: int):
        self._p.max_iterations = int(nr_iterations)

    def setRotationEpsilon(self, eps: float):
        self._p.rotation_epsilon = float(eps)

    def setTransformationEpsilon(self, eps: float):
        self._p.transformation_epsilon = float(eps)

    def setInitialLambdaFactor(self, init_lambda_factor: float):
        self._p.lm_init_lambda_factor = float(init_lambda_factor)

    def params(self) -> GicpParams:
        return self._p

    # --- Registration::align ---
    def align(self, output=None, guess=None) -> np.ndarray:
        if self._tgt is None or len(self._tgt) == 0:
            raise ICP4RError(E_EMPTY, "No input target dataset was given!")
        if self._src is None:
            raise ICP4RError(E_INVALID, "No input source dataset was given!")
        r, aligned = align(self._src, self._tgt, self._p, guess=guess, want_aligned=True, ctx=self._ctx)
        self._result = r
        out = self._src.copy()
        out[:, :3] = aligned[:, :3]
        if output is not None:
            output[...] = out
            return output
        return out

    def hasConverged(self) -> bool:
        return bool(self._result is not None and self._result.converged)

    def getFinalTransformation(self) -> np.ndarray:
        if self._result is None:
            return np.eye(4, dtype=np.float32)
        return self._result.matrix()

    def getFitnessScore(self, max_range: float = DBL_MAX) -> float:
        if self._result is None:
            return DBL_MAX
        if max_range == DBL_MAX:
            return self._result.fitness  # computed once inside align
        return (self._ctx or default_context()).fitness(self._src, self._tgt, self.getFinalTransformation(), max_range)

    def result(self) -> Result | None:
        return self._result

    def nr_iterations(self) -> int:
        return 0 if self._result is None else self._result.iterations
