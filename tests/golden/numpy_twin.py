"""Independent numpy restatement of PCL 1.8.1 default ICP — TEST INFRASTRUCTURE.

Written separately from oracle/icp_oracle.c (different language, vectorised brute-force NN, numpy's
LAPACK SVD) so the two restatements pin each other: SURVEY.md §8c — the reference has no tests and
PCL is not vendored, so parity with the reference is otherwise unpinned.  Semantics: SURVEY.md
Appendix A (icp.hpp computeTransformation / transformCloud, correspondence_estimation.hpp,
Eigen umeyama, default_convergence_criteria.hpp, registration.hpp getFitnessScore).

numpy float32 arithmetic is IEEE single precision without contraction, so the L2_Simple distance
``((dx*dx + dy*dy) + dz*dz)`` and the transform ``((r0*x + r1*y) + r2*z) + t`` below round exactly as
the reference's SSE code does.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def l2_simple_all(q: np.ndarray, tgt: np.ndarray) -> np.ndarray:
    """(len(q), len(tgt)) float32 distances with FLANN's operation order."""
    dx = q[:, None, 0] - tgt[None, :, 0]
    r = dx * dx
    dy = q[:, None, 1] - tgt[None, :, 1]
    r = r + dy * dy
    dz = q[:, None, 2] - tgt[None, :, 2]
    r = r + dz * dz
    return r


def nearest(q: np.ndarray, tgt: np.ndarray, chunk: int = 512):
    """Exact 1-NN; argmin returns the first (lowest) index on ties."""
    q = np.asarray(q, F32)
    tgt = np.asarray(tgt, F32)
    idx = np.empty(len(q), np.int32)
    d2 = np.empty(len(q), F32)
    for a in range(0, len(q), chunk):
        D = l2_simple_all(q[a:a + chunk], tgt)
        j = np.argmin(D, axis=1)
        idx[a:a + chunk] = j
        d2[a:a + chunk] = D[np.arange(len(j)), j]
    return idx, d2


def transform(T: np.ndarray, p: np.ndarray) -> np.ndarray:
    """transformCloud: x' = ((T00*x + T01*y) + T02*z) + T03, float32, unfused."""
    T = np.asarray(T, F32)
    p = np.asarray(p, F32)
    out = np.empty((len(p), 3), F32)
    for r in range(3):
        acc = T[r, 0] * p[:, 0]
        acc = T[r, 1] * p[:, 1] + acc
        acc = T[r, 2] * p[:, 2] + acc
        acc = T[r, 3] + acc
        out[:, r] = acc
    return out


def umeyama_f64(s: np.ndarray, d: np.ndarray) -> np.ndarray:
    """Rigid Umeyama in float64 (no scaling), Eigen's reflection rule, cast to Matrix4f."""
    s = s.astype(np.float64)
    d = d.astype(np.float64)
    ms, md = s.mean(0), d.mean(0)
    sigma = (d - md).T @ (s - ms) / len(s)
    U, _, Vt = np.linalg.svd(sigma)
    S = np.ones(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2] = -1
    R = U @ np.diag(S) @ Vt
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = md - R @ ms
    return T.astype(F32), sigma, ms, md


def eigen_gemm_kc(depth: int, l1: int = 32 * 1024, mr: int = 8, nr: int = 4) -> int:
    """Panel depth of Eigen 3.3's blocked GEMM for sigma = one_over_n * dst_demean * src_demean^T
    (evaluateProductBlockingSizesHeuristic, float, one thread, KcFactor 1): the lhs micro-panel
    (mr x kc) plus the rhs micro-panel (kc x nr) plus the mr x nr result block fit in L1, kc a
    multiple of the peeling factor 8; a longer depth is cut into equal-count panels, the last one as
    large as possible."""
    if depth < 48:
        return depth
    max_kc = max(((l1 - mr * nr * 4) // (mr * 4 + nr * 4)) & ~7, 1)
    if depth <= max_kc:
        return depth
    rem = depth % max_kc
    if rem == 0:
        return max_kc
    return max_kc - 8 * ((max_kc - 1 - rem) // (8 * (depth // max_kc + 1)))


def umeyama_sigma_f32(s: np.ndarray, d: np.ndarray, kc: int | None = None):
    """PCL's float Umeyama moments (Scalar = float): the centroids as Eigen's sequential
    rowwise().sum() times one_over_n, and sigma as Eigen's blocked GEMM — per panel of kc
    correspondences a sequential chain of fl(d'_a * s'_b) from +0, each panel added into sigma (from
    +0) scaled by one_over_n.  Sequential float sums via np.cumsum (numpy's add.reduce is pairwise)."""
    s = np.asarray(s, F32)
    d = np.asarray(d, F32)
    n = len(s)
    oon = F32(1.0) / F32(n)
    ms = np.array([np.cumsum(s[:, k], dtype=F32)[-1] * oon for k in range(3)], F32)
    md = np.array([np.cumsum(d[:, k], dtype=F32)[-1] * oon for k in range(3)], F32)
    sd = s - ms
    dd = d - md
    kc = eigen_gemm_kc(n) if kc is None else kc
    sigma = np.zeros(9, F32)
    for k0 in range(0, n, kc):
        k1 = min(n, k0 + kc)
        for a in range(3):
            for b in range(3):
                prod = dd[k0:k1, a] * sd[k0:k1, b]
                chain = np.cumsum(np.concatenate([np.zeros(1, F32), prod]), dtype=F32)[-1]
                sigma[a * 3 + b] = sigma[a * 3 + b] + oon * chain
    return sigma.reshape(3, 3), ms, md


def mat4_mul_f32(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """Matrix4f product, k-ordered unfused float32 accumulation (Eigen lazy product)."""
    A = np.asarray(A, F32)
    B = np.asarray(B, F32)
    C = np.empty((4, 4), F32)
    for i in range(4):
        for j in range(4):
            acc = A[i, 0] * B[0, j]
            acc = A[i, 1] * B[1, j] + acc
            acc = A[i, 2] * B[2, j] + acc
            acc = A[i, 3] * B[3, j] + acc
            C[i, j] = acc
    return C


def icp(src: np.ndarray, tgt: np.ndarray, max_iterations: int = 10, mse_abs: float = 1e-12,
        max_dist: float = np.sqrt(np.finfo(np.float64).max)):
    """PCL default ICP with float64 Umeyama.  Returns dict(T, iterations, converged, fitness, trace)."""
    src = np.asarray(src, F32)[:, :3]
    tgt = np.asarray(tgt, F32)[:, :3]
    X = src.copy()
    final = np.eye(4, dtype=F32)
    prev_mse = np.finfo(np.float64).max
    max_d2 = max_dist * max_dist
    it = 0
    trace = []
    converged = False
    state = 0
    while True:
        idx, d2 = nearest(X, tgt)
        keep = d2.astype(np.float64) <= max_d2
        if keep.sum() < 3:
            converged, state = False, 5
            break
        Tinc, sigma, ms, md = umeyama_f64(X[keep], tgt[idx[keep]])
        X = transform(Tinc, X)
        final = mat4_mul_f32(Tinc, final)
        it += 1
        mse = float(d2[keep].astype(np.float64).sum() / keep.sum())
        trace.append({"T_inc": Tinc, "T_final": final.copy(), "mse": mse, "ncorr": int(keep.sum()),
                      "sigma": sigma, "mu_src": ms, "mu_dst": md, "nn_idx0": idx if it == 1 else None,
                      "nn_d20": d2 if it == 1 else None})
        if it >= max_iterations:
            converged, state = True, 1
            break
        cos_a = 0.5 * (float(Tinc[0, 0]) + float(Tinc[1, 1]) + float(Tinc[2, 2]) - 1)
        tsq = float(Tinc[0, 3]) ** 2 + float(Tinc[1, 3]) ** 2 + float(Tinc[2, 3]) ** 2
        if cos_a >= 1.0 and tsq <= 0.0:
            converged, state = True, 2
            break
        if abs(mse - prev_mse) < mse_abs:
            converged, state = True, 3
            break
        prev_mse = mse
    Y = transform(final, src)
    _, fd = nearest(Y, tgt)
    fitness = float(fd.astype(np.float64).sum() / len(fd)) if len(fd) else np.finfo(np.float64).max
    return {"T": final, "iterations": it, "converged": converged, "state": state, "fitness": fitness,
            "trace": trace}
