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


def _plane(x, y, c, s):
    """Eigen apply_rotation_in_the_plane on two equal-length float32 lists (in place)."""
    if c == F32(1) and s == F32(0):
        return
    for i in range(len(x)):
        xi, yi = x[i], y[i]
        x[i] = c * xi + s * yi
        y[i] = -s * xi + c * yi


def eigen_jacobi_svd3_f32(A):
    """Eigen 3.3 JacobiSVD<Matrix3f>(A, ComputeFullU | ComputeFullV) in float32 scalars, written from
    Eigen's SVD/JacobiSVD.h compute(), misc/RealSvd2x2.h and Jacobi/Jacobi.h (square input: no QR
    preconditioner; scale by the largest |a_ij|; two-sided 2x2 sweeps over (1,0), (2,0), (2,1) until
    every off-diagonal pair is within max(FLT_MIN, 2 eps * max |diag| seen); sign fix; swap sort).
    Returns U, S, V as 3x3 / 3 float32 arrays (row-major, U[r][c])."""
    one, zero = F32(1), F32(0)
    fmin = F32(np.finfo(np.float32).tiny)
    precision = F32(2) * F32(np.finfo(np.float32).eps)
    A = [[F32(A[r][c]) for c in range(3)] for r in range(3)]
    scale = zero
    for r in range(3):
        for c in range(3):
            scale = abs(A[r][c]) if scale < abs(A[r][c]) else scale
    U = [[one if r == c else zero for c in range(3)] for r in range(3)]
    V = [[one if r == c else zero for c in range(3)] for r in range(3)]
    if not np.isfinite(scale):
        return np.array(U, F32), np.zeros(3, F32), np.array(V, F32)
    if scale == zero:
        scale = one
    W = [[A[r][c] / scale for c in range(3)] for r in range(3)]
    maxd = zero
    for i in range(3):
        maxd = abs(W[i][i]) if maxd < abs(W[i][i]) else maxd
    finished = False
    while not finished:
        finished = True
        for p in (1, 2):
            for q in range(p):
                pm = precision * maxd
                thr = pm if fmin < pm else fmin
                if abs(W[p][q]) > thr or abs(W[q][p]) > thr:
                    finished = False
                    # real_2x2_jacobi_svd
                    m = [[W[p][p], W[p][q]], [W[q][p], W[q][q]]]
                    t = m[0][0] + m[1][1]
                    d = m[1][0] - m[0][1]
                    if abs(d) < fmin:
                        c1, s1 = one, zero
                    else:
                        u = t / d
                        tmp = np.sqrt(one + u * u)
                        s1 = one / tmp
                        c1 = u / tmp
                    r0, r1 = [m[0][0], m[0][1]], [m[1][0], m[1][1]]
                    _plane(r0, r1, c1, s1)
                    m = [r0, r1]
                    x, y, z = m[0][0], m[0][1], m[1][1]
                    deno = F32(2) * abs(y)
                    if deno < fmin:
                        cr, sr = one, zero
                    else:
                        tau = (x - z) / deno
                        w = np.sqrt(tau * tau + one)
                        tt = one / (tau + w) if tau > zero else one / (tau - w)
                        sign_t = one if tt > zero else -one
                        n = one / np.sqrt(tt * tt + one)
                        sr = -sign_t * (y / abs(y)) * abs(tt) * n
                        cr = n
                    c2, s2 = cr, -sr
                    cl = c1 * c2 - s1 * s2
                    sl = c1 * s2 + s1 * c2
                    # W rows p, q (left); U cols (right, j_left^T^T); W, V cols (right, j_right^T)
                    _plane(W[p], W[q], cl, sl)
                    for M, c, s in ((U, cl, sl), (W, cr, -sr), (V, cr, -sr)):
                        cp, cq = [M[k][p] for k in range(3)], [M[k][q] for k in range(3)]
                        _plane(cp, cq, c, s)
                        for k in range(3):
                            M[k][p], M[k][q] = cp[k], cq[k]
                    ap, aq = abs(W[p][p]), abs(W[q][q])
                    mpq = aq if ap < aq else ap
                    maxd = mpq if maxd < mpq else maxd
    S = [zero, zero, zero]
    for i in range(3):
        a = W[i][i]
        S[i] = abs(a)
        if a < zero:
            for k in range(3):
                U[k][i] = -U[k][i]
    S = [s * scale for s in S]
    for i in range(3):
        pos, mx = i, S[i]
        for k in range(i + 1, 3):
            if S[k] > mx:
                pos, mx = k, S[k]
        if mx == zero:
            break
        if pos != i:
            S[i], S[pos] = S[pos], S[i]
            for k in range(3):
                U[k][i], U[k][pos] = U[k][pos], U[k][i]
                V[k][i], V[k][pos] = V[k][pos], V[k][i]
    return np.array(U, F32), np.array(S, F32), np.array(V, F32)


def _det3_f32(M):
    """Eigen's bruteforce 3x3 determinant, float32."""
    return (M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) - M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0])
            + M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]))


def umeyama_rotation_f32(sigma):
    """Eigen::umeyama's rotation, Scalar = float: R = U diag(1, 1, +-1) V^T, each coefficient
    x0 + (x1 + x2) (the lazy product's unrolled redux), x_k = (U[i][k] * S_k) * V[j][k]."""
    U, _, V = eigen_jacobi_svd3_f32(sigma)
    Sd = [F32(1), F32(1), F32(1)]
    if _det3_f32(U) * _det3_f32(V) < F32(0):
        Sd[2] = F32(-1)
    R = np.empty((3, 3), F32)
    for i in range(3):
        for j in range(3):
            x = [(U[i, k] * Sd[k]) * V[j, k] for k in range(3)]
            R[i, j] = x[0] + (x[1] + x[2])
    return R


def umeyama_f32(s: np.ndarray, d: np.ndarray, kc: int | None = None) -> np.ndarray:
    """pcl::umeyama (= Eigen::umeyama, no scaling) in float: T = [R | mu_d - R mu_s] as Matrix4f;
    t_i = mu_d_i - ((R_i0 mu_s_0 + R_i1 mu_s_1) + R_i2 mu_s_2) (a dynamic-size block times a vector:
    the sequential redux)."""
    sigma, ms, md = umeyama_sigma_f32(s, d, kc)
    R = umeyama_rotation_f32(sigma)
    T = np.eye(4, dtype=F32)
    T[:3, :3] = R
    for i in range(3):
        rs = R[i, 0] * ms[0]
        rs = R[i, 1] * ms[1] + rs
        rs = R[i, 2] * ms[2] + rs
        T[i, 3] = md[i] - rs
    return T, sigma, ms, md


def pcl_converged_transform(Tinc) -> tuple[float, float]:
    """DefaultConvergenceCriteria's cos_angle and translation_sqr: float expressions over the
    Matrix4f increment, widened to double only at the end."""
    T = np.asarray(Tinc, F32)
    tr = T[0, 0] + T[1, 1] + T[2, 2] - F32(1)
    tsq = T[0, 3] * T[0, 3] + T[1, 3] * T[1, 3] + T[2, 3] * T[2, 3]
    return 0.5 * float(tr), float(tsq)


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


def _seq_sum_f64(v: np.ndarray) -> float:
    """A sequential double sum of float terms (PCL's calculateMSE / getFitnessScore loops)."""
    v = np.asarray(v, np.float64)
    return float(np.cumsum(v)[-1]) if len(v) else 0.0


def icp(src: np.ndarray, tgt: np.ndarray, max_iterations: int = 10, mse_abs: float = 1e-12,
        max_dist: float = np.sqrt(np.finfo(np.float64).max), numerics: str = "f64"):
    """PCL default ICP.  numerics "f64": the Umeyama solve in float64 (the golden fixtures' form);
    "f32": PCL's own float path end to end (float centroids, Eigen's blocked sigma GEMM, Eigen's
    JacobiSVD<Matrix3f>, float R and t; sequential double MSE and fitness sums).
    Returns dict(T, iterations, converged, fitness, trace)."""
    if numerics == "f32":
        return _icp_f32(src, tgt, max_iterations, mse_abs, max_dist)
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
        cos_a, tsq = pcl_converged_transform(Tinc)
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


def _icp_f32(src, tgt, max_iterations, mse_abs, max_dist):
    src = np.asarray(src, F32)[:, :3]
    tgt = np.asarray(tgt, F32)[:, :3]
    X = src.copy()
    final = np.eye(4, dtype=F32)
    prev_mse = np.finfo(np.float64).max
    max_d2 = max_dist * max_dist
    it, trace, converged, state = 0, [], False, 0
    while True:
        idx, d2 = nearest(X, tgt)
        keep = d2.astype(np.float64) <= max_d2
        nk = int(keep.sum())
        if nk < 3:
            converged, state = False, 5
            break
        Tinc, sigma, ms, md = umeyama_f32(X[keep], tgt[idx[keep]])
        X = transform(Tinc, X)
        final = mat4_mul_f32(Tinc, final)
        it += 1
        mse = _seq_sum_f64(d2[keep]) / nk
        trace.append({"T_inc": Tinc, "T_final": final.copy(), "mse": mse, "ncorr": nk, "sigma": sigma,
                      "mu_src": ms, "mu_dst": md})
        if it >= max_iterations:
            converged, state = True, 1
            break
        cos_a, tsq = pcl_converged_transform(Tinc)
        if cos_a >= 1.0 and tsq <= 0.0:
            converged, state = True, 2
            break
        if abs(mse - prev_mse) < mse_abs:
            converged, state = True, 3
            break
        prev_mse = mse
    Y = transform(final, src)
    _, fd = nearest(Y, tgt)
    fitness = _seq_sum_f64(fd) / len(fd) if len(fd) else np.finfo(np.float64).max
    return {"T": final, "iterations": it, "converged": converged, "state": state, "fitness": fitness,
            "trace": trace}
