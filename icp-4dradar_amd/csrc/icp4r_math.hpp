// icp4r_math.hpp — device arithmetic of one ICP iteration (PCL 1.8.1 semantics).
//
// Every float expression follows the operation order of the upstream code and is compiled with
// -ffp-contract=off (the reference's x86-64 SSE build never fuses):
//   * L2_Simple<float> distance  (FLANN, used by pcl::KdTreeFLANN):  ((dx*dx + dy*dy) + dz*dz)
//   * transformCloud             (icp.hpp, Eigen lazy packet product): ((r0*x + r1*y) + r2*z) + t
//   * final = T_inc * final      (Matrix4f * Matrix4f, k-ordered)
//   * the rigid solve: Eigen umeyama (with_scaling = false) over JacobiSVD<Matrix3f>, in float
//     (PCL numerics, the default), or the product's own double solve (F64 numerics).
#pragma once

#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace icp4r {

// ---- distance & transforms (float, unfused) ------------------------------------------------
__device__ __forceinline__ float l2_simple(float qx, float qy, float qz, float tx, float ty, float tz) {
    float d0 = qx - tx;
    float r = d0 * d0;
    float d1 = qy - ty;
    r = r + d1 * d1;
    float d2 = qz - tz;
    r = r + d2 * d2;
    return r;
}

// ---- the depth blocking of umeyama's sigma GEMM (Eigen 3.3; oracle/icp_oracle.c umeyama_f32) ----
// pcl::umeyama's sigma = one_over_n * dst_demean * src_demean^T is an Eigen GEMM of depth |C|: the
// depth is cut into panels of kc (evaluateProductBlockingSizesHeuristic), and gebp's scalar tail path
// (3 rows < LhsProgress, 3 columns < nr) forms each coefficient of a panel as a sequential chain
// C0 = a*b + C0 from 0, then res += alpha * C0 panel by panel (DESIGN.md §2 has the derivation).
// sigma_max_kc: the largest panel depth for the reference host's L1d size and gebp mr (KcFactor 1,
// nr 4, float, k_peeling 8); l1 < 0: no blocking.
__host__ __device__ inline int32_t sigma_max_kc(int32_t l1, int32_t mr) {
    if (l1 < 0) return INT32_MAX;
    if (l1 == 0) l1 = 32768;
    if (mr <= 0) mr = 8;
    const int32_t k_div = mr * 4 + 4 * 4, k_sub = mr * 4 * 4;
    const int32_t mkc = ((l1 - k_sub) / k_div) & ~7;
    return mkc < 1 ? 1 : mkc;
}
// the panel depth Eigen picks for a depth of k: the same number of panels as max_kc would give, the
// last one as large as possible (k <= max_kc, or k < 48: one panel)
__host__ __device__ inline int32_t sigma_kc(int32_t k, int32_t max_kc) {
    if (max_kc <= 0 || k < 48 || k <= max_kc) return k;
    const int32_t r = k % max_kc;
    return r == 0 ? max_kc : max_kc - 8 * ((max_kc - 1 - r) / (8 * (k / max_kc + 1)));
}

// T: column-major 4x4 float (12 used entries: T[c*4 + r])
__device__ __forceinline__ void xform_pt(const float* T, float x, float y, float z, float& ox, float& oy,
                                         float& oz) {
    float a0 = T[0] * x;
    a0 = T[4] * y + a0;
    a0 = T[8] * z + a0;
    a0 = T[12] + a0;
    float a1 = T[1] * x;
    a1 = T[5] * y + a1;
    a1 = T[9] * z + a1;
    a1 = T[13] + a1;
    float a2 = T[2] * x;
    a2 = T[6] * y + a2;
    a2 = T[10] * z + a2;
    a2 = T[14] + a2;
    ox = a0;
    oy = a1;
    oz = a2;
}

__device__ __forceinline__ void mat4_mul_f(const float* A, const float* B, float* C) {
    float R[16];
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) {
            float acc = A[0 * 4 + i] * B[j * 4 + 0];
            acc = A[1 * 4 + i] * B[j * 4 + 1] + acc;
            acc = A[2 * 4 + i] * B[j * 4 + 2] + acc;
            acc = A[3 * 4 + i] * B[j * 4 + 3] + acc;
            R[j * 4 + i] = acc;
        }
    for (int k = 0; k < 16; ++k) C[k] = R[k];
}

__device__ __forceinline__ void mat4_identity(float* T) {
    for (int k = 0; k < 16; ++k) T[k] = (k % 5 == 0) ? 1.0f : 0.0f;
}

// ---- 3x3 SVD, one-sided (Hestenes) Jacobi in double --------------------------------------
// Singular values sorted descending (Eigen::JacobiSVD order); U completed for rank < 3.  For a
// rank >= 2 cross-covariance the Umeyama rotation U*diag(1,1,s)*V^T is unique, so this returns
// PCL's R up to rounding (oracle/icp_oracle.c svd3_f64 is the same algorithm).
// Runs in ONE thread with its working set in LDS (SvdWork): kept out of VGPRs so the serial solve
// does not inflate the register allocation of the whole persistent kernel.
struct SvdWork {
    double W[9], V[9], U[9], S[3], Vs[9], Ws[9], R[9];
    int ord[3];
};

__device__ inline void svd3(const double* A, SvdWork& w) {
    double* W = w.W;
    double* V = w.V;
    double* U = w.U;
    double* S = w.S;
    for (int k = 0; k < 9; ++k) W[k] = A[k];
    for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0) ? 1.0 : 0.0;
#pragma nounroll
    for (int sweep = 0; sweep < 40; ++sweep) {
        double off = 0;
#pragma nounroll
        for (int r = 0; r < 3; ++r) {
            const int p = r == 2 ? 1 : 0, q = r == 0 ? 1 : 2;
            double al = 0, be = 0, ga = 0;
            for (int k = 0; k < 3; ++k) {
                al += W[k * 3 + p] * W[k * 3 + p];
                be += W[k * 3 + q] * W[k * 3 + q];
                ga += W[k * 3 + p] * W[k * 3 + q];
            }
            if (ga == 0) continue;
            double nrm = sqrt(al * be);
            if (nrm == 0) continue;
            double rel = fabs(ga) / nrm;
            if (rel > off) off = rel;
            if (rel <= 1e-15) continue;
            double zeta = (be - al) / (2 * ga);
            double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
            double c = 1.0 / sqrt(1.0 + t * t);
            double s = c * t;
            for (int k = 0; k < 3; ++k) {
                double wp = W[k * 3 + p], wq = W[k * 3 + q];
                W[k * 3 + p] = c * wp - s * wq;
                W[k * 3 + q] = s * wp + c * wq;
                double vp = V[k * 3 + p], vq = V[k * 3 + q];
                V[k * 3 + p] = c * vp - s * vq;
                V[k * 3 + q] = s * vp + c * vq;
            }
        }
        if (off <= 1e-15) break;
    }
    int* ord = w.ord;
    for (int c = 0; c < 3; ++c) {
        w.S[c] = sqrt(W[0 * 3 + c] * W[0 * 3 + c] + W[1 * 3 + c] * W[1 * 3 + c] + W[2 * 3 + c] * W[2 * 3 + c]);
        ord[c] = c;
    }
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (S[ord[j]] > S[ord[i]]) {
                int tt = ord[i];
                ord[i] = ord[j];
                ord[j] = tt;
            }
    for (int c = 0; c < 3; ++c)
        for (int k = 0; k < 3; ++k) {
            w.Vs[k * 3 + c] = V[k * 3 + ord[c]];
            w.Ws[k * 3 + c] = W[k * 3 + ord[c]];
        }
    double sv[3] = {S[ord[0]], S[ord[1]], S[ord[2]]};
    for (int c = 0; c < 3; ++c) S[c] = sv[c];
    for (int k = 0; k < 9; ++k) V[k] = w.Vs[k];
    int rank = 0;
    for (int c = 0; c < 3; ++c)
        if (S[c] > 1e-12 * (S[0] > 0 ? S[0] : 1.0) && S[c] > 0) rank = c + 1;
    for (int c = 0; c < rank; ++c)
        for (int k = 0; k < 3; ++k) U[k * 3 + c] = w.Ws[k * 3 + c] / S[c];
    if (rank == 0) {
        for (int k = 0; k < 9; ++k) U[k] = (k % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    if (rank == 1) {
        int ax = 0;
        double amin = fabs(U[0]);
        for (int k = 1; k < 3; ++k)
            if (fabs(U[k * 3]) < amin) {
                amin = fabs(U[k * 3]);
                ax = k;
            }
        const double e0 = ax == 0 ? 1.0 : 0.0, e1 = ax == 1 ? 1.0 : 0.0, e2 = ax == 2 ? 1.0 : 0.0;
        double c0 = U[1 * 3] * e2 - U[2 * 3] * e1;
        double c1 = U[2 * 3] * e0 - U[0 * 3] * e2;
        double c2 = U[0 * 3] * e1 - U[1 * 3] * e0;
        double nn = sqrt(c0 * c0 + c1 * c1 + c2 * c2);
        U[0 * 3 + 1] = c0 / nn;
        U[1 * 3 + 1] = c1 / nn;
        U[2 * 3 + 1] = c2 / nn;
    }
    if (rank <= 2) {  // complete U only when sigma is rank-deficient
        U[0 * 3 + 2] = U[1 * 3 + 0] * U[2 * 3 + 1] - U[2 * 3 + 0] * U[1 * 3 + 1];
        U[1 * 3 + 2] = U[2 * 3 + 0] * U[0 * 3 + 1] - U[0 * 3 + 0] * U[2 * 3 + 1];
        U[2 * 3 + 2] = U[0 * 3 + 0] * U[1 * 3 + 1] - U[1 * 3 + 0] * U[0 * 3 + 1];
    }
}

__device__ inline double det3(const double* M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// Eigen 3.3 umeyama: R = U * diag(1, 1, s) * V^T, s = -1 iff det(U) * det(V) < 0.  Result in w.R.
__device__ inline void umeyama_rotation(const double* sigma, SvdWork& w) {
    svd3(sigma, w);
    const double d2 = (det3(w.U) * det3(w.V) < 0) ? -1.0 : 1.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            w.R[i * 3 + j] = w.U[i * 3 + 0] * w.V[j * 3 + 0] + w.U[i * 3 + 1] * w.V[j * 3 + 1] + d2 * w.U[i * 3 + 2] * w.V[j * 3 + 2];
}

// ---- PCL's float rotation: Eigen 3.3 JacobiSVD<Matrix3f> + umeyama (PCL numerics) -----------
// pcl::umeyama -> Eigen::umeyama (Geometry/Umeyama.h, with_scaling = false), Scalar = float:
//   JacobiSVD<Matrix3f> svd(sigma, ComputeFullU | ComputeFullV)       (SVD/JacobiSVD.h compute())
//   S = (1, 1, 1); if (det(U) * det(V) < 0) S(2) = -1;  R = U * S.asDiagonal() * V^T
// Square input: no QR preconditioner.  The matrix is divided by its largest |coefficient|; two-sided
// 2x2 Jacobi steps over (p, q) = (1, 0), (2, 0), (2, 1) repeat until no off-diagonal pair exceeds
// max(FLT_MIN, 2 eps * the largest |diagonal| seen).  A step is real_2x2_jacobi_svd
// (misc/RealSvd2x2.h: a rotation symmetrising the 2x2 block, then JacobiRotation::makeJacobi,
// j_left = rot1 * j_right^T) applied to the work matrix's rows (j_left) and columns (j_right) and
// accumulated into U's and V's columns; apply_rotation_in_the_plane is x' = c x + s y,
// y' = -s x + c y, a no-op for (c, s) = (1, 0).  Then a negative diagonal entry flips U's column,
// the singular values are scaled back and sorted by swaps (the first maximum; a zero maximum stops
// the sort).  R's coefficients: the lazy product's unrolled redux, x0 + (x1 + x2), with
// x_k = (U(i,k) * S(k)) * V(j,k).  Every operation in float, unfused, in this order: the same bits
// as oracle/icp_oracle.c rot_f32 and tests/golden/numpy_twin.py umeyama_rotation_f32.  Static
// indices only, so the whole working set stays in registers (thread 0's serial solve).
// float '/' and sqrtf are correctly rounded on the device (HIP default), like SSE on the host.
__host__ __device__ __forceinline__ void plane_rot3(float& x0, float& x1, float& x2, float& y0, float& y1, float& y2,
                                                    float c, float s) {
    if (c == 1.0f && s == 0.0f) return;
    float xi = x0, yi = y0;
    x0 = c * xi + s * yi;
    y0 = -s * xi + c * yi;
    xi = x1, yi = y1;
    x1 = c * xi + s * yi;
    y1 = -s * xi + c * yi;
    xi = x2, yi = y2;
    x2 = c * xi + s * yi;
    y2 = -s * xi + c * yi;
}

// real_2x2_jacobi_svd of the block (p, q) = [[a, b], [e, f]] = [[W(p,p), W(p,q)], [W(q,p), W(q,q)]]
__host__ __device__ __forceinline__ void real_2x2_jacobi_f32(float a, float b, float e, float f, float& cl, float& sl,
                                                             float& cr, float& sr) {
    float c1, s1;
    const float t = a + f;
    const float d = e - b;
    if (fabsf(d) < FLT_MIN) {
        s1 = 0.0f;
        c1 = 1.0f;
    } else {
        const float u = t / d;
        const float tmp = sqrtf(1.0f + u * u);
        s1 = 1.0f / tmp;
        c1 = u / tmp;
    }
    if (!(c1 == 1.0f && s1 == 0.0f)) {  // m.applyOnTheLeft(0, 1, rot1)
        const float x0 = a, y0 = e, x1 = b, y1 = f;
        a = c1 * x0 + s1 * y0;
        e = -s1 * x0 + c1 * y0;
        b = c1 * x1 + s1 * y1;
        f = -s1 * x1 + c1 * y1;
    }
    const float deno = 2.0f * fabsf(b);  // makeJacobi(m(0,0), m(0,1), m(1,1))
    if (deno < FLT_MIN) {
        cr = 1.0f;
        sr = 0.0f;
    } else {
        const float tau = (a - f) / deno;
        const float w = sqrtf(tau * tau + 1.0f);
        float tt;
        if (tau > 0.0f)
            tt = 1.0f / (tau + w);
        else
            tt = 1.0f / (tau - w);
        const float sign_t = tt > 0.0f ? 1.0f : -1.0f;
        const float n = 1.0f / sqrtf(tt * tt + 1.0f);
        sr = -sign_t * (b / fabsf(b)) * fabsf(tt) * n;
        cr = n;
    }
    const float c2 = cr, s2 = -sr;  // j_left = rot1 * j_right^T
    cl = c1 * c2 - s1 * s2;
    sl = c1 * s2 + s1 * c2;
}

__host__ __device__ __forceinline__ float det3_f32(const float (&M)[9]) {  // LU/Determinant.h, row-major M
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// One Jacobi step on the pair (P, Q) (P > Q) of W, U, V (row-major): returns whether it ran.
template <int P, int Q>
__host__ __device__ __forceinline__ bool jacobi_step_f32(float (&W)[9], float (&U)[9], float (&V)[9], float& max_diag) {
    const float pm = (2.0f * FLT_EPSILON) * max_diag;
    const float threshold = FLT_MIN < pm ? pm : FLT_MIN;
    if (!(fabsf(W[P * 3 + Q]) > threshold || fabsf(W[Q * 3 + P]) > threshold)) return false;
    float cl, sl, cr, sr;
    real_2x2_jacobi_f32(W[P * 3 + P], W[P * 3 + Q], W[Q * 3 + P], W[Q * 3 + Q], cl, sl, cr, sr);
    plane_rot3(W[P * 3 + 0], W[P * 3 + 1], W[P * 3 + 2], W[Q * 3 + 0], W[Q * 3 + 1], W[Q * 3 + 2], cl, sl);  // rows
    plane_rot3(U[0 * 3 + P], U[1 * 3 + P], U[2 * 3 + P], U[0 * 3 + Q], U[1 * 3 + Q], U[2 * 3 + Q], cl, sl);  // cols
    plane_rot3(W[0 * 3 + P], W[1 * 3 + P], W[2 * 3 + P], W[0 * 3 + Q], W[1 * 3 + Q], W[2 * 3 + Q], cr, -sr);
    plane_rot3(V[0 * 3 + P], V[1 * 3 + P], V[2 * 3 + P], V[0 * 3 + Q], V[1 * 3 + Q], V[2 * 3 + Q], cr, -sr);
    const float ap = fabsf(W[P * 3 + P]), aq = fabsf(W[Q * 3 + Q]);
    const float mpq = ap < aq ? aq : ap;
    max_diag = max_diag < mpq ? mpq : max_diag;
    return true;
}

template <int I, int J>
__host__ __device__ __forceinline__ void svd_swap_f32(float (&S)[3], float (&U)[9], float (&V)[9]) {
    float t = S[I];
    S[I] = S[J];
    S[J] = t;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        t = U[k * 3 + I];
        U[k * 3 + I] = U[k * 3 + J];
        U[k * 3 + J] = t;
        t = V[k * 3 + I];
        V[k * 3 + I] = V[k * 3 + J];
        V[k * 3 + J] = t;
    }
}

// JacobiSVD<Matrix3f>(A, ComputeFullU | ComputeFullV); A, U, V row-major.  Returns false (U = V = I,
// S = 0) for a non-finite A (Eigen: InvalidInput).
__host__ __device__ __forceinline__ bool eigen_jacobi_svd3_f32(const float (&A)[9], float (&U)[9], float (&S)[3], float (&V)[9]) {
    float scale = fabsf(A[0]);
#pragma unroll
    for (int k = 1; k < 9; ++k) scale = scale < fabsf(A[k]) ? fabsf(A[k]) : scale;
#pragma unroll
    for (int k = 0; k < 9; ++k) U[k] = V[k] = (k % 4 == 0) ? 1.0f : 0.0f;
    S[0] = S[1] = S[2] = 0.0f;
    if (!(scale <= FLT_MAX)) return false;  // !isfinite (scale >= 0 or NaN)
    if (scale == 0.0f) scale = 1.0f;
    float W[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) W[k] = A[k] / scale;
    float max_diag = fabsf(W[0]);
    max_diag = max_diag < fabsf(W[4]) ? fabsf(W[4]) : max_diag;
    max_diag = max_diag < fabsf(W[8]) ? fabsf(W[8]) : max_diag;
    bool finished = false;
#pragma nounroll
    while (!finished) {
        const bool a = jacobi_step_f32<1, 0>(W, U, V, max_diag);
        const bool b = jacobi_step_f32<2, 0>(W, U, V, max_diag);
        const bool c = jacobi_step_f32<2, 1>(W, U, V, max_diag);
        finished = !(a || b || c);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float a = W[i * 3 + i];
        S[i] = fabsf(a);
        if (a < 0.0f) {
#pragma unroll
            for (int k = 0; k < 3; ++k) U[k * 3 + i] = -U[k * 3 + i];
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) S[i] *= scale;
    // the sort: for i = 0, 1 the first maximum of S[i..2] swapped to i; a zero maximum stops it
    int pos = 0;
    float mx = S[0];
    if (S[1] > mx) { mx = S[1]; pos = 1; }
    if (S[2] > mx) { mx = S[2]; pos = 2; }
    if (mx == 0.0f) return true;
    if (pos == 1) svd_swap_f32<0, 1>(S, U, V);
    if (pos == 2) svd_swap_f32<0, 2>(S, U, V);
    if (S[2] > S[1]) svd_swap_f32<1, 2>(S, U, V);  // (both zero: the sort stops, nothing to swap)
    return true;
}

// Eigen::umeyama's rotation (with_scaling = false), Scalar = float; sigma and R row-major.
__host__ __device__ __forceinline__ void umeyama_rotation_f32_reg(const float (&A)[9], float (&R)[9]) {
    float U[9], S[3], V[9];
    eigen_jacobi_svd3_f32(A, U, S, V);
    float d2 = 1.0f;
    if (det3_f32(U) * det3_f32(V) < 0) d2 = -1.0f;
    const float d[3] = {1.0f, 1.0f, d2};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float x0 = (U[i * 3 + 0] * d[0]) * V[j * 3 + 0];
            const float x1 = (U[i * 3 + 1] * d[1]) * V[j * 3 + 1];
            const float x2 = (U[i * 3 + 2] * d[2]) * V[j * 3 + 2];
            R[i * 3 + j] = x0 + (x1 + x2);
        }
}

// ---- convergence: DefaultConvergenceCriteria<float>::hasConverged ------------------------------
struct ConvParams {
    int32_t max_iterations;
    int32_t max_similar;
    double rot_thr;    // transformation_rotation_epsilon > 0 ? it : 1 - transformation_epsilon
    double trans_thr;  // transformation_epsilon (compared with the squared translation, as PCL)
    double abs_mse;    // mse_threshold_absolute
    double rel_mse;    // euclidean_fitness_epsilon
};

struct ConvState {
    double prev_mse;
    int32_t similar;
    int32_t state;
};

// returns 1 when converged; updates prev_mse only on the no-criterion path (upstream early returns)
__device__ __forceinline__ int has_converged(const ConvParams& p, int32_t iterations, const float* Tinc, double mse,
                                    ConvState& cs) {
    cs.state = 0;
    if (iterations >= p.max_iterations) {
        cs.state = 1;  // CONVERGENCE_CRITERIA_ITERATIONS
        return 1;
    }
    // transformation_ is the ICP's Matrix4f: both expressions in float, only the results widened
    const float tr = Tinc[0] + Tinc[5] + Tinc[10] - 1;
    const double cos_angle = 0.5 * tr;
    const float tsqf = Tinc[12] * Tinc[12] + Tinc[13] * Tinc[13] + Tinc[14] * Tinc[14];
    const double tsq = tsqf;
    if (cos_angle >= p.rot_thr && tsq <= p.trans_thr) {
        if (cs.similar < p.max_similar) {
            ++cs.similar;
            return 0;
        }
        cs.similar = 0;
        cs.state = 2;  // TRANSFORM
        return 1;
    }
    if (fabs(mse - cs.prev_mse) < p.abs_mse) {
        if (cs.similar < p.max_similar) {
            ++cs.similar;
            return 0;
        }
        cs.similar = 0;
        cs.state = 3;  // ABS_MSE
        return 1;
    }
    if (fabs(mse - cs.prev_mse) / cs.prev_mse < p.rel_mse) {
        if (cs.similar < p.max_similar) {
            ++cs.similar;
            return 0;
        }
        cs.similar = 0;
        cs.state = 4;  // REL_MSE
        return 1;
    }
    cs.prev_mse = mse;
    return 0;
}

}  // namespace icp4r
