// icp4r_math.hpp — device arithmetic of one ICP iteration (PCL 1.8.1 semantics).
//
// Every float expression follows the operation order of the upstream code and is compiled with
// -ffp-contract=off (the reference's x86-64 SSE build never fuses):
//   * L2_Simple<float> distance  (FLANN, used by pcl::KdTreeFLANN):  ((dx*dx + dy*dy) + dz*dz)
//   * transformCloud             (icp.hpp, Eigen lazy packet product): ((r0*x + r1*y) + r2*z) + t
//   * final = T_inc * final      (Matrix4f * Matrix4f, k-ordered)
// The rigid solve (Eigen umeyama, with_scaling = false) runs in double here; DESIGN.md §Numerics
// explains why that stays within the parity bar of PCL's float solve.
#pragma once

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

__device__ inline void mat4_mul_f(const float* A, const float* B, float* C) {
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

__device__ inline void mat4_identity(float* T) {
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

// ---- 3x3 SVD + Umeyama rotation in FLOAT (PCL numerics) -------------------------------------
// Same one-sided Jacobi as svd3() with every operation in float and in the operation order of
// oracle/icp_oracle.c svd3_f32 / rot_f32 / det3_f32, so the rotation the PCL-numerics path produces
// is bit-identical to the float restatement of PCL's TransformationEstimationSVD (Scalar = float).
// float '/' and sqrtf are correctly rounded on the device (HIP default), like SSE on the host.
struct SvdWorkF {
    float W[9], V[9], U[9], S[3], Vs[9], Ws[9], R[9];
    int ord[3];
};

__host__ __device__ inline void svd3_f32(const float* A, SvdWorkF& w) {
    float* W = w.W;
    float* V = w.V;
    float* U = w.U;
    float* S = w.S;
    for (int k = 0; k < 9; ++k) W[k] = A[k];
    for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0) ? 1.0f : 0.0f;
#pragma nounroll
    for (int sweep = 0; sweep < 40; ++sweep) {
        float off = 0;
#pragma nounroll
        for (int r = 0; r < 3; ++r) {
            const int p = r == 2 ? 1 : 0, q = r == 0 ? 1 : 2;
            float al = 0, be = 0, ga = 0;
            for (int k = 0; k < 3; ++k) {
                al += W[k * 3 + p] * W[k * 3 + p];
                be += W[k * 3 + q] * W[k * 3 + q];
                ga += W[k * 3 + p] * W[k * 3 + q];
            }
            if (ga == 0) continue;
            float nrm = sqrtf(al * be);
            if (nrm == 0) continue;
            float rel = fabsf(ga) / nrm;
            if (rel > off) off = rel;
            if (rel <= 1e-7f) continue;
            float zeta = (be - al) / (2 * ga);
            float t = (zeta >= 0 ? 1.0f : -1.0f) / (fabsf(zeta) + sqrtf(1.0f + zeta * zeta));
            float c = 1.0f / sqrtf(1.0f + t * t);
            float s = c * t;
            for (int k = 0; k < 3; ++k) {
                float wp = W[k * 3 + p], wq = W[k * 3 + q];
                W[k * 3 + p] = c * wp - s * wq;
                W[k * 3 + q] = s * wp + c * wq;
                float vp = V[k * 3 + p], vq = V[k * 3 + q];
                V[k * 3 + p] = c * vp - s * vq;
                V[k * 3 + q] = s * vp + c * vq;
            }
        }
        if (off <= 1e-7f) break;
    }
    float sv[3];
    for (int c = 0; c < 3; ++c)
        sv[c] = sqrtf(W[0 * 3 + c] * W[0 * 3 + c] + W[1 * 3 + c] * W[1 * 3 + c] + W[2 * 3 + c] * W[2 * 3 + c]);
    int* ord = w.ord;
    for (int c = 0; c < 3; ++c) ord[c] = c;
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (sv[ord[j]] > sv[ord[i]]) {
                int tt = ord[i];
                ord[i] = ord[j];
                ord[j] = tt;
            }
    for (int c = 0; c < 3; ++c) {
        S[c] = sv[ord[c]];
        for (int k = 0; k < 3; ++k) {
            w.Vs[k * 3 + c] = V[k * 3 + ord[c]];
            w.Ws[k * 3 + c] = W[k * 3 + ord[c]];
        }
    }
    for (int k = 0; k < 9; ++k) V[k] = w.Vs[k];
    int rank = 0;
    for (int c = 0; c < 3; ++c)
        if (S[c] > 1e-6f * (S[0] > 0 ? S[0] : 1.0f) && S[c] > 0) rank = c + 1;
    for (int c = 0; c < rank; ++c)
        for (int k = 0; k < 3; ++k) U[k * 3 + c] = w.Ws[k * 3 + c] / S[c];
    if (rank == 0) {
        for (int k = 0; k < 9; ++k) U[k] = (k % 4 == 0) ? 1.0f : 0.0f;
        return;
    }
    if (rank == 1) {
        int ax = 0;
        float amin = fabsf(U[0]);
        for (int k = 1; k < 3; ++k)
            if (fabsf(U[k * 3]) < amin) {
                amin = fabsf(U[k * 3]);
                ax = k;
            }
        const float e0 = ax == 0 ? 1.0f : 0.0f, e1 = ax == 1 ? 1.0f : 0.0f, e2 = ax == 2 ? 1.0f : 0.0f;
        float c0 = U[1 * 3] * e2 - U[2 * 3] * e1;
        float c1 = U[2 * 3] * e0 - U[0 * 3] * e2;
        float c2 = U[0 * 3] * e1 - U[1 * 3] * e0;
        float nn = sqrtf(c0 * c0 + c1 * c1 + c2 * c2);
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

__host__ __device__ inline float det3_f32(const float* M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

__host__ __device__ inline void umeyama_rotation_f32(const float* sigma, SvdWorkF& w) {
    svd3_f32(sigma, w);
    float d[3] = {1.0f, 1.0f, 1.0f};
    if (det3_f32(w.U) * det3_f32(w.V) < 0) d[2] = -1.0f;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            float acc = 0;
            for (int k = 0; k < 3; ++k) acc += w.U[i * 3 + k] * d[k] * w.V[j * 3 + k];
            w.R[i * 3 + j] = acc;
        }
}

// The same float SVD + Umeyama rotation as umeyama_rotation_f32, every operation in the same order,
// with all indices static so the arrays live in registers: on the device the LDS-resident work
// struct put a dependent LDS round trip on every access of thread 0's serial solve.
__host__ __device__ inline void umeyama_rotation_f32_reg(const float (&A)[9], float (&R)[9]) {
    float W[9], V[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) W[k] = A[k];
#pragma unroll
    for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0) ? 1.0f : 0.0f;
#pragma nounroll
    for (int sweep = 0; sweep < 40; ++sweep) {
        float off = 0;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int p = r == 2 ? 1 : 0, q = r == 0 ? 1 : 2;
            float al = 0, be = 0, ga = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                al += W[k * 3 + p] * W[k * 3 + p];
                be += W[k * 3 + q] * W[k * 3 + q];
                ga += W[k * 3 + p] * W[k * 3 + q];
            }
            if (ga == 0) continue;
            float nrm = sqrtf(al * be);
            if (nrm == 0) continue;
            float rel = fabsf(ga) / nrm;
            if (rel > off) off = rel;
            if (rel <= 1e-7f) continue;
            float zeta = (be - al) / (2 * ga);
            float t = (zeta >= 0 ? 1.0f : -1.0f) / (fabsf(zeta) + sqrtf(1.0f + zeta * zeta));
            float c = 1.0f / sqrtf(1.0f + t * t);
            float s = c * t;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                float wp = W[k * 3 + p], wq = W[k * 3 + q];
                W[k * 3 + p] = c * wp - s * wq;
                W[k * 3 + q] = s * wp + c * wq;
                float vp = V[k * 3 + p], vq = V[k * 3 + q];
                V[k * 3 + p] = c * vp - s * vq;
                V[k * 3 + q] = s * vp + c * vq;
            }
        }
        if (off <= 1e-7f) break;
    }
    float sv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
        sv[c] = sqrtf(W[0 * 3 + c] * W[0 * 3 + c] + W[1 * 3 + c] * W[1 * 3 + c] + W[2 * 3 + c] * W[2 * 3 + c]);
    // the column order by descending singular value: the same three compare-and-swaps, on registers
    int o0 = 0, o1 = 1, o2 = 2;
    auto svo = [&](int i) { return i == 0 ? sv[0] : (i == 1 ? sv[1] : sv[2]); };
    if (svo(o1) > svo(o0)) { const int tt = o0; o0 = o1; o1 = tt; }
    if (svo(o2) > svo(o0)) { const int tt = o0; o0 = o2; o2 = tt; }
    if (svo(o2) > svo(o1)) { const int tt = o1; o1 = o2; o2 = tt; }
    const int ord[3] = {o0, o1, o2};
    auto col = [&](const float (&M)[9], int k, int c) {  // M[k][c] for a runtime column c in 0..2
        return c == 0 ? M[k * 3 + 0] : (c == 1 ? M[k * 3 + 1] : M[k * 3 + 2]);
    };
    float S[3], Vs[9], Ws[9], U[9];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        S[c] = svo(ord[c]);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            Vs[k * 3 + c] = col(V, k, ord[c]);
            Ws[k * 3 + c] = col(W, k, ord[c]);
        }
    }
    int rank = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c)
        if (S[c] > 1e-6f * (S[0] > 0 ? S[0] : 1.0f) && S[c] > 0) rank = c + 1;
#pragma unroll
    for (int k = 0; k < 9; ++k) U[k] = 0.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c)
        if (c < rank)
#pragma unroll
            for (int k = 0; k < 3; ++k) U[k * 3 + c] = Ws[k * 3 + c] / S[c];
    if (rank == 0) {
#pragma unroll
        for (int k = 0; k < 9; ++k) U[k] = (k % 4 == 0) ? 1.0f : 0.0f;
    } else {
        if (rank == 1) {
            int ax = 0;
            float amin = fabsf(U[0]);
#pragma unroll
            for (int k = 1; k < 3; ++k)
                if (fabsf(U[k * 3]) < amin) {
                    amin = fabsf(U[k * 3]);
                    ax = k;
                }
            const float e0 = ax == 0 ? 1.0f : 0.0f, e1 = ax == 1 ? 1.0f : 0.0f, e2 = ax == 2 ? 1.0f : 0.0f;
            float c0 = U[1 * 3] * e2 - U[2 * 3] * e1;
            float c1 = U[2 * 3] * e0 - U[0 * 3] * e2;
            float c2 = U[0 * 3] * e1 - U[1 * 3] * e0;
            float nn = sqrtf(c0 * c0 + c1 * c1 + c2 * c2);
            U[0 * 3 + 1] = c0 / nn;
            U[1 * 3 + 1] = c1 / nn;
            U[2 * 3 + 1] = c2 / nn;
        }
        if (rank <= 2) {
            U[0 * 3 + 2] = U[1 * 3 + 0] * U[2 * 3 + 1] - U[2 * 3 + 0] * U[1 * 3 + 1];
            U[1 * 3 + 2] = U[2 * 3 + 0] * U[0 * 3 + 1] - U[0 * 3 + 0] * U[2 * 3 + 1];
            U[2 * 3 + 2] = U[0 * 3 + 0] * U[1 * 3 + 1] - U[1 * 3 + 0] * U[0 * 3 + 1];
        }
    }
    float d[3] = {1.0f, 1.0f, 1.0f};
    if (det3_f32(U) * det3_f32(Vs) < 0) d[2] = -1.0f;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            float acc = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) acc += U[i * 3 + k] * d[k] * Vs[j * 3 + k];
            R[i * 3 + j] = acc;
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
__device__ inline int has_converged(const ConvParams& p, int32_t iterations, const float* Tinc, double mse,
                                    ConvState& cs) {
    cs.state = 0;
    if (iterations >= p.max_iterations) {
        cs.state = 1;  // CONVERGENCE_CRITERIA_ITERATIONS
        return 1;
    }
    double cos_angle = 0.5 * ((double)Tinc[0] + (double)Tinc[5] + (double)Tinc[10] - 1);
    double tsq = (double)Tinc[12] * Tinc[12] + (double)Tinc[13] * Tinc[13] + (double)Tinc[14] * Tinc[14];
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
