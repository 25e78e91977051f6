// icp4r_ego.hip — radar ego-velocity kernels for gfx950 (include/icp4r/icp4r_ego.h).
//
// The reference node (src/iterative_closest_point.cpp) parses each scan into float features
// (:373-384), fits a two-point sine model v_r cos(beta) = A cos(arfa + b) by RANSAC with
// (int)(0.2 N) hypotheses, each scored against all N points (:85-128 — O(0.2 N²) double cos calls,
// the node's most expensive step), splits static from dynamic points (:391-407) and solves the
// normal equations for the ego velocity (:410-431).  Here:
//
//   ego_features_kernel  per point: the float features exactly as the node forms them, and the
//                        doubles the model needs (cos(beta) v_r, cos/sin(DEG2RAD(arfa)), DEG2RAD(arfa))
//   ego_ransac_kernel    grid (hypothesis tiles, point tiles, scans): one lane per hypothesis, the
//                        point tile staged in LDS and broadcast; integer inlier counts merged with
//                        atomicAdd (exact, order-free)
//   ego_select_kernel    one workgroup per scan: first strict maximum (the node's `score > bestScore`
//                        from 0), the winner's model recomputed, split, KᵀK / KᵀVr in double with a
//                        fixed-order reduction, Eigen's cofactor 3x3 inverse
//
// The inlier test evaluates A cos(a_j + b_h) as (A cos b_h) cos a_j - (A sin b_h) sin a_j with two
// FMAs (a_j per point, b_h per hypothesis): it differs from the direct form by a few ulp of double, so
// a score can differ only for a point whose |delta| lies within ~1e-14 of sigma — never observed
// (tests/test_ego.py compares every hypothesis score with the oracle's direct evaluation).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "icp4r/icp4r_ego.h"
#include "icp4r_internal.hpp"

namespace icp4r {

constexpr double kPiEgo = 3.14159265358979323846;  // glibc's M_PI (math.h), the reference's constant
constexpr double kDeg2Rad = 0.017453293;            // PCL 1.8 pcl_macros.h: DEG2RAD(x) ((x)*0.017453293)

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// iterative_closest_point.cpp:373-384: float sqrt of ((x*x + y*y) + z*z); float atan2 / asin,
// `* 180` in float, `/ M_PI` in double, stored as float.
__global__ __launch_bounds__(256) void ego_features_kernel(const float* __restrict__ rec, const int64_t* __restrict__ off,
                                                           const int32_t* __restrict__ cnt, int64_t stride,
                                                           float4* __restrict__ feat, double4* __restrict__ pd,
                                                           float4* __restrict__ xyzi) {
    const int s = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= cnt[s] || i >= stride) return;  // a count above the declared max_n is rejected in select
    const float* r = rec + 5 * (off[s] + i);
    const float x = r[0], y = r[1], z = r[2], in = r[3], vr = r[4];
    float q = x * x;
    q = q + y * y;
    q = q + z * z;
    const float distance = sqrtf(q);
    // atan2f / asinf as the correctly rounded float of the double function (ROCm's float versions are
    // within 2 ulp, glibc's within 1: this keeps the device within 1 ulp of the node's glibc values)
    const float at = (float)atan2((double)y, (double)x);
    const float as = (float)asin((double)(z / distance));
    const float arfa = (float)((double)(at * 180.0f) / kPiEgo);
    const float beta = (float)((double)(as * 180.0f) / kPiEgo);
    const int64_t o = (int64_t)s * stride + i;
    feat[o] = make_float4(distance, arfa, beta, vr);
    const double ar = (double)arfa * kDeg2Rad;
    pd[o] = make_double4(cos((double)beta * kDeg2Rad) * vr, cos(ar), sin(ar), ar);
    if (xyzi) xyzi[off[s] + i] = make_float4(x, y, z, in);
}

// The two-point model of hypothesis h (:98-108): A, b from points i1, i2 (float features, double math).
__device__ __forceinline__ void ego_model(const float4* f, int n, uint64_t seed, int h, double& A, double& b) {
    const float4 p1 = f[splitmix64(seed + 2 * (uint64_t)h) % (uint64_t)n];
    const float4 p2 = f[splitmix64(seed + 2 * (uint64_t)h + 1) % (uint64_t)n];
    // .y = arfa, .z = beta, .w = v_r
    const double k = (p1.w * cos((double)p1.z * kDeg2Rad)) / (p2.w * cos((double)p2.z * kDeg2Rad));
    b = atan((cos((double)p1.y * kDeg2Rad) - k * cos((double)p2.y * kDeg2Rad)) /
             (sin((double)p1.y * kDeg2Rad) - k * sin((double)p2.y * kDeg2Rad)));
    A = cos((double)p1.z * kDeg2Rad) * p1.w / cos(((double)p1.y * kDeg2Rad) + b);
}

__device__ __forceinline__ int ego_hyps(const EgoArgs& e, int n) {
    return e.iterations > 0 ? e.iterations : (int)(n * 0.2);
}

constexpr int kEgoWG = 256;   // threads per RANSAC workgroup
constexpr int kEgoPer = 4;    // hypotheses per thread (each LDS point read feeds 4 tests)
constexpr int kEgoHyp = kEgoWG * kEgoPer;  // hypotheses per workgroup
constexpr int kEgoPts = 512;  // points per workgroup tile

// Inlier test of point j against hypothesis h: |cbv_j - A cos(a_j + b)| < sigma with
// A cos(a_j + b) = (A cos b) cos a_j - (A sin b) sin a_j: two fused multiply-adds per test.
__global__ __launch_bounds__(kEgoWG) void ego_ransac_kernel(EgoArgs e) {
    __shared__ double sc[kEgoPts], sca[kEgoPts], ssa[kEgoPts];
    const int s = blockIdx.z;
    const int n = e.cnt[s];
    if (n > e.stride) return;
    const int H = ego_hyps(e, n);
    const int h0 = blockIdx.x * kEgoHyp, j0 = blockIdx.y * kEgoPts;
    if (n <= 0 || h0 >= H || j0 >= n) return;
    const int64_t base = (int64_t)s * e.stride;
    const int len = min(kEgoPts, n - j0);
    for (int k = threadIdx.x; k < len; k += kEgoWG) {
        const double4 v = e.pd[base + j0 + k];
        sc[k] = v.x;
        sca[k] = v.y;
        ssa[k] = v.z;
    }
    double acb[kEgoPer], asb[kEgoPer];
#pragma unroll
    for (int q = 0; q < kEgoPer; ++q) {
        const int h = h0 + threadIdx.x + q * kEgoWG;
        acb[q] = 0.0;
        asb[q] = 0.0;
        if (h < H) {
            double A, b;
            ego_model(e.feat + base, n, e.seed + ((uint64_t)s << 32), h, A, b);
            acb[q] = A * cos(b);
            asb[q] = A * sin(b);
        }
    }
    __syncthreads();
    int score[kEgoPer] = {};
    const double sigma = e.sigma;
    for (int k = 0; k < len; ++k) {
        const double c = sc[k], ca = sca[k], sa = ssa[k];
#pragma unroll
        for (int q = 0; q < kEgoPer; ++q) {
            const double delta = __builtin_fma(asb[q], sa, __builtin_fma(-acb[q], ca, c));
            score[q] += fabs(delta) < sigma ? 1 : 0;  // NaN models (a degenerate pair) never count
        }
    }
#pragma unroll
    for (int q = 0; q < kEgoPer; ++q) {
        const int h = h0 + threadIdx.x + q * kEgoWG;
        if (h < H && score[q]) atomicAdd(e.scores + (int64_t)s * e.max_h + h, score[q]);
    }
}

constexpr int kEgoSelWG = 256;

__global__ __launch_bounds__(kEgoSelWG) void ego_select_kernel(EgoArgs e) {
    __shared__ uint64_t skey[kEgoSelWG / 64];
    __shared__ int sidx[kEgoSelWG / 64];
    __shared__ double red[kEgoSelWG / 64][9];
    __shared__ double model[2];
    __shared__ int best_s, best_h;
    const int s = blockIdx.x;
    const bool too_big = e.cnt[s] > e.stride;  // above the batch's declared max_n: nothing computed
    const int n = too_big ? 0 : e.cnt[s];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int H = n > 0 ? ego_hyps(e, n) : 0;
    const int64_t base = (int64_t)s * e.stride;
    // first strict maximum over the hypotheses (the node keeps A, b only on score > bestScore, from
    // 0): the largest key (score << 32 | ~h) is the highest score at the lowest index
    uint64_t bk = 0;
    for (int h = tid; h < H; h += kEgoSelWG) {
        const uint32_t v = (uint32_t)e.scores[(int64_t)s * e.max_h + h];
        const uint64_t k = v ? (((uint64_t)v << 32) | (uint32_t)~(uint32_t)h) : 0ull;
        bk = k > bk ? k : bk;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(bk, off, 64);
        bk = o > bk ? o : bk;
    }
    if (lane == 0) skey[wave] = bk;
    __syncthreads();
    if (tid == 0) {
        uint64_t k = 0;
        for (int w = 0; w < kEgoSelWG / 64; ++w) k = skey[w] > k ? skey[w] : k;
        const int B = (int)(k >> 32), I = k ? (int)~(uint32_t)k : -1;
        best_s = B;
        best_h = I;
        double A = 0.0, b = 0.0;  // A_src = b_src = 0 in the node (:387-388)
        if (I >= 0) ego_model(e.feat + base, n, e.seed + ((uint64_t)s << 32), I, A, b);
        model[0] = A;
        model[1] = b;
    }
    __syncthreads();
    const double A = model[0], b = model[1];
    // split (:391-407) and the normal equations over the static points (:410-431)
    double m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // KᵀK (6 unique) , KᵀVr (3)
    int ns = 0;
    for (int i = tid; i < n; i += kEgoSelWG) {
        const double4 v = e.pd[base + i];
        const float4 f = e.feat[base + i];
        const double delta = v.x - A * cos(v.w + b);
        const bool stat = !(delta > e.dyn);
        if (e.mask) e.mask[e.off[s] + i] = stat ? 1 : 0;
        if (!stat) continue;
        ++ns;
        const double br = (double)f.z * kDeg2Rad;
        const double cbr = cos(br), sbr = sin(br);
        const double k0 = v.y * cbr, k1 = v.z * cbr, k2 = sbr;
        const double vr = (double)f.w;
        m[0] += k0 * k0; m[1] += k0 * k1; m[2] += k0 * k2;
        m[3] += k1 * k1; m[4] += k1 * k2; m[5] += k2 * k2;
        m[6] += k0 * vr; m[7] += k1 * vr; m[8] += k2 * vr;
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) m[k] += __shfl_xor(m[k], off, 64);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ns += __shfl_xor(ns, off, 64);
    if (lane == 0) {
        for (int k = 0; k < 9; ++k) red[wave][k] = m[k];
        sidx[wave] = ns;
    }
    __syncthreads();
    if (tid != 0) return;
    double t[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int nst = 0;
    for (int w = 0; w < kEgoSelWG / 64; ++w) {
        for (int k = 0; k < 9; ++k) t[k] += red[w][k];
        nst += sidx[w];
    }
    // Eigen 3.3 compute_inverse<Matrix3d>: first-column cofactors, det, adjugate / det
    const double M[9] = {t[0], t[1], t[2], t[1], t[3], t[4], t[2], t[4], t[5]};
#define EM(i, j) M[3 * (i) + (j)]
    const double c0 = EM(1, 1) * EM(2, 2) - EM(1, 2) * EM(2, 1);
    const double c1 = EM(2, 1) * EM(0, 2) - EM(2, 2) * EM(0, 1);
    const double c2 = EM(0, 1) * EM(1, 2) - EM(0, 2) * EM(1, 1);
    const double det = c0 * EM(0, 0) + c1 * EM(1, 0) + c2 * EM(2, 0);
    const double inv = 1.0 / det;
    const double R[9] = {c0 * inv, c1 * inv, c2 * inv,
                         (EM(1, 2) * EM(2, 0) - EM(1, 0) * EM(2, 2)) * inv,
                         (EM(2, 2) * EM(0, 0) - EM(2, 0) * EM(0, 2)) * inv,
                         (EM(0, 2) * EM(1, 0) - EM(0, 0) * EM(1, 2)) * inv,
                         (EM(1, 0) * EM(2, 1) - EM(1, 1) * EM(2, 0)) * inv,
                         (EM(2, 0) * EM(0, 1) - EM(2, 1) * EM(0, 0)) * inv,
                         (EM(0, 0) * EM(1, 1) - EM(0, 1) * EM(1, 0)) * inv};
#undef EM
    icp4r_ego_result r;
    r.A = A;
    r.b = b;
    for (int k = 0; k < 3; ++k) r.v[k] = R[3 * k] * t[6] + R[3 * k + 1] * t[7] + R[3 * k + 2] * t[8];
    r.score = (double)best_s;
    r.n = n;
    r.n_static = nst;
    r.iterations = H;
    r.best = best_h;
    r.status = too_big ? ICP4R_E_INVALID : n > 0 ? 0 : ICP4R_E_EMPTY;
    r.reserved = 0;
    e.results[s] = r;
}

hipError_t launch_ego(const EgoArgs& e, int nscans, int max_n, float4* xyzi, hipStream_t st) {
    if (nscans <= 0 || max_n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ego_features_kernel, dim3((max_n + 255) / 256, nscans), dim3(256), 0, st, e.rec, e.off, e.cnt,
                       e.stride, e.feat, e.pd, xyzi);
    if (e.max_h > 0) {
        hipError_t err = hipMemsetAsync(e.scores, 0, (size_t)nscans * e.max_h * sizeof(int32_t), st);
        if (err != hipSuccess) return err;
        hipLaunchKernelGGL(ego_ransac_kernel, dim3((e.max_h + kEgoHyp - 1) / kEgoHyp, (max_n + kEgoPts - 1) / kEgoPts, nscans),
                           dim3(kEgoWG), 0, st, e);
    }
    hipLaunchKernelGGL(ego_select_kernel, dim3(nscans), dim3(kEgoSelWG), 0, st, e);
    return hipGetLastError();
}

hipError_t launch_ego_features(const EgoArgs& e, int nscans, int max_n, float4* xyzi, hipStream_t st) {
    hipLaunchKernelGGL(ego_features_kernel, dim3((max_n + 255) / 256, nscans), dim3(256), 0, st, e.rec, e.off, e.cnt,
                       e.stride, e.feat, e.pd, xyzi);
    return hipGetLastError();
}

}  // namespace icp4r
