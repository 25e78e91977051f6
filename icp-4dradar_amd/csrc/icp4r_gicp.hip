// icp4r_gicp.hip — generalized ICP for gfx950 (include/icp4r/icp4r_gicp.h).
//
// fast_gicp's FastGICPSingleThread, as the reference's radar_odometry node runs it on the scan-to-map
// path (radar_odometry.cpp:398-411), restated device-resident:
//
//   gicp_knn_cov_kernel<K>  per point: exact K nearest neighbours in its own cloud (the point
//   / gicp_cov_kernel<K>    included; (d², index) keys) — pruned over the ICP core's Morton index of
//                        the cloud, or brute force through LDS tiles for small clouds — then the
//                        mean-centred covariance in double, regularised (PLANE: U diag(1, 1, 1e-3) Uᵀ
//                        from a cyclic-Jacobi eigendecomposition)
//   per iteration        the exact NN pass of the ICP core (pruned / brute / LDS kernels, unchanged)
//                        over X = float(x0) · src, then
//   gicp_iter_kernel     one workgroup per pair: Mahalanobis M_i = (C_B + R C_A Rᵀ)⁻¹, the
//                        Gauss-Newton system (H = Σ JᵀMJ, g = Σ JᵀMe, y = Σ eᵀMe, J = [skew(T a), -I])
//                        in double with a fixed-order reduction, then Levenberg-Marquardt trials —
//                        thread 0 solves (H + λI) d = -g by LDLᵀ and forms delta = [so3_exp | t]; the
//                        whole workgroup re-evaluates the error at delta · x0 on the cached
//                        correspondences; accept / reject / converge as LsqRegistration::step_lm;
//                        then X := float(x0) · src for the next NN pass.
//
// Per-pair flags (PairState.phase) stop converged / failed pairs; the host launches the iterations
// in short runs and checks the flags in between.
#include <float.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "icp4r_device.hpp"
#include "icp4r_internal.hpp"
#include "icp4r_math.hpp"

namespace icp4r {

// ---- small double linear algebra (device)

// symmetric 3x3 eigendecomposition by cyclic Jacobi: a (row-major) -> w (descending), V (columns)
__device__ void gicp_sym_eig3(const double* a_in, double* w, double* V) {
    double a[9];
    for (int i = 0; i < 9; ++i) a[i] = a_in[i];
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        // converged: the off-diagonal mass is below 1e-30 of the diagonal's (~1e-15 relative per
        // element, the double rounding level; waiting for an exact zero took many more sweeps)
        if (a[1] * a[1] + a[2] * a[2] + a[5] * a[5] <= 1e-30 * (a[0] * a[0] + a[4] * a[4] + a[8] * a[8])) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                const double apq = a[3 * p + q];
                if (apq == 0.0) continue;
                const double theta = (a[3 * q + q] - a[3 * p + p]) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 3; ++k) {
                    const double akp = a[3 * k + p], akq = a[3 * k + q];
                    a[3 * k + p] = c * akp - s * akq;
                    a[3 * k + q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    const double apk = a[3 * p + k], aqk = a[3 * q + k];
                    a[3 * p + k] = c * apk - s * aqk;
                    a[3 * q + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    const double vkp = V[3 * k + p], vkq = V[3 * k + q];
                    V[3 * k + p] = c * vkp - s * vkq;
                    V[3 * k + q] = s * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < 3; ++i) w[i] = a[4 * i];
    for (int i = 0; i < 2; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (w[j] > w[i]) {
                const double tw = w[i];
                w[i] = w[j];
                w[j] = tw;
                for (int k = 0; k < 3; ++k) {
                    const double tv = V[3 * k + i];
                    V[3 * k + i] = V[3 * k + j];
                    V[3 * k + j] = tv;
                }
            }
}

// Eigen-style cofactor inverse of a 3x3 (row-major)
__device__ __forceinline__ void gicp_inv3(const double* m, double* r) {
    const double c0 = m[4] * m[8] - m[5] * m[7];
    const double c1 = m[7] * m[2] - m[8] * m[1];
    const double c2 = m[1] * m[5] - m[2] * m[4];
    const double id = 1.0 / (c0 * m[0] + c1 * m[3] + c2 * m[6]);
    r[0] = c0 * id;
    r[1] = c1 * id;
    r[2] = c2 * id;
    r[3] = (m[5] * m[6] - m[3] * m[8]) * id;
    r[4] = (m[8] * m[0] - m[6] * m[2]) * id;
    r[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    r[6] = (m[3] * m[7] - m[4] * m[6]) * id;
    r[7] = (m[6] * m[1] - m[7] * m[0]) * id;
    r[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

// fast_gicp::RegularizationMethod applied to a 3x3 covariance (row-major, symmetric)
__device__ void gicp_regularize(const double* c, int reg, double* o) {
    if (reg == ICP4R_GICP_REG_NONE) {
        for (int t = 0; t < 9; ++t) o[t] = c[t];
        return;
    }
    if (reg == ICP4R_GICP_REG_FROBENIUS) {
        double C[9], Ci[9], nrm = 0.0;
        for (int t = 0; t < 9; ++t) C[t] = c[t];
        for (int t = 0; t < 3; ++t) C[4 * t] += 1e-3;
        gicp_inv3(C, Ci);
        for (int t = 0; t < 9; ++t) nrm += Ci[t] * Ci[t];
        nrm = sqrt(nrm);
        for (int t = 0; t < 9; ++t) Ci[t] /= nrm;
        gicp_inv3(Ci, o);
        return;
    }
    double w[3], V[9], v[3];
    gicp_sym_eig3(c, w, V);
    for (int t = 0; t < 3; ++t) {
        if (reg == ICP4R_GICP_REG_PLANE) {
            v[t] = t < 2 ? 1.0 : 1e-3;
        } else if (reg == ICP4R_GICP_REG_MIN_EIG) {
            v[t] = fmax(w[t], 1e-3);
        } else {  // NORMALIZED_MIN_EIG
            v[t] = fmax(w[0] != 0.0 ? w[t] / w[0] : 0.0, 1e-3);
        }
    }
    for (int r = 0; r < 3; ++r)
        for (int s = 0; s < 3; ++s) o[3 * r + s] = V[3 * r] * v[0] * V[3 * s] + V[3 * r + 1] * v[1] * V[3 * s + 1] + V[3 * r + 2] * v[2] * V[3 * s + 2];
}

// mean-centred covariance of the kk nearest neighbours (sorted keys), divided by k as
// calculate_covariances does, regularised; out: the upper triangle (xx, xy, xz, yy, yz, zz)
// (the index is clamped to the cloud: an unfilled slot can never address outside it)
template <int K>
__device__ __forceinline__ void gicp_cov_from_knn(const uint64_t (&best)[K], int kk, int k, int reg, const float4* c,
                                                  int n, double* out) {
    double mean[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < K; ++s) {
        if (s < kk) {
            const float4 v = c[min((uint32_t)best[s], (uint32_t)(n - 1))];
            mean[0] += (double)v.x;
            mean[1] += (double)v.y;
            mean[2] += (double)v.z;
        }
    }
    for (int r = 0; r < 3; ++r) mean[r] /= (double)kk;
    double cv[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < K; ++s) {
        if (s < kk) {
            const float4 v = c[min((uint32_t)best[s], (uint32_t)(n - 1))];
            const double d[3] = {(double)v.x - mean[0], (double)v.y - mean[1], (double)v.z - mean[2]};
            for (int r = 0; r < 3; ++r)
                for (int t = 0; t < 3; ++t) cv[3 * r + t] += d[r] * d[t];
        }
    }
    for (int t = 0; t < 9; ++t) cv[t] /= (double)k;
    double o[9];
    gicp_regularize(cv, reg, o);
    out[0] = o[0];
    out[1] = o[1];
    out[2] = o[2];
    out[3] = o[4];
    out[4] = o[5];
    out[5] = o[8];
}

// insert key into the ascending top-K list (registers: a fully unrolled compare-exchange chain)
template <int K>
__device__ __forceinline__ void knn_insert(uint64_t (&best)[K], uint64_t key) {
    if (key < best[K - 1]) {
#pragma unroll
        for (int s = 0; s < K; ++s) {
            const uint64_t lo = key < best[s] ? key : best[s];
            key = key < best[s] ? best[s] : key;
            best[s] = lo;
        }
    }
}

// ---- covariances
constexpr int kCovWG = 256;
constexpr int kCovTile = 1024;

// the L lists of a query (lanes lane ^ o, o < L) into one: each lane takes in its partners' keys, so all
// L lanes end with the K smallest of their union
template <int K, int L>
__device__ __forceinline__ void knn_merge_lanes(uint64_t (&best)[K]) {
#pragma unroll
    for (int o = 1; o < L; o <<= 1) {
        uint64_t other[K];
#pragma unroll
        for (int s = 0; s < K; ++s) {
            const uint32_t lo = __shfl_xor((uint32_t)best[s], o, 64), hi = __shfl_xor((uint32_t)(best[s] >> 32), o, 64);
            other[s] = (uint64_t)hi << 32 | lo;
        }
#pragma unroll
        for (int s = 0; s < K; ++s) knn_insert<K>(best, other[s]);
    }
}

// Brute-force exact k-NN (every point of the cloud through LDS tiles), L lanes per query each taking
// every L-th point of a tile: plans that do not prune, and the reference the pruned walk is tested
// against (slower than index + pruned walk even for one 8k scan, §6d).
template <int K, int L>
__global__ __launch_bounds__(kCovWG) void gicp_cov_kernel(const float4* __restrict__ cloud, const int64_t* __restrict__ off,
                                                          const int32_t* __restrict__ cnt, int64_t stride, int k, int reg,
                                                          double* __restrict__ cov_out) {
    __shared__ float4 tile[kCovTile];
    constexpr int QW = kCovWG / L;  // queries per workgroup
    const int p = blockIdx.y;
    const int n = cnt[p];
    const int i = blockIdx.x * QW + threadIdx.x / L, sub = threadIdx.x % L;
    if (blockIdx.x * QW >= n) return;
    const float4* c = cloud + off[p];
    const float4 q = c[min(i, n - 1)];
    uint64_t best[K];
#pragma unroll
    for (int s = 0; s < K; ++s) best[s] = ~0ull;
    for (int j0 = 0; j0 < n; j0 += kCovTile) {
        const int len = min(kCovTile, n - j0);
        __syncthreads();
        for (int t = threadIdx.x; t < len; t += kCovWG) tile[t] = c[j0 + t];
        __syncthreads();
        for (int t = sub; t < len; t += L) {
            const float4 v = tile[t];
            const float d2 = l2_simple(q.x, q.y, q.z, v.x, v.y, v.z);
            knn_insert<K>(best, make_key(d2, (uint32_t)(j0 + t)));
        }
    }
    knn_merge_lanes<K, L>(best);
    if (sub != 0 || i >= n) return;
    gicp_cov_from_knn<K>(best, min(k, n), k, reg, c, n, cov_out + ((int64_t)p * stride + i) * 6);
}

// Pruned exact k-NN over the cloud's own Morton index (index_kernel of the ICP core, built with the
// cloud as target: tsort / tbox / sbox).  L lanes per query, each taking every L-th point of a block
// into a top-K list of its own; the 64 / L queries of a wave are Morton-contiguous (sorted position =
// query); the wave walks superblocks outward from its own and skips a (super)block whose box lower
// bound exceeds every query's bound (the least K-th best d² of its L lanes, kLbShrink margin: the
// K-th best of the union is no larger). At the end the L lists of a query merge (shuffles + inserts).
// Keys are (d², index): the K smallest are exactly the brute-force set, ties to the lowest index.
// (L = 1 had one wave walk ~25 blocks of 16 points one after another for 64 queries, ~400 distance
// evaluations per query on the bench clouds: latency-bound, a wave per SIMD on a single 8k cloud.)
__device__ __forceinline__ float box_lb(const v4f lo, const v4f hi, float x, float y, float z) {
    const float gx = fmaxf(fmaxf(lo.x - x, x - hi.x), 0.0f);
    const float gy = fmaxf(fmaxf(lo.y - y, y - hi.y), 0.0f);
    const float gz = fmaxf(fmaxf(lo.z - z, z - hi.z), 0.0f);
    return __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, gx * gx));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, v)));
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off, 64));
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, v)));
}

template <int K, int L>
__global__ __launch_bounds__(kCovWG) void gicp_knn_cov_kernel(const float4* __restrict__ cloud,
                                                              const int64_t* __restrict__ off,
                                                              const int32_t* __restrict__ cnt, WorkArgs w,
                                                              int64_t stride, int k, int reg,
                                                              double* __restrict__ cov_out) {
    constexpr int B = 16, Q = 64 / L;
    static_assert(L == 1 || L == 2 || L == 4 || L == 8, "lanes per query");
    const int chunks = gridDim.x;
    const int g = xcd_remap(blockIdx.x + chunks * blockIdx.y, chunks * gridDim.y);
    const int p = g / chunks, ch = g - p * chunks;
    const int n = uload(cnt + p);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int base = ch * (kCovWG / L) + wave * Q;
    if (base >= n) return;
    const int qi = lane / L, sub = lane % L;
    const float4* tsg = w.tsort + (int64_t)p * w.t_stride;
    const float4 qv = tsg[min(base + qi, n - 1)];
    const float x = qv.x, y = qv.y, z = qv.z;
    // empty slots hold (+inf, ~0): a real d² bound for the pruning tests (all-ones bits would be a NaN
    // d² that no box bound passes) that every finite key beats
    uint64_t best[K];
#pragma unroll
    for (int s = 0; s < K; ++s) best[s] = make_key(INFINITY, 0xFFFFFFFFu);
    float qlo[3] = {wave_min(x), wave_min(y), wave_min(z)};
    float qhi[3] = {wave_max(x), wave_max(y), wave_max(z)};
    float qmax = INFINITY;
    float gb = INFINITY;  // this query's bound: the least K-th best of its L lanes
    auto group_bound = [&]() {
        float b = __uint_as_float((uint32_t)(best[K - 1] >> 32));
#pragma unroll
        for (int o = 1; o < L; o <<= 1) b = fminf(b, __shfl_xor(b, o, 64));
        return b;
    };
    const int nb = (n + B - 1) / B, nsb = (nb + kSuper - 1) / kSuper;
    const int sb0 = base / (B * kSuper);  // (Q divides B * kSuper: the wave's queries share it)
    const cv4f_ptr ts = as_const(tsg);
    const cv4f_ptr tb = as_const(w.tbox + (int64_t)p * 2 * w.b_stride);
    const cv4f_ptr sbx = as_const(w.sbox + (int64_t)p * 2 * w.sb_stride);
    auto maybe = [&](const v4f lo, const v4f hi) {
        const float gx = fmaxf(fmaxf(lo.x - qhi[0], qlo[0] - hi.x), 0.0f);
        const float gy = fmaxf(fmaxf(lo.y - qhi[1], qlo[1] - hi.y), 0.0f);
        const float gz = fmaxf(fmaxf(lo.z - qhi[2], qlo[2] - hi.z), 0.0f);
        return __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, gx * gx)) * kLbShrink <= qmax;
    };
    auto needed = [&](const v4f lo, const v4f hi) { return __any(box_lb(lo, hi, x, y, z) * kLbShrink <= gb); };
    unsigned long long swept = 0;
    auto visit = [&](int sb, bool test) {  // sweep superblock sb's needed blocks, then refresh the bound
        const v4f slo = sbx[2 * sb], shi = sbx[2 * sb + 1];
        if (test && (!maybe(slo, shi) || !needed(slo, shi))) return;
        for (int b = sb * kSuper; b < (sb + 1) * kSuper; ++b) {
            const v4f blo = tb[2 * b], bhi = tb[2 * b + 1];
            if (!maybe(blo, bhi) || !needed(blo, bhi)) continue;
            const cv4f_ptr blk = ts + (int64_t)b * B;
#pragma unroll
            for (int t = 0; t < B / L; ++t) {
                const v4f v = blk[sub + L * t];
                knn_insert<K>(best, make_key(l2_simple(x, y, z, v.x, v.y, v.z), __float_as_uint(v.w)));
            }
            ++swept;
            gb = group_bound();
        }
        qmax = wave_max(gb);
    };
    if (nsb <= 64) {
        // the wave's own superblock first (a finite K-th bound for every lane), then one lane-parallel
        // coarse test of every superblock against the wave's query box with that bound, and only the
        // survivors, outward from the own one (a scalar walk over all superblocks cost a box load and
        // ~10 SALU per superblock per wave)
        visit(sb0, false);
        const int sl = min(lane, nsb - 1);
        const v4f* sbv = reinterpret_cast<const v4f*>(w.sbox + (int64_t)p * 2 * w.sb_stride);
        if (L > 1) {
            // (lanes per query, small grids) nearest first: each lane holds its superblock's gap to the
            // wave's query box; the survivors are visited in increasing gap (a wave argmin per visit), so
            // the bound tightens soonest, and the walk ends when the nearest left is beyond it — the
            // k = 20 pair 0.56 -> 0.54 ms; on the one-lane batch the argmins cost more than they saved
            // (3.37 -> 3.41 ms), so it keeps the outward walk
            const v4f mlo = sbv[2 * sl], mhi = sbv[2 * sl + 1];
            const float gx = fmaxf(fmaxf(mlo.x - qhi[0], qlo[0] - mhi.x), 0.0f);
            const float gy = fmaxf(fmaxf(mlo.y - qhi[1], qlo[1] - mhi.y), 0.0f);
            const float gz = fmaxf(fmaxf(mlo.z - qhi[2], qlo[2] - mhi.z), 0.0f);
            const float gap = __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, gx * gx)) * kLbShrink;
            uint64_t cm = __ballot(lane < nsb && lane != sb0 && gap <= qmax);
            while (cm) {
                const float mine = (cm >> lane) & 1 ? gap : INFINITY;
                const float mn = wave_min(mine);
                if (mn > qmax) break;  // every superblock left is beyond the bound
                const int sb = __builtin_ctzll(__ballot(((cm >> lane) & 1) && mine == mn));
                cm &= ~(1ull << sb);
                visit(sb, true);
            }
        } else {
            const uint64_t cm = __ballot(lane < nsb && lane != sb0 && maybe(sbv[2 * sl], sbv[2 * sl + 1]));
            uint64_t um = sb0 < 63 ? (cm >> (sb0 + 1)) << (sb0 + 1) : 0ull, dm = cm & ~um;
            for (bool upnext = true; um | dm; upnext = !upnext) {
                int sb;
                if (um && (upnext || !dm)) {
                    sb = __builtin_ctzll(um);
                    um &= um - 1;
                } else {
                    sb = 63 - __builtin_clzll(dm);
                    dm &= ~(1ull << sb);
                }
                visit(sb, true);
            }
        }
    } else {  // large clouds (the scan-to-map submap): the superblocks 64 at a time, groups outward from
              // the own one — one lane-parallel coarse test per group with the bound reached so far, then
              // only its survivors, in outward order (a scalar walk over every superblock had cost a box
              // load and a test per superblock per wave: 512 of them per wave on the 65k map)
        visit(sb0, false);
        const v4f* sbv = reinterpret_cast<const v4f*>(w.sbox + (int64_t)p * 2 * w.sb_stride);
        const int ng = (nsb + 63) / 64, g0 = sb0 / 64;
        for (int d = 0; g0 - d >= 0 || g0 + d < ng; ++d) {
            for (int side = 0; side < 2; ++side) {
                const int g = side == 0 ? g0 + d : g0 - d;
                if (g < 0 || g >= ng || (d == 0 && side == 1)) continue;
                const int sl = min(g * 64 + lane, nsb - 1);
                const uint64_t cm = __ballot(g * 64 + lane < nsb && g * 64 + lane != sb0 && maybe(sbv[2 * sl], sbv[2 * sl + 1]));
                if (g > g0) {  // ascending from the group's start
                    for (uint64_t m = cm; m; m &= m - 1) visit(g * 64 + __builtin_ctzll(m), true);
                } else if (g < g0) {  // descending from its end
                    for (uint64_t m = cm; m;) {
                        const int b = 63 - __builtin_clzll(m);
                        m &= ~(1ull << b);
                        visit(g * 64 + b, true);
                    }
                } else {  // the own group: outward from sb0
                    const int r0 = sb0 - g * 64;
                    uint64_t um = r0 < 63 ? (cm >> (r0 + 1)) << (r0 + 1) : 0ull, dm = cm & ~um;
                    for (bool upnext = true; um | dm; upnext = !upnext) {
                        int b;
                        if (um && (upnext || !dm)) {
                            b = __builtin_ctzll(um);
                            um &= um - 1;
                        } else {
                            b = 63 - __builtin_clzll(dm);
                            dm &= ~(1ull << b);
                        }
                        visit(g * 64 + b, true);
                    }
                }
            }
        }
    }
    if (lane == 0 && w.evals) count_add(w.evals, 0, swept * B * (unsigned long long)min(n - base, Q));
    knn_merge_lanes<K, L>(best);
    if (sub != 0 || base + qi >= n) return;
    const uint32_t oi = __float_as_uint(qv.w);
    gicp_cov_from_knn<K>(best, min(k, n), k, reg, cloud + off[p], n, cov_out + ((int64_t)p * stride + oi) * 6);
}

// ---- per-iteration update
constexpr int kGicpSliceWG = 256;  // threads per slice workgroup; a slice is a multiple of it
constexpr int kGicpSliceWaves = kGicpSliceWG / 64;
// (the linearisation's deciding workgroup hands out its copies by thread ranges up to thread 140)
static_assert(kGicpSliceWG >= 128 + 12 && kGicpSliceWG >= kGicpSpec * 12, "slice workgroup too small");

// points per slice and slices of an n-point source: at least one slice (an empty source still
// decides), at most kGicpMaxSlices, a slice a multiple of kGicpSliceWG points
__host__ __device__ __forceinline__ int gicp_slice_pts(int n) {
    const int m = (n + kGicpSliceWG * kGicpMaxSlices - 1) / (kGicpSliceWG * kGicpMaxSlices);
    return kGicpSliceWG * (m > 1 ? m : 1);
}
__host__ __device__ __forceinline__ int gicp_slices(int n) {
    const int s = (n + gicp_slice_pts(n) - 1) / gicp_slice_pts(n);
    return s > 1 ? s : 1;
}

__device__ __forceinline__ void sym_unpack(const double* s, double* m) {
    m[0] = s[0]; m[1] = s[1]; m[2] = s[2];
    m[3] = s[1]; m[4] = s[3]; m[5] = s[4];
    m[6] = s[2]; m[7] = s[4]; m[8] = s[5];
}

// so3_exp (fast_gicp so3.hpp) then Eigen's Quaternion::toRotationMatrix
__device__ void gicp_so3_exp(const double* w, double* R) {
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double imag, real;
    if (th2 < 1e-10) {
        const double th4 = th2 * th2;
        imag = 0.5 - 1.0 / 48.0 * th2 + 1.0 / 3840.0 * th4;
        real = 1.0 - 1.0 / 8.0 * th2 + 1.0 / 384.0 * th4;
    } else {
        const double th = sqrt(th2), half = 0.5 * th;
        imag = sin(half) / th;
        real = cos(half);
    }
    const double qw = real, qx = imag * w[0], qy = imag * w[1], qz = imag * w[2];
    const double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
    const double twx = tx * qw, twy = ty * qw, twz = tz * qw, txx = tx * qx, txy = ty * qx, txz = tz * qx;
    const double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

// (A) x = b, A symmetric positive definite 6x6 (row-major), LDLᵀ without pivoting; L overwrites A's
// strict lower triangle (each A[i][j], i > j, is read once, just before L[i][j] replaces it: the same
// operations in the same order as with a separate L, in a third of the registers — the separate 6x6
// arrays beside the LM state had spilled the iteration kernel to scratch)
__device__ void gicp_ldlt6(double (&A)[36], const double (&b)[6], double (&x)[6]) {
    double D[6], y[6];
    for (int j = 0; j < 6; ++j) {
        double s = A[6 * j + j];
        for (int k = 0; k < j; ++k) s -= A[6 * j + k] * A[6 * j + k] * D[k];
        D[j] = s;
        for (int i = j + 1; i < 6; ++i) {
            double t = A[6 * i + j];
            for (int k = 0; k < j; ++k) t -= A[6 * i + k] * A[6 * j + k] * D[k];
            A[6 * i + j] = D[j] != 0.0 ? t / D[j] : t;  // Eigen: a zero pivot leaves its column undivided
        }
    }
    for (int i = 0; i < 6; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= A[6 * i + k] * y[k];
        y[i] = s;
    }
    for (int i = 0; i < 6; ++i) y[i] = fabs(D[i]) > DBL_MIN ? y[i] / D[i] : 0.0;  // Eigen's LDLT::solve
    for (int i = 5; i >= 0; --i) {
        double s = y[i];
        for (int k = i + 1; k < 6; ++k) s -= A[6 * k + i] * x[k];
        x[i] = s;
    }
}

__device__ __forceinline__ bool gicp_converged(const double* R, const double* t, double rot_eps, double trans_eps) {
    double m = 0.0;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) m = fmax(m, 1.0 / rot_eps * fabs(R[3 * r + c] - (r == c ? 1.0 : 0.0)));
    for (int r = 0; r < 3; ++r) m = fmax(m, 1.0 / trans_eps * fabs(t[r]));
    return m < 1.0;
}

// the error eᵀMe of correspondence (a, b) at transform (R, t), and with LIN its terms of H = Σ JᵀMJ and
// g = Σ JᵀMe (J = [skew(Ta), -I]) and the count, into acc (fast_gicp's linearize / compute_error)
template <bool LIN>
__device__ __forceinline__ void gicp_point(const float4 sa, const float4 sb, const double (&M)[9], const double* R,
                                           const double* t, double* acc) {
    const double a[3] = {sa.x, sa.y, sa.z};
    double ta[3];
    for (int r = 0; r < 3; ++r) ta[r] = R[3 * r] * a[0] + R[3 * r + 1] * a[1] + R[3 * r + 2] * a[2] + t[r];
    const double e[3] = {(double)sb.x - ta[0], (double)sb.y - ta[1], (double)sb.z - ta[2]};
    double Me[3];
    for (int r = 0; r < 3; ++r) Me[r] = M[3 * r] * e[0] + M[3 * r + 1] * e[1] + M[3 * r + 2] * e[2];
    if (!LIN) {
        acc[0] += e[0] * Me[0] + e[1] * Me[1] + e[2] * Me[2];
        return;
    }
    acc[27] += e[0] * Me[0] + e[1] * Me[1] + e[2] * Me[2];
    acc[28] += 1.0;
    // J = [skew(Ta), -I] (row k: J[k][0..2] = skew, J[k][3 + k] = -1). The terms with a zero or -1
    // factor of J are left out or reduced to a negation: the same values as the generic JᵀMJ / JᵀMe
    // sums (x + (+-0) = x), in half the operations.
    auto js = [&](int k, int c) -> double {  // skew(Ta)[k][c], k != c
        return k == 0 ? (c == 1 ? -ta[2] : ta[1]) : k == 1 ? (c == 0 ? ta[2] : -ta[0]) : (c == 0 ? -ta[1] : ta[0]);
    };
    double MS[9];  // M skew(Ta)
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int k0 = c == 0 ? 1 : 0, k1 = c == 2 ? 1 : 2;
            MS[3 * r + c] = M[3 * r + k0] * js(k0, c) + M[3 * r + k1] * js(k1, c);
        }
    int u = 0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const int k0 = r == 0 ? 1 : 0, k1 = r == 2 ? 1 : 2;  // the rows k != r of column r of J
#pragma unroll
        for (int c = r; c < 3; ++c) acc[u++] += js(k0, r) * MS[3 * k0 + c] + js(k1, r) * MS[3 * k1 + c];
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[u++] += js(k0, r) * -M[3 * k0 + c] + js(k1, r) * -M[3 * k1 + c];
        acc[21 + r] += js(k0, r) * Me[k0] + js(k1, r) * Me[k1];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = r; c < 3; ++c) acc[u++] += M[3 * r + c];
        acc[24 + r] += -Me[r];
    }
}

// Σ over the workgroup of each v[k] in a fixed order (butterfly per wave, then the waves in order);
// the sum of v[k] is returned to thread k < NV. red: kGicpSliceWaves * NV doubles of LDS.
template <int NV>
__device__ __forceinline__ double gicp_slice_sum(double (&v)[NV], double* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off, 64);
    }
    if (lane == 0)
        for (int k = 0; k < NV; ++k) red[wave * NV + k] = v[k];
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x < NV)
        for (int q = 0; q < kGicpSliceWaves; ++q) r += red[q * NV + threadIdx.x];
    __syncthreads();  // red is free again
    return r;
}

// The same for the 29 sums of the linearisation, as a transposing reduction: at each step a lane keeps
// half of its values and adds its partner's copy of that half (one shuffle per kept value), so the 32
// padded values take 16 + 8 + 4 + 2 + 1 + 1 shuffles instead of 29 x 6; lanes 2k and 2k + 1 end with
// the wave's sum of value k (another fixed order than the butterfly's). In place in v.
__device__ __forceinline__ double gicp_slice_sum_sys(double (&v)[kGicpSys], double* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    {
        const bool hi = lane & 32;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const double lo_v = v[k], hi_v = k + 16 < kGicpSys ? v[k + 16] : 0.0;
            v[k] = (hi ? hi_v : lo_v) + __shfl_xor(hi ? lo_v : hi_v, 32, 64);
        }
    }
#pragma unroll
    for (int h = 8, o = 16; h >= 1; h >>= 1, o >>= 1) {
        const bool hi = lane & o;
#pragma unroll
        for (int k = 0; k < h; ++k) {
            const double a = v[k], b = v[k + h];
            v[k] = (hi ? b : a) + __shfl_xor(hi ? a : b, o, 64);
        }
    }
    const double r1 = v[0] + __shfl_xor(v[0], 1, 64);
    const int k = lane >> 1;  // the value this lane pair holds
    if (!(lane & 1) && k < kGicpSys) red[wave * kGicpSys + k] = r1;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x < kGicpSys)
        for (int q = 0; q < kGicpSliceWaves; ++q) r += red[q * kGicpSys + threadIdx.x];
    __syncthreads();
    return r;
}

// the LM trial of damping lambda from the system sys at x0 = (R0, t0): delta from (H + λI) d = -g,
// the trial transform delta * x0 (fast_gicp LsqRegistration::step_lm)
__device__ void gicp_make_trial(const double* sys, double lambda, const double* R0, const double* t0, GicpTrial& o) {
    double A[36], nb[6];
    int u = 0;
    for (int r = 0; r < 6; ++r)
        for (int c = r; c < 6; ++c) A[6 * r + c] = A[6 * c + r] = sys[u++];
    for (int k = 0; k < 6; ++k) A[7 * k] += lambda;
    for (int k = 0; k < 6; ++k) nb[k] = -sys[21 + k];
    double d[6];
    gicp_ldlt6(A, nb, d);
    for (int k = 0; k < 6; ++k) o.d[k] = d[k];
    gicp_so3_exp(d, o.dR);
    o.dt[0] = d[3];
    o.dt[1] = d[4];
    o.dt[2] = d[5];
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) o.R[3 * r + c] = o.dR[3 * r] * R0[c] + o.dR[3 * r + 1] * R0[3 + c] + o.dR[3 * r + 2] * R0[6 + c];
        o.t[r] = o.dR[3 * r] * t0[0] + o.dR[3 * r + 1] * t0[1] + o.dR[3 * r + 2] * t0[2] + o.dt[r];
    }
    o.lambda = lambda;
}

struct GicpPairView {
    int n, ps, ns;  // points, points per slice, slices
    const float4 *src, *tgt;
    const NNKey* key;
    double* mah;
};

__device__ __forceinline__ GicpPairView gicp_view(const PairArgs& a, const WorkArgs& w, const GicpArgs& g, int p) {
    GicpPairView v;
    v.n = a.src_n[p];
    v.ps = gicp_slice_pts(v.n);
    v.ns = gicp_slices(v.n);
    v.src = a.src + a.src_off[p];
    v.tgt = a.tgt + a.tgt_off[p];
    v.key = w.nn_key + (int64_t)p * w.x_stride;
    v.mah = g.mah + (int64_t)p * w.x_stride * 6;
    return v;
}

// Workgroup j of a pair takes its slices j, j + W, j + 2W, ... (W workgroups per pair, fewer for many pairs:
// the slicing, and so every sum, depends on n only; W only spreads the slices over the chip).
// The per-slice sums of one pair reach the workgroup that finishes last (the counter form of the
// hand-off in cdna_hip_programming.md §6 Guideline 16, with write-through sum stores, gicp_publish,
// in place of a release fence in every workgroup): every workgroup waits for its stores and draws a
// ticket; the one drawing nw - 1 acquires, resets the counter for the next launch and returns true
// (in all its threads).
// This block's pair and its index j < W among the pair's workgroups: the W workgroups of a pair on one
// XCD, as blocks are dealt round-robin over the 8 XCDs (blocks b and b + 8 share one), so a pair's
// gathered target data is fetched into one L2, not eight (a speed choice only: nothing depends on it)
__device__ __forceinline__ bool gicp_block(int npairs, int W, int& p, int& j) {
    const int b = blockIdx.x, x = b & 7, r = b >> 3;
    p = (r / W) * 8 + x;
    j = r % W;
    return p < npairs;
}

__device__ __forceinline__ void gicp_publish(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool gicp_last_slice(int32_t* cnt, int nw, int32_t* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == nw - 1;
        if (last) {
            __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    return *flag != 0;
}

// (1) update_correspondences + linearize over one slice: M_i = (C_B + R C_A Rᵀ)⁻¹ of every valid
// correspondence (kept for the trials) and the slice's sums of H, g, y, |valid| at x0. The last slice
// sums the slices in order and solves the first LM trials (step_lm's (H + λI) d = -g, λ, 2λ, 8λ, ...).
__global__ __launch_bounds__(kGicpSliceWG) void gicp_lin_kernel(PairArgs a, WorkArgs w, GicpArgs g, int npairs, int W) {
    __shared__ double red[kGicpSliceWaves * kGicpSys];
    __shared__ int32_t last;
    int p, j;
    if (!gicp_block(npairs, W, p, j)) return;
    if (w.state[p].phase != kPhaseActive) return;
    const GicpPairView v = gicp_view(a, w, g, p);
    if (j >= v.ns) return;
    const int nw = min(W, v.ns);
    const double* cs = g.cov_src + (int64_t)p * w.x_stride * 6;
    const double* ct = g.cov_tgt + (int64_t)p * g.t_stride * 6;
    const GicpState& gs = g.gs[p];
    double R[9], t[3];
    for (int k = 0; k < 9; ++k) R[k] = gs.R[k];
    for (int k = 0; k < 3; ++k) t[k] = gs.t[k];
    double* part = g.part_lin + (int64_t)p * kGicpMaxSlices * kGicpSys;
    for (int q = j; q < v.ns; q += W) {
        double acc[kGicpSys];
        for (int k = 0; k < kGicpSys; ++k) acc[k] = 0.0;
        const int hi = min(v.n, (q + 1) * v.ps);
        for (int i = q * v.ps + threadIdx.x; i < hi; i += kGicpSliceWG) {
            const NNKey kk = v.key[i];
            if (!((double)key_d2(kk) < g.max_d2)) continue;
            const int j = key_idx(kk);
            double CA[9], CB[9], RC[9], RCR[9], Mi[9];
            sym_unpack(cs + (int64_t)i * 6, CA);
            sym_unpack(ct + (int64_t)j * 6, CB);
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) RC[3 * r + c] = R[3 * r] * CA[c] + R[3 * r + 1] * CA[3 + c] + R[3 * r + 2] * CA[6 + c];
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c)
                    RCR[3 * r + c] = CB[3 * r + c] + (RC[3 * r] * R[3 * c] + RC[3 * r + 1] * R[3 * c + 1] + RC[3 * r + 2] * R[3 * c + 2]);
            gicp_inv3(RCR, Mi);
            const double m6[6] = {Mi[0], Mi[1], Mi[2], Mi[4], Mi[5], Mi[8]};
            double* o = v.mah + (int64_t)i * 6;
            for (int k = 0; k < 6; ++k) o[k] = m6[k];
            double M[9];
            sym_unpack(m6, M);
            gicp_point<true>(v.src[i], v.tgt[j], M, R, t, acc);
        }
        const double r = gicp_slice_sum_sys(acc, red);
        if (threadIdx.x < kGicpSys) gicp_publish(part + q * kGicpSys + threadIdx.x, r);
    }
    if (!gicp_last_slice(g.cnt + p, nw, &last)) return;
    // the slices' sums staged in LDS by all threads at once (one round trip, not one per slice), then
    // added in slice order
    __shared__ double stage[kGicpMaxSlices * kGicpSys];
    for (int e = threadIdx.x; e < v.ns * kGicpSys; e += kGicpSliceWG) stage[e] = part[e];
    __syncthreads();
    double* sys = red;  // (free again)
    if (threadIdx.x < kGicpSys) {
        double t = 0.0;
        for (int q = 0; q < v.ns; ++q) t += stage[q * kGicpSys + threadIdx.x];
        sys[threadIdx.x] = t;
    }
    __syncthreads();
    GicpCand& gc = g.cand[p];
    const int nt = min(g.spec, g.lm_max_iterations);
    if (threadIdx.x < nt) {
        const int k = threadIdx.x;
        double lambda = gs.lambda, nu = 2.0;
        if (lambda < 0.0) {
            double mx = 0.0;
            const int diag[6] = {0, 6, 11, 15, 18, 20};  // (r, r) in the packed upper triangle
            for (int q = 0; q < 6; ++q) mx = fmax(mx, fabs(sys[diag[q]]));
            lambda = g.lm_init * mx;
        }
        for (int q = 0; q < k; ++q) {
            lambda = nu * lambda;
            nu = 2 * nu;
        }
        GicpTrial tr;
        gicp_make_trial(sys, lambda, R, t, tr);
        gc.c[k] = tr;
    }
    if (threadIdx.x == 63) {  // (independent of nt: gicp_spec = 0 runs every trial one by one from it)
        double lambda = gs.lambda;
        if (lambda < 0.0) {
            double mx = 0.0;
            const int diag[6] = {0, 6, 11, 15, 18, 20};
            for (int q = 0; q < 6; ++q) mx = fmax(mx, fabs(sys[diag[q]]));
            lambda = g.lm_init * mx;
        }
        gc.lambda0 = lambda;
    }
    if (threadIdx.x >= 64 && threadIdx.x < 64 + kGicpSys) gc.sys[threadIdx.x - 64] = sys[threadIdx.x - 64];
    if (threadIdx.x >= 128 && threadIdx.x < 140) {
        const int q = threadIdx.x - 128;
        if (q < 9) gc.R0[q] = R[q];
        else gc.t0[q - 9] = t[q - 9];
    }
}

// (2) the trials' errors over one slice. The last slice sums them in order and decides (accept, converge
// on a rejected step, or raise λ); in the rare case every speculative trial was rejected it runs the
// further trials one by one over all slices, each summed slice by slice exactly as above; then it
// writes x0, λ and the pair's state.
__global__ __launch_bounds__(kGicpSliceWG) void gicp_trial_kernel(PairArgs a, WorkArgs w, GicpArgs g, int npairs, int W, int it) {
    __shared__ double red[kGicpSliceWaves * kGicpSpec];
    __shared__ double pose[kGicpSpec][12];
    __shared__ double err[kGicpSpec];
    __shared__ double x0[12];   // the transform after this iteration
    __shared__ GicpTrial cur;   // the last trial decided on
    __shared__ double lam, nuv;
    __shared__ int32_t stop;    // 1 accepted, 2 converged on a rejected step, 0 none yet
    __shared__ int32_t last;
    int p, j;
    if (!gicp_block(npairs, W, p, j)) return;
    PairState& st = w.state[p];
    if (st.phase != kPhaseActive) return;
    const GicpPairView v = gicp_view(a, w, g, p);
    const int ns = v.ns;
    if (j >= ns) return;
    const int nw = min(W, ns);
    const int nt = min(g.spec, g.lm_max_iterations);
    const GicpCand& gc = g.cand[p];
    if (threadIdx.x < nt * 12) {
        const int k = threadIdx.x / 12, q = threadIdx.x % 12;
        pose[k][q] = q < 9 ? gc.c[k].R[q] : gc.c[k].t[q - 9];
    }
    __syncthreads();
    {
        double* part = g.part_err + (int64_t)p * kGicpMaxSlices * kGicpSpec;
        for (int q = j; q < ns; q += W) {
            double acc[kGicpSpec];
            for (int k = 0; k < kGicpSpec; ++k) acc[k] = 0.0;
            const int hi = min(v.n, (q + 1) * v.ps);
            for (int i = q * v.ps + threadIdx.x; i < hi; i += kGicpSliceWG) {
                const NNKey kk = v.key[i];
                if (!((double)key_d2(kk) < g.max_d2)) continue;
                const float4 sa = v.src[i], sb = v.tgt[key_idx(kk)];
                double M[9];
                sym_unpack(v.mah + (int64_t)i * 6, M);
                for (int k = 0; k < nt; ++k) gicp_point<false>(sa, sb, M, pose[k], pose[k] + 9, acc + k);
            }
            const double r = gicp_slice_sum(acc, red);
            if (threadIdx.x < kGicpSpec) gicp_publish(part + q * kGicpSpec + threadIdx.x, r);
        }
        if (!gicp_last_slice(g.cnt + p, nw, &last)) return;
        __shared__ double stage[kGicpMaxSlices * kGicpSpec];  // (as in the linearisation)
        for (int e = threadIdx.x; e < ns * kGicpSpec; e += kGicpSliceWG) stage[e] = part[e];
        __syncthreads();
        if (threadIdx.x < nt) {
            double t = 0.0;
            for (int q = 0; q < ns; ++q) t += stage[q * kGicpSpec + threadIdx.x];
            err[threadIdx.x] = t;
        }
    }
    __syncthreads();
    const double y0 = gc.sys[27];
    // rho = (y0 - yi) / dᵀ(λd - g)
    auto decide = [&](double yi) {
        const double lambda = cur.lambda;
        double den = 0.0;
        for (int k = 0; k < 6; ++k) den += cur.d[k] * (lambda * cur.d[k] - gc.sys[21 + k]);
        const double rho = (y0 - yi) / den;
        if (rho < 0) {
            if (gicp_converged(cur.dR, cur.dt, g.rot_eps, g.trans_eps)) {
                stop = 2;
            } else {
                lam = nuv * lambda;
                nuv = 2 * nuv;
            }
        } else {
            for (int k = 0; k < 9; ++k) x0[k] = cur.R[k];
            for (int k = 0; k < 3; ++k) x0[9 + k] = cur.t[k];
            lam = lambda * fmax(1.0 / 3.0, 1 - pow(2 * rho - 1, 3));
            stop = 1;
        }
    };
    if (threadIdx.x == 0) {
        for (int k = 0; k < 9; ++k) x0[k] = gc.R0[k];
        for (int k = 0; k < 3; ++k) x0[9 + k] = gc.t0[k];
        stop = 0;
        nuv = 2.0;
        lam = gc.lambda0;  // (== gc.c[0].lambda when trials were solved up front)
        for (int k = 0; k < nt && !stop; ++k) {
            cur = gc.c[k];
            decide(err[k]);
        }
    }
    __syncthreads();
    for (int k = nt; k < g.lm_max_iterations; ++k) {
        if (stop) break;
        __syncthreads();  // every thread read stop
        if (threadIdx.x == 0) gicp_make_trial(gc.sys, lam, gc.R0, gc.t0, cur);
        __syncthreads();
        double tot = 0.0;
        for (int q = 0; q < ns; ++q) {
            double e[1] = {0.0};
            const int hi = min(v.n, (q + 1) * v.ps);
            for (int i = q * v.ps + threadIdx.x; i < hi; i += kGicpSliceWG) {
                const NNKey kk = v.key[i];
                if (!((double)key_d2(kk) < g.max_d2)) continue;
                double M[9];
                sym_unpack(v.mah + (int64_t)i * 6, M);
                gicp_point<false>(v.src[i], v.tgt[key_idx(kk)], M, cur.R, cur.t, e);
            }
            tot += gicp_slice_sum(e, red);
        }
        if (threadIdx.x == 0) decide(tot);
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    GicpState& gs = g.gs[p];
    st.ncorr = (int)gc.sys[28];
    st.iterations = it;  // nr_iterations_ = i
    gs.lambda = lam;
    for (int k = 0; k < 9; ++k) gs.R[k] = x0[k];
    for (int k = 0; k < 3; ++k) gs.t[k] = x0[9 + k];
    // final_transformation_ = x0.cast<float>() (column-major)
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) st.final_T[4 * c + r] = (float)x0[3 * r + c];
        st.final_T[12 + r] = (float)x0[9 + r];
        st.final_T[4 * r + 3] = 0.0f;
    }
    st.final_T[15] = 1.0f;
    if (!stop) {
        st.phase = kPhaseFailed;  // step_lm returned false: "lm not converged!!", break
    } else if (gicp_converged(cur.dR, cur.dt, g.rot_eps, g.trans_eps)) {
        st.phase = kPhaseConverged;
        st.conv_state = 2;
    } else if (it + 1 >= g.max_iterations) {
        st.conv_state = 1;
    }
}

// (3) X := trans.cast<float>() * src over one slice for the next NN pass (float, Eigen's order), for the
// pairs still iterating
__global__ __launch_bounds__(kGicpSliceWG) void gicp_move_kernel(PairArgs a, WorkArgs w, GicpArgs g, int npairs, int W) {
    int p, j;
    if (!gicp_block(npairs, W, p, j)) return;
    if (w.state[p].phase != kPhaseActive) return;
    const GicpPairView v = gicp_view(a, w, g, p);
    const GicpState& gs = g.gs[p];
    float Rf[9], tf[3];
    for (int k = 0; k < 9; ++k) Rf[k] = (float)gs.R[k];
    for (int k = 0; k < 3; ++k) tf[k] = (float)gs.t[k];
    float4* X = w.X + (int64_t)p * w.x_stride;
    for (int i = j * kGicpSliceWG + threadIdx.x; i < v.n; i += W * kGicpSliceWG) {
        const float4 sp = v.src[i];
        float o[3];
        for (int r = 0; r < 3; ++r) {
            float x = Rf[3 * r] * sp.x;
            x = x + Rf[3 * r + 1] * sp.y;
            x = x + Rf[3 * r + 2] * sp.z;
            o[r] = x + tf[r];
        }
        X[i] = make_float4(o[0], o[1], o[2], sp.w);
    }
}

__global__ void gicp_init_kernel(const float* guess, GicpState* gs, int npairs) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npairs) return;
    GicpState& s = gs[p];
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) s.R[3 * r + c] = guess ? (double)guess[(int64_t)p * 16 + 4 * c + r] : (r == c ? 1.0 : 0.0);
        s.t[r] = guess ? (double)guess[(int64_t)p * 16 + 12 + r] : 0.0;
    }
    s.lambda = -1.0;
}

// number of pairs still iterating -> *out, and (host_out) with a system-scope store into pinned host
// memory the host polls (the host's early exit between runs of iterations)
__global__ void gicp_active_kernel(const PairState* st, int npairs, int32_t* out, int64_t* host_out, uint32_t seq) {
    __shared__ int32_t tot;
    if (threadIdx.x == 0) tot = 0;
    __syncthreads();
    int c = 0;
    for (int p = threadIdx.x; p < npairs; p += blockDim.x) c += st[p].phase == kPhaseActive;
    if (c) atomicAdd(&tot, c);
    __syncthreads();
    if (threadIdx.x == 0) {
        *out = tot;
        if (host_out)
            __hip_atomic_store(host_out, (int64_t)(((uint64_t)seq << 32) | (uint32_t)tot), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t launch_gicp_active(const PairState* st, int npairs, int32_t* out, int64_t* host_out, uint32_t seq,
                              hipStream_t s) {
    hipLaunchKernelGGL(gicp_active_kernel, dim3(1), dim3(1024), 0, s, st, npairs, out, host_out, seq);
    return hipGetLastError();
}

hipError_t launch_gicp_init(const float* guess, GicpState* gs, int npairs, hipStream_t st) {
    hipLaunchKernelGGL(gicp_init_kernel, dim3((npairs + 255) / 256), dim3(256), 0, st, guess, gs, npairs);
    return hipGetLastError();
}

// lanes per query: up to 8 while the grid stays within kGicpKnnWaves waves (0: this rule)
static int knn_lanes(int lanes, int npairs, int max_n) {
    if (lanes != 0) return lanes;
    const int64_t waves1 = (int64_t)npairs * ((max_n + 63) / 64);
    lanes = 1;
    while (lanes < 8 && waves1 * lanes * 2 <= kGicpKnnWaves) lanes *= 2;
    return lanes;
}

#define ICP4R_COV_LANES(KERNEL, KK, ...)                                                                  \
    switch (lanes) {                                                                                     \
        case 1: hipLaunchKernelGGL((KERNEL<KK, 1>), grid, block, 0, st, __VA_ARGS__); break;             \
        case 2: hipLaunchKernelGGL((KERNEL<KK, 2>), grid, block, 0, st, __VA_ARGS__); break;             \
        case 4: hipLaunchKernelGGL((KERNEL<KK, 4>), grid, block, 0, st, __VA_ARGS__); break;             \
        default: hipLaunchKernelGGL((KERNEL<KK, 8>), grid, block, 0, st, __VA_ARGS__); break;            \
    }
// the list length K is the next instantiated size >= k: the node's k = 5 and fast_gicp's default 20
// have their own (a longer list costs insertion work and loosens the K-th-best pruning bound)
#define ICP4R_COV_K(KERNEL, ...)                 \
    if (k <= 5) {                                \
        ICP4R_COV_LANES(KERNEL, 5, __VA_ARGS__)  \
    } else if (k <= 8) {                         \
        ICP4R_COV_LANES(KERNEL, 8, __VA_ARGS__)  \
    } else if (k <= 16) {                        \
        ICP4R_COV_LANES(KERNEL, 16, __VA_ARGS__) \
    } else if (k <= 20) {                        \
        ICP4R_COV_LANES(KERNEL, 20, __VA_ARGS__) \
    } else if (k <= 32) {                        \
        ICP4R_COV_LANES(KERNEL, 32, __VA_ARGS__) \
    } else {                                     \
        return hipErrorInvalidValue;             \
    }

hipError_t launch_gicp_cov(const float4* cloud, const int64_t* off, const int32_t* cnt, int npairs, int max_n,
                           int64_t stride, int k, int reg, double* cov, int lanes, hipStream_t st) {
    if (npairs <= 0 || max_n <= 0) return hipSuccess;
    lanes = knn_lanes(lanes, npairs, max_n);
    if (lanes != 1 && lanes != 2 && lanes != 4 && lanes != 8) return hipErrorInvalidValue;
    const int qpw = kCovWG / lanes;
    const dim3 grid((max_n + qpw - 1) / qpw, npairs), block(kCovWG);
    ICP4R_COV_K(gicp_cov_kernel, cloud, off, cnt, stride, k, reg, cov)
    return hipGetLastError();
}

hipError_t launch_gicp_knn_cov(const float4* cloud, const int64_t* off, const int32_t* cnt, const WorkArgs& w,
                               int npairs, int max_n, int64_t stride, int k, int reg, double* cov, int lanes,
                               hipStream_t st) {
    if (npairs <= 0 || max_n <= 0) return hipSuccess;
    if (w.leaf != 16) return hipErrorInvalidValue;
    // (a single 8k scan: 128 waves at one lane per query; the map call's two clouds 1.42 -> 1.29 ms at 8
    // lanes, while a 256-pair batch, 32k waves, ran 1.57 -> 4.57 ms of covariances at 8)
    lanes = knn_lanes(lanes, npairs, max_n);
    if (lanes != 1 && lanes != 2 && lanes != 4 && lanes != 8) return hipErrorInvalidValue;
    const int qpw = kCovWG / lanes;  // queries per workgroup
    const dim3 grid((max_n + qpw - 1) / qpw, npairs), block(kCovWG);
    ICP4R_COV_K(gicp_knn_cov_kernel, cloud, off, cnt, w, stride, k, reg, cov)
    return hipGetLastError();
}
#undef ICP4R_COV_K
#undef ICP4R_COV_LANES

hipError_t launch_gicp_iter(const PairArgs& a, const WorkArgs& w, const GicpArgs& g, int npairs, int max_n, int it,
                            hipStream_t st) {
    if (npairs <= 0) return hipSuccess;
    // about g.grid workgroups in all (a single pair: one per slice)
    const int ns = gicp_slices(max_n);
    const int per = g.grid / npairs;
    const int W = per < 1 ? 1 : per > ns ? ns : per;
    const dim3 grid((unsigned)W * ((npairs + 7) / 8 * 8)), block(kGicpSliceWG);
    hipLaunchKernelGGL(gicp_lin_kernel, grid, block, 0, st, a, w, g, npairs, W);
    hipLaunchKernelGGL(gicp_trial_kernel, grid, block, 0, st, a, w, g, npairs, W, it);
    hipLaunchKernelGGL(gicp_move_kernel, grid, block, 0, st, a, w, g, npairs, W);
    return hipGetLastError();
}

}  // namespace icp4r
