// icp4r_kernels.hip — HIP kernels for gfx950 (MI355X): device-resident PCL ICP over many pairs.
//
// One registration = SURVEY.md §3.2 / Appendix A.  The loop runs entirely on the device as a fixed
// sequence of launches on one stream (no host synchronisation, per-pair early-exit flags):
//
//   init_kernel                      validate, X := guess * src (or src), final := guess
//   repeat max_iterations times:
//     nn_kernel<Q>                   exact 1-NN of every X_i in the pair's target      (HOT: FP32 VALU)
//     update_kernel<NUM>             correspondences -> Umeyama moments -> 3x3 solve ->
//                                    hasConverged -> X := T_inc * X in place (PCL transformCloud)
//   fitness_prep_kernel              X := final * src
//   nn_kernel<Q>                     fitness pass (getFitnessScore)
//   finish_kernel                    mean d² over d² <= max_range, results, aligned output
//
// The hot kernel holds Q queries per lane in VGPRs and streams the target cloud through the SCALAR
// cache: the target address is wave-uniform, so each target point lands in SGPRs and is broadcast
// to 64 lanes x Q queries with no LDS traffic and no VGPRs.  Per (query, target) the VALU executes
// 3 sub + 3 mul + 2 add (FLANN's L2_Simple, unfused) + 1 cmp + 2 cndmask.  Splitting the serial
// solve into its own kernel keeps the sweep at <= 128 VGPRs (4 waves/SIMD).
//
// Determinism: fixed-order reductions only (xor-butterfly per wave, waves in index order, splits
// in index order); no float atomics.  NN ties resolve to the lowest target index.
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "icp4r_internal.hpp"
#include "icp4r_math.hpp"

namespace icp4r {

using v4f = float __attribute__((ext_vector_type(4)));
// Target pointers are re-typed into the AMDGPU constant address space (4): with a wave-uniform
// address every load becomes an s_load (scalar cache -> SGPRs) whatever alias analysis can prove.
using cv4f_ptr = const __attribute__((address_space(4))) v4f*;

// The address is also made PROVABLY wave-uniform (readfirstlane of both halves, once), so hipcc
// keeps it in SGPRs instead of re-reading it with v_readfirstlane inside the sweep loop.
__device__ __forceinline__ cv4f_ptr as_const(const float4* p) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return reinterpret_cast<cv4f_ptr>(((uint64_t)hi << 32) | lo);
}

// Wave-uniform scalar reads of per-pair metadata (read-only during a launch) via s_load, so counts,
// offsets and loop bounds stay in SGPRs.
template <typename T>
__device__ __forceinline__ T uload(const T* p) {
    return *reinterpret_cast<const __attribute__((address_space(4))) T*>(reinterpret_cast<uintptr_t>(p));
}

// ---------------------------------------------------------------------------------------------
// Exact brute-force 1-NN of Q register-resident queries per lane over targets [j0, j1) of a
// wave-uniform target array; increasing index order and strict '<' => lowest index wins ties.
template <int Q>
__device__ __forceinline__ void nn_sweep(const float (&x)[Q], const float (&y)[Q], const float (&z)[Q],
                                         const float4* tgt_generic, int j0, int j1, float (&best)[Q],
                                         int (&bi)[Q]) {
    const cv4f_ptr tgt = as_const(tgt_generic);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        best[q] = INFINITY;
        bi[q] = j0;
    }
    // 4 targets per trip (one s_load_dwordx16).  The last partial group re-reads target j1-1 in
    // its empty slots: a duplicate can never beat its own first occurrence under strict '<', so
    // no tail loop is needed (a tail loop — like a rotated prefetch — made hipcc keep two copies
    // of `best`, i.e. 12 instead of 11 VALU ops per pair).  Requires j1 > j0.
    const int last = j1 - 1;
    for (int j = j0; j < j1; j += 4) {
        const v4f c[4] = {tgt[j], tgt[min(j + 1, last)], tgt[min(j + 2, last)], tgt[min(j + 3, last)]};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const float d = l2_simple(x[q], y[q], z[q], c[t].x, c[t].y, c[t].z);
                if (d < best[q]) {
                    best[q] = d;
                    bi[q] = j + t;
                }
            }
        }
    }
}

// Packed variant: two queries per v2f register pair, so the 8 arithmetic ops per pair issue as
// 4 v_pk_{add,mul}_f32 per (query-pair, target) — identical IEEE results per component (unfused,
// -ffp-contract=off) to the scalar form.  Compare/select stays scalar (no packed cmp on gfx950).
using v2f = float __attribute__((ext_vector_type(2)));

template <int Q>
__device__ __forceinline__ void nn_sweep_packed(const float (&x)[Q], const float (&y)[Q], const float (&z)[Q],
                                                const float4* tgt_generic, int j0, int j1, float (&best)[Q],
                                                int (&bi)[Q]) {
    static_assert(Q % 2 == 0, "packed sweep needs an even Q");
    constexpr int H = Q / 2;
    const cv4f_ptr tgt = as_const(tgt_generic);
    v2f px[H], py[H], pz[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
        px[h] = v2f{x[2 * h], x[2 * h + 1]};
        py[h] = v2f{y[2 * h], y[2 * h + 1]};
        pz[h] = v2f{z[2 * h], z[2 * h + 1]};
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        best[q] = INFINITY;
        bi[q] = j0;
    }
    const int last = j1 - 1;
    for (int j = j0; j < j1; j += 4) {
        const v4f c[4] = {tgt[j], tgt[min(j + 1, last)], tgt[min(j + 2, last)], tgt[min(j + 3, last)]};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const v2f tx = v2f{c[t].x, c[t].x}, ty = v2f{c[t].y, c[t].y}, tz = v2f{c[t].z, c[t].z};
#pragma unroll
            for (int h = 0; h < H; ++h) {
                const v2f d0 = px[h] - tx;
                v2f r = d0 * d0;
                const v2f d1 = py[h] - ty;
                r = r + d1 * d1;
                const v2f d2 = pz[h] - tz;
                r = r + d2 * d2;
                if (r.x < best[2 * h]) {
                    best[2 * h] = r.x;
                    bi[2 * h] = j + t;
                }
                if (r.y < best[2 * h + 1]) {
                    best[2 * h + 1] = r.y;
                    bi[2 * h + 1] = j + t;
                }
            }
        }
    }
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Sum N doubles over a workgroup of NW waves in a fixed order (xor-butterfly per wave, then waves
// in index order by thread k for component k); totals land in `out` (LDS).
template <int N, int NW>
__device__ __forceinline__ void block_sum(double (&v)[N], double* sh /* [NW*N] */, double* out /* [N] */) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < N; ++k) sh[wave * N + k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x < N) {
        double t = 0.0;
        for (int w = 0; w < NW; ++w) t += sh[w * N + threadIdx.x];
        out[threadIdx.x] = t;
    }
    __syncthreads();
}

__device__ __forceinline__ double huber_w(float d2, double delta) {
    const double r = sqrt((double)d2);
    return r <= delta ? 1.0 : delta / r;
}

// Per-query NN result merged over target splits: lexicographic (d², index) minimum == the
// unsplit sweep's answer (lowest index among equal distances).
__device__ __forceinline__ void merge_nn(const WorkArgs& w, int64_t slot, float& d2, int& idx) {
    d2 = w.nn_d2[slot];
    idx = w.nn_idx[slot];
    for (int s = 1; s < w.splits; ++s) {
        const float d = w.nn_d2[slot + (int64_t)s * w.slot_stride];
        const int j = w.nn_idx[slot + (int64_t)s * w.slot_stride];
        if (d < d2 || (d == d2 && j < idx)) {
            d2 = d;
            idx = j;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// init_kernel: one workgroup per pair.
constexpr int kInitWG = 256;
__global__ __launch_bounds__(kInitWG) void init_kernel(PairArgs a, WorkArgs w) {
    __shared__ float Tg[16];
    __shared__ int ident;
    const int p = blockIdx.x;
    const int tid = threadIdx.x;
    const int n = a.src_n[p], m = a.tgt_n[p];
    const float4* src = a.src + a.src_off[p];
    const float4* tgt = a.tgt + a.tgt_off[p];
    PairState& st = w.state[p];
    int bad = 0;
    for (int i = tid; i < m; i += kInitWG) {
        const float4 t = tgt[i];
        bad |= !(isfinite(t.x) && isfinite(t.y) && isfinite(t.z));
    }
    for (int i = tid; i < n; i += kInitWG) {
        const float4 s = src[i];
        bad |= !(isfinite(s.x) && isfinite(s.y) && isfinite(s.z));
    }
    bad = __syncthreads_or(bad);
    if (tid == 0) {
        bool id = true;
        for (int k = 0; k < 16; ++k) {
            const float g = a.guess ? a.guess[(int64_t)p * 16 + k] : ((k % 5 == 0) ? 1.0f : 0.0f);
            Tg[k] = g;
            id = id && (g == ((k % 5 == 0) ? 1.0f : 0.0f));
        }
        ident = id ? 1 : 0;
        mat4_identity(st.T_inc);
        st.prev_mse = DBL_MAX;
        st.similar = 0;
        st.conv_state = 0;
        st.iterations = 0;
        st.ncorr = 0;
        if (m <= 0 || bad) {
            // Registration::initCompute fails (no target) -> align returns; final stays identity.
            mat4_identity(st.final_T);
            st.phase = kPhaseInvalid;
            st.status = m <= 0 ? kStatusEmpty : kStatusNonFinite;
        } else {
            for (int k = 0; k < 16; ++k) st.final_T[k] = Tg[k];  // final_transformation_ = guess
            st.phase = kPhaseActive;
            st.status = 0;
        }
    }
    __syncthreads();
    if (m <= 0 || bad) return;
    float4* X = w.X + (int64_t)p * w.x_stride;
    const bool id = ident != 0;
    for (int i = tid; i < n; i += kInitWG) {
        const float4 s = src[i];
        float4 o = s;
        if (!id) xform_pt(Tg, s.x, s.y, s.z, o.x, o.y, o.z);  // transformCloud(input, guess)
        X[i] = o;
    }
}

// ---------------------------------------------------------------------------------------------
// nn_kernel<Q>: blockIdx.x = query block (WG*Q queries), blockIdx.y = pair, blockIdx.z = target
// split.  Writes the (d², index) of each query's nearest target in the split's index range.
template <int Q, bool PACKED>
__global__ __launch_bounds__(kNNWG) void nn_kernel(PairArgs a, WorkArgs w, int fitness_pass) {
    const int p = blockIdx.y;
    const int phase = uload(&w.state[p].phase);
    if (fitness_pass ? (phase == kPhaseInvalid) : (phase != kPhaseActive)) return;
    const int n = uload(a.src_n + p), m = uload(a.tgt_n + p);
    const int base = blockIdx.x * (kNNWG * Q);
    if (base >= n) return;
    const int s = blockIdx.z;
    const int j0 = (int)(((int64_t)m * s) / w.splits), j1 = (int)(((int64_t)m * (s + 1)) / w.splits);
    const float4* X = w.X + (int64_t)p * w.x_stride;
    float x[Q], y[Q], z[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int i = base + threadIdx.x + q * kNNWG;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < n) v = X[i];
        x[q] = v.x;
        y[q] = v.y;
        z[q] = v.z;
    }
    float best[Q];
    int bi[Q];
    if constexpr (PACKED)
            nn_sweep_packed<Q>(x, y, z, a.tgt + uload(a.tgt_off + p), j0, j1, best, bi);
    else
        nn_sweep<Q>(x, y, z, a.tgt + uload(a.tgt_off + p), j0, j1, best, bi);
    const int64_t slot0 = (int64_t)s * w.slot_stride + (int64_t)p * w.x_stride;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int i = base + threadIdx.x + q * kNNWG;
        if (i < n) {
            w.nn_d2[slot0 + i] = best[q];
            w.nn_idx[slot0 + i] = bi[q];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Sequential folds over an LDS chunk, one lane per chain.  The order of the additions is exactly
// the reference loop's; the loads are issued 16 ahead (ds_read_b128) so the chain runs at the
// dependent-add latency instead of the LDS round trip per element.
__device__ __forceinline__ float fold_f32(const float* f, int len, float acc) {
    int k = 0;
    for (; k + 16 <= len; k += 16) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(f + k + 4 * u);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            acc = acc + v[u].x;
            acc = acc + v[u].y;
            acc = acc + v[u].z;
            acc = acc + v[u].w;
        }
    }
    for (; k < len; ++k) acc = acc + f[k];
    return acc;
}

__device__ __forceinline__ double fold_f64(const double* f, int len, double acc) {
    int k = 0;
    for (; k + 8 <= len; k += 8) {
        double2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const double2*>(f + k + 2 * u);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            acc = acc + v[u].x;
            acc = acc + v[u].y;
        }
    }
    for (; k < len; ++k) acc = acc + f[k];
    return acc;
}

// sigma chain: acc = a*b + acc (oracle umeyama_f32, unweighted)
__device__ __forceinline__ float fold_prod_f32(const float* fa, const float* fb, int len, float acc) {
    int k = 0;
    for (; k + 8 <= len; k += 8) {
        float4 a[2], b[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            a[u] = *reinterpret_cast<const float4*>(fa + k + 4 * u);
            b[u] = *reinterpret_cast<const float4*>(fb + k + 4 * u);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            acc = a[u].x * b[u].x + acc;
            acc = a[u].y * b[u].y + acc;
            acc = a[u].z * b[u].z + acc;
            acc = a[u].w * b[u].w + acc;
        }
    }
    for (; k < len; ++k) acc = fa[k] * fb[k] + acc;
    return acc;
}

// Huber sigma chain: acc = acc + (w*a)*b (oracle umeyama_f32, weighted)
__device__ __forceinline__ float fold_wprod_f32(const float* fw, const float* fa, const float* fb, int len, float acc) {
    int k = 0;
    for (; k + 4 <= len; k += 4) {
        const float4 w = *reinterpret_cast<const float4*>(fw + k);
        const float4 a = *reinterpret_cast<const float4*>(fa + k);
        const float4 b = *reinterpret_cast<const float4*>(fb + k);
        acc = acc + w.x * a.x * b.x;
        acc = acc + w.y * a.y * b.y;
        acc = acc + w.z * a.z * b.z;
        acc = acc + w.w * a.w * b.w;
    }
    for (; k < len; ++k) acc = acc + fw[k] * fa[k] * fb[k];
    return acc;
}

// ---------------------------------------------------------------------------------------------
// update_kernel<NUM>: one workgroup per active pair: correspondences -> moments -> solve ->
// convergence -> X := T_inc * X (in place, float, PCL transformCloud order).
constexpr int kUpdWG = 512;
constexpr int kUpdWaves = kUpdWG / 64;
constexpr int kFoldCh = 7;  // fold chains: s.xyz, d.xyz, weight (== validity when unweighted)

template <int NUM> struct MomLayout;
template <> struct MomLayout<kNumericsPCL> {  // |C| only: every other sum is a sequential fold
    static constexpr int N = 1, CNT = 0;
};
template <> struct MomLayout<kNumericsF64> {  // Σ w·d·sᵀ [9], Σ w·s [3], Σ w·d [3], Σ w, Σ d², |C|
    static constexpr int N = 18, MSE = 16, CNT = 17;
};

struct UpdShared {
    float fold[kFoldCh + 2][kFoldChunk];  // pass A: 7 float chains; pass B: s'xyz, d'xyz, w
    double dfold[kFoldChunk];             // pass A: d² (MSE chain, double)
    double red[kUpdWaves * 20];
    double mom[20];
    double sigma[9], ms[3], md[3];
    SvdWork svd;
    SvdWorkF svdf;
    float sigmaf[9];
    float mean[6];
    float one_over_n;
    double mse_sum;
    float T_inc[16];
    int32_t flag;  // 0 continue, 1 error (no transform), 2 converged after this transform
};

// Thread 0: count check, Umeyama solve, final := T_inc * final, hasConverged (all in LDS/state).
template <int NUM>
__device__ void solve_pair(UpdShared& sh, PairState& st, const KParams& kp) {
    constexpr int I_CNT = MomLayout<NUM>::CNT;
    const int cnt = (int)sh.mom[I_CNT];
    st.ncorr = cnt;
    if (cnt < kp.min_corr) {
        // PCL_ERROR "Not enough correspondences found. Relax your threshold parameters."
        st.phase = kPhaseFailed;
        st.status = kStatusTooFewCorr;
        st.conv_state = 5;  // CONVERGENCE_CRITERIA_NO_CORRESPONDENCES
        sh.flag = 1;
        return;
    }
    float* Tinc = sh.T_inc;
    mat4_identity(Tinc);
    double mse;
    if constexpr (NUM == kNumericsPCL) {
        // Eigen umeyama, Scalar = float: sigma = one_over_n * Σ d' s'ᵀ (the fold above), float SVD,
        // R as Matrix4f, Rt.col(3) = dst_mean; Rt.col(3) -= R * src_mean.
        for (int k = 0; k < 9; ++k) sh.sigmaf[k] = sh.one_over_n * sh.sigmaf[k];
        umeyama_rotation_f32(sh.sigmaf, sh.svdf);
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) Tinc[j * 4 + i] = sh.svdf.R[i * 3 + j];
            float rs = sh.svdf.R[i * 3 + 0] * sh.mean[0];
            rs = sh.svdf.R[i * 3 + 1] * sh.mean[1] + rs;
            rs = sh.svdf.R[i * 3 + 2] * sh.mean[2] + rs;
            Tinc[12 + i] = sh.mean[3 + i] - rs;
        }
        mse = sh.mse_sum / (double)cnt;  // calculateMSE: sequential double sum / |C|
    } else {
        const double sw = sh.mom[15];
        for (int k = 0; k < 3; ++k) {
            sh.ms[k] = sh.mom[9 + k] / sw;
            sh.md[k] = sh.mom[12 + k] / sw;
        }
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) sh.sigma[i * 3 + j] = sh.mom[i * 3 + j] / sw - sh.md[i] * sh.ms[j];
        umeyama_rotation(sh.sigma, sh.svd);
        const double* R = sh.svd.R;
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) Tinc[j * 4 + i] = (float)R[i * 3 + j];
            Tinc[12 + i] = (float)(sh.md[i] - (R[i * 3 + 0] * sh.ms[0] + R[i * 3 + 1] * sh.ms[1] + R[i * 3 + 2] * sh.ms[2]));
        }
        mse = sh.mom[MomLayout<kNumericsF64>::MSE] / (double)cnt;
    }
    for (int k = 0; k < 16; ++k) st.T_inc[k] = Tinc[k];
    mat4_mul_f(Tinc, st.final_T, st.final_T);  // final_transformation_ = transformation_ * final
    st.iterations += 1;
    ConvState cs;
    cs.prev_mse = st.prev_mse;
    cs.similar = st.similar;
    cs.state = st.conv_state;
    const int conv = has_converged(kp.conv, st.iterations, Tinc, mse, cs);
    st.prev_mse = cs.prev_mse;
    st.similar = cs.similar;
    st.conv_state = cs.state;
    if (conv) st.phase = kPhaseConverged;
    sh.flag = conv ? 2 : 0;
}

template <int NUM>
__global__ __launch_bounds__(kUpdWG) void update_kernel(PairArgs a, WorkArgs w) {
    constexpr int NM = MomLayout<NUM>::N;
    constexpr int I_CNT = MomLayout<NUM>::CNT;
    __shared__ UpdShared sh;
    const int p = blockIdx.x;
    PairState& st = w.state[p];
    if (st.phase != kPhaseActive) return;
    const int tid = threadIdx.x;
    const int n = a.src_n[p];
    const float4* tgt = a.tgt + a.tgt_off[p];
    float4* X = w.X + (int64_t)p * w.x_stride;
    const int64_t slot0 = (int64_t)p * w.x_stride;
    const KParams& kp = a.kp;
    const bool weighted = kp.huber_delta < INFINITY;

    double mom[NM];
#pragma unroll
    for (int k = 0; k < NM; ++k) mom[k] = 0.0;

    if constexpr (NUM == kNumericsPCL) {
        // Bit-exact float restatement of TransformationEstimationSVD (use_umeyama, Scalar = float)
        // and calculateMSE: every sum is the sequential fold the reference performs, in
        // correspondence (= source index) order, by one lane per chain of wave 0 over LDS chunks.
        //  pass A: Σs, Σd (Eigen 3.3 rowwise().sum(): fold from the first element == fold from -0.0f;
        //          Huber: fold of w·x from +0), Σw (== |C| unweighted), Σd² in double (MSE).
        //  pass B: Σ d'_a s'_b (sigma, float, from +0) over the float-demeaned points.
        // Rejected correspondences contribute the fold's identity (-0.0f / +0), i.e. nothing.
        const int lane = tid & 63, wave = tid >> 6;
        const float ident = weighted ? 0.0f : -0.0f;
        float acc = (lane < 6) ? ident : 0.0f;
        double dacc = 0.0;
        double cntd = 0.0;
        for (int base = 0; base < n; base += kFoldChunk) {
            for (int o = tid; o < kFoldChunk && base + o < n; o += kUpdWG) {
                const int i = base + o;
                float d2;
                int j;
                merge_nn(w, slot0 + i, d2, j);
                float wt = 0.f, sx = ident, sy = ident, sz = ident, dx = ident, dy = ident, dz = ident;
                double dd = 0.0;
                if (!(d2 > kp.max_d2)) {
                    const float4 s = X[i];
                    const float4 d = tgt[j];
                    if (weighted) {
                        wt = (float)huber_w(d2, kp.huber_delta);
                        sx = wt * s.x; sy = wt * s.y; sz = wt * s.z;
                        dx = wt * d.x; dy = wt * d.y; dz = wt * d.z;
                    } else {
                        wt = 1.0f;
                        sx = s.x; sy = s.y; sz = s.z;
                        dx = d.x; dy = d.y; dz = d.z;
                    }
                    dd = (double)d2;
                    cntd += 1.0;
                }
                sh.fold[0][o] = sx; sh.fold[1][o] = sy; sh.fold[2][o] = sz;
                sh.fold[3][o] = dx; sh.fold[4][o] = dy; sh.fold[5][o] = dz;
                sh.fold[6][o] = wt;
                sh.dfold[o] = dd;
            }
            __syncthreads();
            if (wave == 0 && lane < 8) {
                const int len = (n - base) < kFoldChunk ? (n - base) : kFoldChunk;
                if (lane < kFoldCh) {
                    acc = fold_f32(sh.fold[lane], len, acc);
                } else {
                    dacc = fold_f64(sh.dfold, len, dacc);
                }
            }
            __syncthreads();
        }
        mom[I_CNT] = cntd;
        if (wave == 0 && lane < kFoldCh) sh.fold[lane][0] = acc;
        if (wave == 0 && lane == 7) sh.mse_sum = dacc;
        __syncthreads();
        if (tid == 0) {
            // unweighted: one_over_n = 1/(float)n (fold of 1.0f == n exactly); Huber: 1/Σw
            const float one_over_n = 1.0f / sh.fold[6][0];
            sh.one_over_n = one_over_n;
            for (int c = 0; c < 6; ++c) sh.mean[c] = sh.fold[c][0] * one_over_n;
        }
        __syncthreads();
        const float msx = sh.mean[0], msy = sh.mean[1], msz = sh.mean[2];
        const float mdx = sh.mean[3], mdy = sh.mean[4], mdz = sh.mean[5];
        float sacc = 0.0f;  // lane a*3+b of wave 0: sigma(a, b)
        const int ca = lane / 3, cb = lane % 3;
        for (int base = 0; base < n; base += kFoldChunk) {
            for (int o = tid; o < kFoldChunk && base + o < n; o += kUpdWG) {
                const int i = base + o;
                float d2;
                int j;
                merge_nn(w, slot0 + i, d2, j);
                float wt = 0.f, s0 = 0.f, s1 = 0.f, s2 = 0.f, d0 = 0.f, d1 = 0.f, dv2 = 0.f;
                if (!(d2 > kp.max_d2)) {
                    const float4 s = X[i];
                    const float4 d = tgt[j];
                    s0 = s.x - msx; s1 = s.y - msy; s2 = s.z - msz;
                    d0 = d.x - mdx; d1 = d.y - mdy; dv2 = d.z - mdz;
                    wt = weighted ? (float)huber_w(d2, kp.huber_delta) : 1.0f;
                }
                sh.fold[0][o] = s0; sh.fold[1][o] = s1; sh.fold[2][o] = s2;
                sh.fold[3][o] = d0; sh.fold[4][o] = d1; sh.fold[5][o] = dv2;
                sh.fold[6][o] = wt;
            }
            __syncthreads();
            if (wave == 0 && lane < 9) {
                const int len = (n - base) < kFoldChunk ? (n - base) : kFoldChunk;
                const float* fa = sh.fold[3 + ca];
                const float* fb = sh.fold[cb];
                if (weighted)
                    sacc = fold_wprod_f32(sh.fold[6], fa, fb, len, sacc);
                else
                    sacc = fold_prod_f32(fa, fb, len, sacc);
            }
            __syncthreads();
        }
        if (wave == 0 && lane < 9) sh.sigmaf[lane] = sacc;
    } else {
        for (int i = tid; i < n; i += kUpdWG) {
            float d2;
            int j;
            merge_nn(w, slot0 + i, d2, j);
            if (d2 > kp.max_d2) continue;
            const float4 s = X[i];
            const float4 d = tgt[j];
            const double wt = weighted ? huber_w(d2, kp.huber_delta) : 1.0;
            const double s0 = s.x, s1 = s.y, s2 = s.z;
            const double w0 = wt * (double)d.x, w1 = wt * (double)d.y, w2 = wt * (double)d.z;
            mom[0] += w0 * s0; mom[1] += w0 * s1; mom[2] += w0 * s2;
            mom[3] += w1 * s0; mom[4] += w1 * s1; mom[5] += w1 * s2;
            mom[6] += w2 * s0; mom[7] += w2 * s1; mom[8] += w2 * s2;
            mom[9] += wt * s0; mom[10] += wt * s1; mom[11] += wt * s2;
            mom[12] += w0; mom[13] += w1; mom[14] += w2;
            mom[15] += wt;
            mom[MomLayout<kNumericsF64>::MSE] += (double)d2;
            mom[I_CNT] += 1.0;
        }
    }
    block_sum<NM, kUpdWaves>(mom, sh.red, sh.mom);
    if (tid == 0) solve_pair<NUM>(sh, st, kp);
    __syncthreads();
    if (sh.flag == 1) return;  // error: PCL breaks before transforming
    // transformCloud(*input_transformed, *input_transformed, transformation_)
    float Tl[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) Tl[k] = sh.T_inc[k];
    for (int i = tid; i < n; i += kUpdWG) {
        float4 s = X[i];
        xform_pt(Tl, s.x, s.y, s.z, s.x, s.y, s.z);
        X[i] = s;
    }
}

// ---------------------------------------------------------------------------------------------
// fitness_prep_kernel: X := final * input (Registration::getFitnessScore / align's output).
__global__ __launch_bounds__(256) void fitness_prep_kernel(PairArgs a, WorkArgs w) {
    const int p = blockIdx.x;
    const PairState& st = w.state[p];
    if (st.phase == kPhaseInvalid) return;
    __shared__ float Tf[16];
    if (threadIdx.x < 16) Tf[threadIdx.x] = st.final_T[threadIdx.x];
    __syncthreads();
    const int n = a.src_n[p];
    const float4* src = a.src + a.src_off[p];
    float4* X = w.X + (int64_t)p * w.x_stride;
    for (int i = threadIdx.x; i < n; i += 256) {
        const float4 s = src[i];
        float4 o = s;
        xform_pt(Tf, s.x, s.y, s.z, o.x, o.y, o.z);
        X[i] = o;
    }
}

// finish_kernel: fitness = mean of d² over d² <= max_range (double), results, aligned output.
constexpr int kFinWG = 256;
__global__ __launch_bounds__(kFinWG) void finish_kernel(PairArgs a, WorkArgs w) {
    const int p = blockIdx.x;
    const PairState& st = w.state[p];
    const int n = a.src_n[p];
    const int64_t slot0 = (int64_t)p * w.x_stride;
    const bool have = st.phase != kPhaseInvalid && a.kp.compute_fitness && n > 0;
    // Registration::getFitnessScore: sequential double sum over points with d² <= max_range, in
    // index order (one lane over LDS chunks), so the score is bit-identical to the reference loop.
    __shared__ double chunk[kFoldChunk];
    double fsum = 0.0, fcnt = 0.0;
    if (have) {
        for (int base = 0; base < n; base += kFoldChunk) {
            for (int o = threadIdx.x; o < kFoldChunk && base + o < n; o += kFinWG) {
                float d2;
                int j;
                merge_nn(w, slot0 + base + o, d2, j);
                chunk[o] = ((double)d2 <= a.kp.fit_max_range) ? (double)d2 : -1.0;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                const int len = (n - base) < kFoldChunk ? (n - base) : kFoldChunk;
                int k = 0;
                for (; k + 8 <= len; k += 8) {  // loads hoisted ahead of the dependent adds
                    double v[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) v[u] = chunk[k + u];
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (v[u] >= 0.0) {
                            fsum = fsum + v[u];
                            fcnt += 1.0;
                        }
                }
                for (; k < len; ++k)
                    if (chunk[k] >= 0.0) {
                        fsum = fsum + chunk[k];
                        fcnt += 1.0;
                    }
            }
            __syncthreads();
        }
    }
    if (a.aligned && st.phase != kPhaseInvalid) {
        const float4* src = a.src + a.src_off[p];
        const float4* X = w.X + (int64_t)p * w.x_stride;
        float4* out = a.aligned + a.src_off[p];
        for (int i = threadIdx.x; i < n; i += kFinWG) {
            float4 v = X[i];
            v.w = src[i].w;  // intensity copied through
            out[i] = v;
        }
    }
    if (threadIdx.x == 0) {
        Result r;
        for (int k = 0; k < 16; ++k) r.T[k] = st.final_T[k];
        r.fitness = (have && fcnt > 0) ? fsum / fcnt : DBL_MAX;
        r.iterations = st.iterations;
        r.converged = st.phase == kPhaseConverged ? 1 : 0;
        r.status = st.status;
        r.convergence_state = st.conv_state;
        r.n_correspondences = st.ncorr;
        r.reserved = 0;
        a.results[p] = r;
    }
}

// ---------------------------------------------------------------------------------------------
// Standalone exact 1-NN (icp4r_nearest / icp4r_fitness): one query per thread, optional transform.
__global__ __launch_bounds__(256) void nn_query_kernel(const float4* __restrict__ q, int n, const float4* tgt, int m,
                                                       const float* __restrict__ T, int32_t* __restrict__ idx,
                                                       float* __restrict__ d2) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    float x[1], y[1], z[1];
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < n) s = q[i];
    if (T) {
        float Tl[16];
        for (int k = 0; k < 16; ++k) Tl[k] = T[k];
        xform_pt(Tl, s.x, s.y, s.z, x[0], y[0], z[0]);
    } else {
        x[0] = s.x;
        y[0] = s.y;
        z[0] = s.z;
    }
    float best[1];
    int bi[1];
    nn_sweep<1>(x, y, z, tgt, 0, m, best, bi);
    if (i < n) {
        idx[i] = bi[0];
        d2[i] = best[0];
    }
}

// Test hook: the device float Umeyama rotation for k sigma matrices (one thread each).
__global__ void rot_f32_kernel(const float* sigma, float* R, int k) {
    __shared__ SvdWorkF ws[64];
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= k) return;
    umeyama_rotation_f32(sigma + 9 * i, ws[threadIdx.x]);
    for (int e = 0; e < 9; ++e) R[9 * i + e] = ws[threadIdx.x].R[e];
}

hipError_t launch_rot_f32(const float* sigma, float* R, int k, hipStream_t st) {
    hipLaunchKernelGGL(rot_f32_kernel, dim3((k + 63) / 64), dim3(64), 0, st, sigma, R, k);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
hipError_t launch_init(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st) {
    hipLaunchKernelGGL(init_kernel, dim3(npairs), dim3(kInitWG), 0, st, a, w);
    return hipGetLastError();
}

hipError_t launch_nn(int q, bool packed, const PairArgs& a, const WorkArgs& w, int npairs, int max_n,
                     int fitness_pass, hipStream_t st) {
    const int per_block = kNNWG * q;
    const dim3 grid((max_n + per_block - 1) / per_block, npairs, w.splits), block(kNNWG);
#define ICP4R_NN_CASE(QQ, PP) hipLaunchKernelGGL((nn_kernel<QQ, PP>), grid, block, 0, st, a, w, fitness_pass)
    if (packed && q >= 2) {
        switch (q) {
            case 2: ICP4R_NN_CASE(2, true); break;
            case 4: ICP4R_NN_CASE(4, true); break;
            case 8: ICP4R_NN_CASE(8, true); break;
            case 16: ICP4R_NN_CASE(16, true); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (q) {
            case 1: ICP4R_NN_CASE(1, false); break;
            case 2: ICP4R_NN_CASE(2, false); break;
            case 4: ICP4R_NN_CASE(4, false); break;
            case 8: ICP4R_NN_CASE(8, false); break;
            case 16: ICP4R_NN_CASE(16, false); break;
            default: return hipErrorInvalidValue;
        }
    }
#undef ICP4R_NN_CASE
    return hipGetLastError();
}

hipError_t launch_update(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st) {
    if (a.kp.numerics == kNumericsPCL)
        hipLaunchKernelGGL(update_kernel<kNumericsPCL>, dim3(npairs), dim3(kUpdWG), 0, st, a, w);
    else
        hipLaunchKernelGGL(update_kernel<kNumericsF64>, dim3(npairs), dim3(kUpdWG), 0, st, a, w);
    return hipGetLastError();
}

hipError_t launch_fitness_prep(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st) {
    hipLaunchKernelGGL(fitness_prep_kernel, dim3(npairs), dim3(256), 0, st, a, w);
    return hipGetLastError();
}

hipError_t launch_finish(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st) {
    hipLaunchKernelGGL(finish_kernel, dim3(npairs), dim3(kFinWG), 0, st, a, w);
    return hipGetLastError();
}

hipError_t launch_nn_query(const float4* q, int n, const float4* tgt, int m, const float* T, int32_t* idx, float* d2,
                           hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(nn_query_kernel, dim3((n + 255) / 256), dim3(256), 0, st, q, n, tgt, m, T, idx, d2);
    return hipGetLastError();
}

}  // namespace icp4r
