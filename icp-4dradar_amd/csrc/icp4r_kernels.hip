// icp4r_kernels.hip — HIP kernels for gfx950 (MI355X): device-resident PCL ICP over many pairs.
//
// One registration = SURVEY.md §3.2 / Appendix A.  The loop runs entirely on the device as a fixed
// sequence of launches on one stream (no host synchronisation, per-pair early-exit flags):
//
//   init_kernel                      validate, X := guess * src (or src), final := guess
//   index_kernel                     (pruned mode) Morton counting sort of target and source,
//                                    target block / superblock bounding boxes
//   repeat max_iterations times:
//     nn_pruned_kernel<Q,B>          exact 1-NN of every X_i in the pair's target      (HOT: FP32 VALU)
//       or nn_kernel<Q>              (brute force: small targets / ICP4R_NN_BRUTE)
//     update_kernel<NUM>             correspondences -> Umeyama moments -> 3x3 solve ->
//                                    hasConverged -> X := T_inc * X in place (PCL transformCloud)
//   fitness_prep_kernel              X := final * src
//   NN pass                          fitness pass (getFitnessScore)
//   finish_kernel                    mean d² over d² <= max_range, results, aligned output
//
// Both NN kernels hold Q queries per lane in VGPRs and stream targets through the SCALAR cache:
// the target address is wave-uniform, so each target point lands in SGPRs and is broadcast to
// 64 lanes x Q queries with no LDS traffic and no VGPRs.  Per (query, target) the VALU executes
// 3 sub + 3 mul + 2 add (FLANN's L2_Simple, unfused) and a compare/select.  Every NN result is a
// u64 key (d² bits, target index) whose minimum is PCL's answer (lowest index among ties), so
// pruning, visiting order and target splits cannot change it.
//
// Determinism: fixed-order reductions only (xor-butterfly per wave, waves in index order, the
// PCL-numerics folds sequential in source order); no float atomics.
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "icp4r_device.hpp"
#include "icp4r_internal.hpp"
#include "icp4r_math.hpp"

namespace icp4r {

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

// Per-query NN result: one key (splits were merged by atomicMin on the key, i.e. the lexicographic
// (d², index) minimum == the unsplit sweep's answer).
__device__ __forceinline__ void load_nn(const WorkArgs& w, int64_t slot, float& d2, int& idx) {
    const NNKey k = w.nn_key[slot];
    d2 = key_d2(k);
    idx = key_idx(k);
}

// Correspondence records (PCL numerics): per source point, in source-index order (the fold order),
// two float4 at corr + (p*x_stride + i)*2: {s.xyz (the transformed source point searched with),
// w (Huber weight, 1 unweighted)}, {d.xyz (its nearest target), d² (float, as FLANN returned it)}.
// Written by the pruned NN kernel's tail, or by corr_kernel after a brute-force pass.
__device__ __forceinline__ void write_corr(const WorkArgs& w, const PairArgs& a, int p, int i, float sx, float sy,
                                           float sz, NNKey k, const float4* tgt) {
    float4* C = w.corr + ((int64_t)p * w.x_stride + i) * 2;
    const float d2 = key_d2(k);
    const float4 t = tgt[key_idx(k)];
    const float wt = a.kp.huber_delta < INFINITY ? (float)huber_w(d2, a.kp.huber_delta) : 1.0f;
    C[0] = make_float4(sx, sy, sz, wt);
    C[1] = make_float4(t.x, t.y, t.z, d2);
}

// ---------------------------------------------------------------------------------------------
// init_kernel: one workgroup per pair.
// WG threads per pair: 256 for batches (HBM-bound there), 1024 for a few pairs, whose validation
// passes are latency-bound rounds of loads (C5's 65k-point map: 16 rounds of 256 x 16 -> 4)
template <int kInitWG>
__global__ __launch_bounds__(kInitWG) void init_kernel(PairArgs a, WorkArgs w) {
    __shared__ float Tg[16];
    __shared__ int ident;
    const int p = xcd_remap(blockIdx.x, gridDim.x);
    const int tid = threadIdx.x;
    const int n = a.src_n[p], m = a.tgt_n[p];
    const float4* src = a.src + a.src_off[p];
    const float4* tgt = a.tgt + a.tgt_off[p];
    PairState& st = w.state[p];
    if (tid < 16) Tg[tid] = a.guess ? a.guess[(int64_t)p * 16 + tid] : ((tid % 5 == 0) ? 1.0f : 0.0f);
    __syncthreads();
    if (tid == 0) {
        bool id = true;
        for (int k = 0; k < 16; ++k) id = id && (Tg[k] == ((k % 5 == 0) ? 1.0f : 0.0f));
        ident = id ? 1 : 0;
    }
    __syncthreads();
    // One pass over the source: validated and written transformed (transformCloud(input, guess)) in
    // the same read — X of a pair found invalid below is never read.  Counts above the workspace
    // stride are not copied (too_big below marks the pair invalid).  kInitPer points per thread in
    // flight, every load of a round before its stores.
    constexpr int kInitPer = 4;
    float4* X = w.X + (int64_t)p * w.x_stride;
    const bool id = ident != 0;
    const int nc = min(n, (int)w.x_stride);
    int bad = 0;
    // coordinates beyond 1e17 could square into an overflowing (inf) distance, which PCL rejects: such
    // a pair never skips pass A's distance check (PairState::sums_ok = -1)
    constexpr float kBig = 1e17f;
    int big = 0;
    // (the target is only validated: 16 points per thread in flight — a scan-to-map target of 65k
    // points had taken 64 dependent rounds of 1024, ~65 us of a single registration)
    // (and its bounding box, for the Morton index of a large target: w.tbb)
    constexpr int kTgtPer = 16;
    float bl[3] = {INFINITY, INFINITY, INFINITY}, bh[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i0 = 0; i0 < m; i0 += kInitWG * kTgtPer) {
        float4 t[kTgtPer];
#pragma unroll
        for (int e = 0; e < kTgtPer; ++e) t[e] = tgt[min(i0 + e * kInitWG + tid, m - 1)];
#pragma unroll
        for (int e = 0; e < kTgtPer; ++e) {  // (a clamped duplicate of point m - 1 changes no extent)
            bad |= !(isfinite(t[e].x) && isfinite(t[e].y) && isfinite(t[e].z));
            big |= fmaxf(fabsf(t[e].x), fmaxf(fabsf(t[e].y), fabsf(t[e].z))) > kBig;
            bl[0] = fminf(bl[0], t[e].x); bl[1] = fminf(bl[1], t[e].y); bl[2] = fminf(bl[2], t[e].z);
            bh[0] = fmaxf(bh[0], t[e].x); bh[1] = fmaxf(bh[1], t[e].y); bh[2] = fmaxf(bh[2], t[e].z);
        }
    }
    if (w.tbb) {
        __shared__ float bred[kInitWG / 64][6];
#pragma unroll
        for (int k = 0; k < 3; ++k) {  // (DPP)
            bl[k] = wave_minf(bl[k]);
            bh[k] = wave_maxf(bh[k]);
        }
        if ((tid & 63) == 0)
            for (int k = 0; k < 3; ++k) {
                bred[tid >> 6][k] = bl[k];
                bred[tid >> 6][3 + k] = bh[k];
            }
        __syncthreads();
        if (tid < 6) {
            float v = bred[0][tid];
            for (int q = 1; q < kInitWG / 64; ++q) v = tid < 3 ? fminf(v, bred[q][tid]) : fmaxf(v, bred[q][tid]);
            w.tbb[(int64_t)p * 8 + tid] = v;
        }
    }
    for (int i0 = 0; i0 < n; i0 += kInitWG * kInitPer) {
        float4 v[kInitPer];
#pragma unroll
        for (int e = 0; e < kInitPer; ++e) v[e] = src[min(i0 + e * kInitWG + tid, n - 1)];
#pragma unroll
        for (int e = 0; e < kInitPer; ++e) {
            const int i = i0 + e * kInitWG + tid;
            bad |= !(isfinite(v[e].x) && isfinite(v[e].y) && isfinite(v[e].z));
            float4 o = v[e];
            if (!id) xform_pt(Tg, v[e].x, v[e].y, v[e].z, o.x, o.y, o.z);
            big |= fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z))) > kBig;
            if (i < nc) X[i] = o;
        }
    }
    // the pass-scoped state this registration starts from: the pair's miss bitmap and count (cached-
    // neighbour plans) and, by the group's first pair, its work-list counters (plist_n[0..3]: items,
    // queue, part size, the fused order's arrival counter)
    if (w.need) {
        uint32_t* gneed = w.need + (int64_t)p * w.need_stride;
        for (int k = tid; k < w.need_stride; k += kInitWG) gneed[k] = 0u;
    }
    if (tid == 0 && w.miss_cnt) w.miss_cnt[p] = 0;
    if (tid < 4 && p == 0 && w.plist_n) w.plist_n[tid] = 0;
    bad = __syncthreads_or(bad);
    big = __syncthreads_or(big);
    if (tid == 0) {
        mat4_identity(st.T_inc);
        st.prev_mse = DBL_MAX;
        st.similar = 0;
        st.conv_state = 0;
        st.iterations = 0;
        st.ncorr = 0;
        st.sums_ok = big ? -1 : 0;
        // counts above the batch's declared max_src_n / max_tgt_n would overrun the workspace strides
        const bool too_big = n > w.x_stride || (w.leaf > 0 && m > w.t_stride);
        if (m <= 0 || bad || too_big) {
            // Registration::initCompute fails (no target) -> align returns; final stays identity.
            mat4_identity(st.final_T);
            st.phase = kPhaseInvalid;
            st.status = too_big ? kStatusInvalid : m <= 0 ? kStatusEmpty : kStatusNonFinite;
        } else {
            for (int k = 0; k < 16; ++k) st.final_T[k] = Tg[k];  // final_transformation_ = guess
            st.phase = kPhaseActive;
            st.status = 0;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// nn_kernel<Q>: blockIdx.x = query block (WG*Q queries), blockIdx.y = pair, blockIdx.z = target
// split.  Writes the key of each query's nearest target in the split's index range; with several
// splits the keys are merged by a u64 atomicMin into a 0xFF..-initialised array (exact: the
// minimum key is the lexicographic (d², index) minimum, independent of arrival order).
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
    NNKey* key = w.nn_key + (int64_t)p * w.x_stride;
    if (threadIdx.x == 0)
        count_add(w.evals, 0, (unsigned long long)(j1 - j0) * (unsigned long long)min(n - base, kNNWG * Q));
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int i = base + threadIdx.x + q * kNNWG;
        if (i < n) {
            const NNKey k = make_key(best[q], (uint32_t)bi[q]);
            if (w.splits > 1)
                atomicMin(reinterpret_cast<unsigned long long*>(key + i), (unsigned long long)k);
            else
                key[i] = k;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// index_kernel: the pruned search's per-pair index (once per registration; the target never moves
// and a rigid motion keeps the source's spatial order).  blockIdx.x = pair, blockIdx.y = 0 target /
// 1 source.  The order only decides how well blocks prune — the search is exact for any order.
//
//  * n <= kKdMaxN (every scan of the benchmark): a balanced kd-tree order.  Segment [s, e) splits at
//    the median of its widest axis into a left part of floor(units / 2) whole units (unit = one
//    superblock of leaf * kSuper points while the segment is larger than that, else one leaf), so
//    every block of `leaf` consecutive positions is a kd leaf and every superblock a kd subtree.
//    Measured on the benchmark pairs (CPU model of the exact pruning, blocks whose box can reach
//    the second-nearest distance): 2.4 blocks / 1.6 superblocks per query vs 6.6 / 4.7 for the
//    Morton-cell order — the Morton blocks straddle cell boundaries and their boxes are long.
//    Built in LDS with the classic presorted-lists method: the points sorted once per axis
//    (bitonic, unique keys (coordinate, index), so deterministic), then per level a stable
//    partition of all three lists by "left of the split", which keeps each list sorted inside
//    every segment.
//  * larger clouds (the C5 scan-to-map target): a counting sort over 2^14 Morton cells of the
//    bounding box (x, y: 32 cells, z: 16 — radar scans are flat); order inside a cell is whatever
//    the LDS atomics give.
constexpr int kIdxWG = 512;  // two index workgroups per CU (74 KB of LDS each): their barrier-bound levels overlap
constexpr int kIdxWaves = kIdxWG / 64;
constexpr int kCellBins = 1 << 14;
constexpr int kKdMaxN = 8192;
constexpr int kKdPer = kKdMaxN / kIdxWG;  // consecutive list positions per thread

constexpr int kKdBins = 2048;             // counting-sort bins per axis (11-bit quantised coordinate)

#ifndef ICP4R_FLAG32
#define ICP4R_FLAG32 0  // kd levels: one dword per point flag instead of a byte (measured: no change)
#endif
#if ICP4R_FLAG32
typedef uint32_t kd_flag_t;
#else
typedef uint8_t kd_flag_t;
#endif
struct KdShared {
    uint16_t L[3][kKdMaxN];  // per axis: the point indices, sorted by that axis inside every segment
    union {
        uint32_t hist[3][kKdBins];  // the per-axis counting sorts
        struct {
            kd_flag_t left[kKdMaxN + 4];  // per point: left of its segment's split (+ a junk slot)
            uint16_t tpre[3][kIdxWG];  // per list: exclusive prefix of "left" at each thread's first position
        } p;
        float4 bbox[2 * kKdMaxN / 16];  // index_kernel: block boxes (lo, hi) for the superblock boxes
    } u;
    uint16_t seg_mid[kIdxWG];  // per segment, at the thread owning its first position: split position
    uint8_t seg_ax[kIdxWG];    // ... and axis (3: leaf)
    alignas(16) uint16_t wsum[3][kIdxWaves];
    float red[kIdxWaves][6];
    float lo[3], sc[3];
};

struct MortonShared {
    uint32_t bins[kCellBins];
    float red[kIdxWaves][6];
    uint32_t wsum[kIdxWaves];
    float lo_s[3], sc_s[3];
};

#ifndef ICP4R_WG_TICKS
#define ICP4R_WG_TICKS 0  // diagnostic builds: per-workgroup phase stamps (tools/experiments/wg_ticks.py)
#endif

union IndexShared {
    KdShared kd;
    MortonShared mo;
};

__device__ __forceinline__ uint32_t cell_code(float x, float y, float z, const float* lo, const float* sc) {
    const int cx = min(31, max(0, (int)((x - lo[0]) * sc[0])));
    const int cy = min(31, max(0, (int)((y - lo[1]) * sc[1])));
    const int cz = min(15, max(0, (int)((z - lo[2]) * sc[2])));
    uint32_t c = 0;
#pragma unroll
    for (int b = 4; b >= 0; --b) {  // interleave, most significant level first: x y z per level
        c = (c << 1) | ((cx >> b) & 1);
        c = (c << 1) | ((cy >> b) & 1);
        if (b < 4) c = (c << 1) | ((cz >> b) & 1);
    }
    return c;
}

// float -> u32 with the same order (finite inputs)
__device__ __forceinline__ uint32_t ord_key(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// The split of segment [s, e) (see above): left part [s, s + h); h = 0 for a leaf.
__device__ __forceinline__ int kd_split(int S, int leaf) {
    if (S <= leaf) return 0;
    const int unit = S > leaf * kSuper ? leaf * kSuper : leaf;
    return (((S + unit - 1) / unit) >> 1) * unit;
}

// Balanced kd order of pts[0, n) (n <= kKdMaxN) into sh.L[0][0, n).  The per-axis orders are
// counting sorts of the coordinate quantised to kKdBins levels over the cloud's extent; the order
// of equal keys (LDS atomics) is arbitrary, which only moves points between the two sides of a
// split among equals — the search is exact for any order.
// kdn (nullable): the tree is also written out for src_order_kernel — the quantisation (lo, scale
// bits at [0, 6)) and every internal node at [8 + heap id] (root 1, children 2i / 2i + 1) as
// 1 << 31 | mid << 13 | axis << 11 | key of the first point right of the split (on its axis); the
// caller zeroes the node slots (0: leaf).
// KPER: list positions per thread in the levels (16 covers kKdMaxN; 8 for clouds of at most
// kKdMaxN / 2 points, so that a level's per-thread LDS work halves).
template <int KPER, typename Get>  // Get: int -> float4, point i of the cloud
__device__ void kd_order(KdShared& sh, Get pts, int n, int leaf, uint64_t* tk, uint32_t* kdn = nullptr,
                         uint16_t* gk = nullptr) {
    static_assert(KPER % 8 == 0 && KPER <= 16 && KPER * kIdxWG >= kKdMaxN / 2, "list positions per thread");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tk) tk[0] = __builtin_amdgcn_s_memrealtime();
    // 1. bounding box -> quantisation.  The thread's points (i = tid + k * kIdxWG) are loaded once,
    // every load in flight together, and kept for the counting sorts: three load-use passes over the
    // cloud had waited out a global round trip per point and pass (45 us of a build under load).
    float px[kKdPer], py[kKdPer], pz[kKdPer];  // (xyz only: whole float4s spilled registers)
#pragma unroll
    for (int k = 0; k < kKdPer; ++k) {
        const float4 v = pts(min(tid + k * kIdxWG, n - 1));
        px[k] = v.x;
        py[k] = v.y;
        pz[k] = v.z;
    }
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int k = 0; k < kKdPer; ++k) {  // (a clamped duplicate of point n - 1 changes no extent)
        const float4 v = make_float4(px[k], py[k], pz[k], 0.0f);
        mn[0] = fminf(mn[0], v.x); mn[1] = fminf(mn[1], v.y); mn[2] = fminf(mn[2], v.z);
        mx[0] = fmaxf(mx[0], v.x); mx[1] = fmaxf(mx[1], v.y); mx[2] = fmaxf(mx[2], v.z);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // (DPP: no ds_bpermute round trips)
        mn[k] = wave_minf(mn[k]);
        mx[k] = wave_maxf(mx[k]);
    }
    if (lane == 0)
        for (int k = 0; k < 3; ++k) {
            sh.red[wave][k] = mn[k];
            sh.red[wave][3 + k] = mx[k];
        }
    for (int b = tid; b < 3 * kKdBins; b += kIdxWG) (&sh.u.hist[0][0])[b] = 0;
    __syncthreads();
    if (tid < 3) {
        float l = INFINITY, h = -INFINITY;
        for (int v = 0; v < kIdxWaves; ++v) {
            l = fminf(l, sh.red[v][tid]);
            h = fmaxf(h, sh.red[v][3 + tid]);
        }
        sh.lo[tid] = l;
        sh.sc[tid] = h > l ? (float)kKdBins / (h - l) : 0.0f;
        if (kdn) {
            kdn[tid] = __float_as_uint(l);
            kdn[3 + tid] = __float_as_uint(sh.sc[tid]);
        }
    }
    __syncthreads();
    const float lo[3] = {sh.lo[0], sh.lo[1], sh.lo[2]}, sc[3] = {sh.sc[0], sh.sc[1], sh.sc[2]};
    auto bin = [&](float c, int ax) { return min(kKdBins - 1, max(0, (int)((c - lo[ax]) * sc[ax]))); };
    // 2. three counting sorts at once: histogram, exclusive scan, scatter
#pragma unroll
    for (int k = 0; k < kKdPer; ++k) {
        if (tid + k * kIdxWG >= n) continue;
        const float4 v = make_float4(px[k], py[k], pz[k], 0.0f);
        atomicAdd(&sh.u.hist[0][bin(v.x, 0)], 1u);
        atomicAdd(&sh.u.hist[1][bin(v.y, 1)], 1u);
        atomicAdd(&sh.u.hist[2][bin(v.z, 2)], 1u);
    }
    __syncthreads();
    {
        constexpr int per = 3 * kKdBins / kIdxWG;  // 6 bins per thread; an axis = 2048 / 6 threads (not whole)
        static_assert(3 * kKdBins % kIdxWG == 0, "bins per thread");
        uint32_t* hb = &sh.u.hist[0][0];
        uint32_t loc[per], run = 0;
        // scan each axis separately: a thread's bins may straddle two axes, so carry the axis start
#pragma unroll
        for (int k = 0; k < per; ++k) {
            const int gb = tid * per + k;
            loc[k] = run;
            run += hb[gb];
        }
        uint32_t incl = run;
        incl = wave_scan_incl(incl);  // (DPP)
        if (lane == 63) sh.red[wave][0] = __uint_as_float(incl);  // (the bbox partials are consumed)
        __syncthreads();
        uint32_t wbase = 0;
        for (int v = 0; v < wave; ++v) wbase += __float_as_uint(sh.red[v][0]);
        const uint32_t tbase = wbase + incl - run;  // exclusive prefix over all 3 axes' bins
        __syncthreads();
#pragma unroll
        for (int k = 0; k < per; ++k) {
            const int gb = tid * per + k;
            hb[gb] = tbase + loc[k] - (uint32_t)(gb / kKdBins) * (uint32_t)n;  // axis a's bins start at a * n
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kKdPer; ++k) {
        const int i = tid + k * kIdxWG;
        if (i >= n) continue;
        const float4 v = make_float4(px[k], py[k], pz[k], 0.0f);
        const int bx = bin(v.x, 0), by = bin(v.y, 1), bz = bin(v.z, 2);
        if (gk) {  // (coalesced: the levels read them back from this XCD's L2)
            gk[i] = (uint16_t)bx;
            gk[kKdMaxN + i] = (uint16_t)by;
            gk[2 * kKdMaxN + i] = (uint16_t)bz;
        }
        sh.L[0][atomicAdd(&sh.u.hist[0][bx], 1u)] = (uint16_t)i;
        sh.L[1][atomicAdd(&sh.u.hist[1][by], 1u)] = (uint16_t)i;
        sh.L[2][atomicAdd(&sh.u.hist[2][bz], 1u)] = (uint16_t)i;
    }
    __syncthreads();
    if (tk) tk[1] = __builtin_amdgcn_s_memrealtime();
    // 3. levels: split every non-leaf segment at the median of its widest axis.  Segment bounds are
    // multiples of 16 >= KPER, so a thread's positions [p0, p0 + KPER) share one segment [s, e),
    // tracked per thread; the thread owning a segment's first position decides its split.
    const int p0 = tid * KPER;
    int s = 0, e = n, node = 1;  // this thread's segment and its heap id
    for (;;) {
        bool any = false;
        if (p0 == s && p0 < n) {
            const int h = kd_split(e - s, leaf);
            uint8_t ax = 3;
            if (h) {
                // the segment's extent per axis from the keys of its first and last point in that axis'
                // list, re-quantised from the (cache-resident) cloud: no per-point key array in LDS
                // (keeping the small clouds' bins in LDS instead was measured: no faster)
                float ext[3];
                if (gk) {  // the quantised keys written above: 2-B reads of an L2-resident 48 KB
                    int kf[3], kl[3];
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        kf[a] = gk[a * kKdMaxN + sh.L[a][s]];
                        kl[a] = gk[a * kKdMaxN + sh.L[a][e - 1]];
                    }
#pragma unroll
                    for (int a = 0; a < 3; ++a) ext[a] = (float)(kl[a] - kf[a]) / sc[a];
                } else {
                    float4 pf[3], pl[3];
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        pf[a] = pts(sh.L[a][s]);
                        pl[a] = pts(sh.L[a][e - 1]);
                    }
                    ext[0] = (float)(bin(pl[0].x, 0) - bin(pf[0].x, 0)) / sc[0];
                    ext[1] = (float)(bin(pl[1].y, 1) - bin(pf[1].y, 1)) / sc[1];
                    ext[2] = (float)(bin(pl[2].z, 2) - bin(pf[2].z, 2)) / sc[2];
                }
                ax = ext[0] >= ext[1] && ext[0] >= ext[2] ? 0 : (ext[1] >= ext[2] ? 1 : 2);
                any = true;
                if (kdn && node < kKdNodes) {
                    uint32_t km;
                    if (gk) {
                        km = gk[ax * kKdMaxN + sh.L[ax][s + h]];
                    } else {
                        const float4 pm = pts(sh.L[ax][s + h]);
                        km = (uint32_t)bin(ax == 0 ? pm.x : (ax == 1 ? pm.y : pm.z), ax);
                    }
                    kdn[8 + node] = 0x80000000u | ((uint32_t)(s + h) << 13) | ((uint32_t)ax << 11) | km;
                }
            }
            sh.seg_mid[tid] = (uint16_t)(s + h);
            sh.seg_ax[tid] = ax;
        }
        if (!__syncthreads_or(any)) {
            if (tk) tk[2] = __builtin_amdgcn_s_memrealtime();
            break;
        }
        int mid = 0, ax = 3;
        if (p0 < n) {
            mid = sh.seg_mid[s / KPER];
            ax = sh.seg_ax[s / KPER];
        }
        // this thread's list entries (one 16-B LDS read per list; entries >= n are never used), two
        // u16 entries per register as read (a u16 array went to scratch, 32-bit elements filled the
        // register budget: a spill in every level)
        uint32_t vp[3][KPER / 2];
        static_assert(KPER % 8 == 0, "whole 16-B reads of the lists");
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int q8 = 0; q8 < KPER / 8; ++q8) {
                const uint4 r = *reinterpret_cast<const uint4*>(&sh.L[a][p0 + 8 * q8]);
                vp[a][4 * q8] = r.x;
                vp[a][4 * q8 + 1] = r.y;
                vp[a][4 * q8 + 2] = r.z;
                vp[a][4 * q8 + 3] = r.w;
            }
        auto ent = [&](int a, int k) -> uint32_t { return (vp[a][k >> 1] >> (16 * (k & 1))) & 0xffffu; };
        const int nv = min(KPER, n - p0);  // valid entries (<= 0: none)
        const bool act = nv > 0 && ax < 3;    // this thread's segment splits
        // Every LDS access of the level below is unconditional: a per-entry guard had put a branch and
        // a wait around each (~6 us per level on a single 2k-point build).  Entries past nv (the thread
        // holding position n - 1) may hold anything: their flag goes to the junk slot, their flag reads
        // are masked into range and dropped, and their partition writes land in [n, p0 + KPER).
        if (act) {  // "left" per point, from the split axis' list
            uint32_t va[KPER / 2];  // the split axis' entries, re-read from LDS (a select among the
                                      // registers became a dynamic index: a round trip through scratch)
#pragma unroll
            for (int q8 = 0; q8 < KPER / 8; ++q8) {
                const uint4 r = *reinterpret_cast<const uint4*>(&sh.L[ax][p0 + 8 * q8]);
                va[4 * q8] = r.x;
                va[4 * q8 + 1] = r.y;
                va[4 * q8 + 2] = r.z;
                va[4 * q8 + 3] = r.w;
            }
            const uint32_t lf = p0 < mid ? 1u : 0u;  // (segment bounds and mid are multiples of KPER)
#pragma unroll
            for (int k = 0; k < KPER; ++k) {
                const uint32_t i = (va[k >> 1] >> (16 * (k & 1))) & 0xffffu;
                sh.u.p.left[k < nv ? i : kKdMaxN] = (kd_flag_t)lf;
            }
        }
        __syncthreads();
        // stable partition of the three lists: exclusive prefix of "left" in list order; the flags of
        // this thread's entries as bit masks (the split axis' own read back what this thread wrote)
        uint32_t fb[3] = {0u, 0u, 0u};
        if (act) {
            uint32_t fl[3][KPER];
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int k = 0; k < KPER; ++k) fl[a][k] = sh.u.p.left[ent(a, k) & (kKdMaxN - 1)];
            const uint32_t vm = nv >= 32 ? ~0u : (1u << nv) - 1u;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
#pragma unroll
                for (int k = 0; k < KPER; ++k) fb[a] |= fl[a][k] << k;
                fb[a] &= vm;
            }
        }
        const int cnt[3] = {__builtin_popcount(fb[0]), __builtin_popcount(fb[1]), __builtin_popcount(fb[2])};
        int incl[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) incl[a] = (int)wave_scan_incl((uint32_t)cnt[a]);  // (DPP)
        if (lane == 63)
#pragma unroll
            for (int a = 0; a < 3; ++a) sh.wsum[a][wave] = (uint16_t)incl[a];
#pragma unroll
        for (int a = 0; a < 3; ++a) sh.u.p.tpre[a][tid] = (uint16_t)(incl[a] - cnt[a]);  // in-wave exclusive
        __syncthreads();  // wave totals and in-wave prefixes visible; every thread holds its entries in v
        const int sw = (s / KPER) >> 6;  // the wave owning the segment's first position
        if (act) {
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                if (a == ax) continue;  // already partitioned: every entry stays where it is
                // the wave totals before `wave` and before `sw` (u16 each, 16-B LDS reads)
                static_assert(kIdxWaves % 8 == 0 && kIdxWaves <= 16, "wave totals in whole 16-B reads");
                uint32_t ww[kIdxWaves / 2];
#pragma unroll
                for (int q8 = 0; q8 < kIdxWaves / 8; ++q8) {
                    const uint4 r = *reinterpret_cast<const uint4*>(&sh.wsum[a][8 * q8]);
                    ww[4 * q8] = r.x; ww[4 * q8 + 1] = r.y; ww[4 * q8 + 2] = r.z; ww[4 * q8 + 3] = r.w;
                }
                int bw = 0, bs = 0;
#pragma unroll
                for (int k = 0; k < kIdxWaves; ++k) {
                    const int c = (int)((ww[k >> 1] >> (16 * (k & 1))) & 0xffffu);
                    bw += k < wave ? c : 0;
                    bs += k < sw ? c : 0;
                }
                // "left" points before p0 inside the segment
                int ones = (bw + incl[a] - cnt[a]) - (bs + (int)sh.u.p.tpre[a][s / KPER]);
#pragma unroll
                for (int k = 0; k < KPER; ++k) {
                    const int f = (fb[a] >> k) & 1;
                    const int np = f ? s + ones : mid + (p0 + k - s) - ones;
                    ones += f;
                    sh.L[a][np] = (uint16_t)ent(a, k);
                }
            }
            if (p0 < mid) {
                e = mid;
                node = 2 * node;
            } else {
                s = mid;
                node = 2 * node + 1;
            }
        }
        __syncthreads();
    }
}

__device__ void index_boxes(const WorkArgs& w, int p, int n) {
    const int tid = threadIdx.x;
    float4* ts = w.tsort + (int64_t)p * w.t_stride;
    __syncthreads();  // workgroup-scope release/acquire: the scatter above is visible to this WG
    // 5. tail duplicates, block boxes, superblock boxes
    // padding: +inf coordinates (d² = +inf never beats a real target, and no padding entry
    // can pose as a second-nearest duplicate of a real one); .w = the last target's index
    const float4 last = ts[n - 1];
    for (int64_t pos = n + tid; pos < w.t_stride; pos += kIdxWG) ts[pos] = make_float4(INFINITY, INFINITY, INFINITY, last.w);
    const int B = w.leaf;
    const int nb = (n + B - 1) / B;
    float4* tb = w.tbox + (int64_t)p * 2 * w.b_stride;
    // (each block's points, and each superblock's block boxes, loaded all at once: a load-use loop
    // had waited out one round trip per point — 8 blocks x 16 points per thread for a 65k-point map)
    constexpr int kHalf = 16;  // w.leaf: 16 or 32 points, 16 at a time
    for (int b = tid; b < w.b_stride; b += kIdxWG) {
        float4 l = make_float4(INFINITY, INFINITY, INFINITY, 0.f), h = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
        if (b < nb) {
            const int e = min(n, (b + 1) * B) - 1;  // the block's last real point
            for (int h0 = 0; h0 < B; h0 += kHalf) {
                float vx[kHalf], vy[kHalf], vz[kHalf];
#pragma unroll
                for (int k = 0; k < kHalf; ++k) {  // (repeats of the last point: no change)
                    const float4 v = ts[min(b * B + h0 + k, e)];
                    vx[k] = v.x;
                    vy[k] = v.y;
                    vz[k] = v.z;
                }
#pragma unroll
                for (int k = 0; k < kHalf; ++k) {
                    l.x = fminf(l.x, vx[k]); l.y = fminf(l.y, vy[k]); l.z = fminf(l.z, vz[k]);
                    h.x = fmaxf(h.x, vx[k]); h.y = fmaxf(h.y, vy[k]); h.z = fmaxf(h.z, vz[k]);
                }
            }
        }
        tb[2 * b] = l;
        tb[2 * b + 1] = h;
    }
    __syncthreads();  // workgroup-scope release/acquire: the scatter above is visible to this WG
    float4* sbx = w.sbox + (int64_t)p * 2 * w.sb_stride;
    for (int s = tid; s < w.sb_stride; s += kIdxWG) {
        float4 l = make_float4(INFINITY, INFINITY, INFINITY, 0.f), h = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
        float4 bb[2 * kSuper];
#pragma unroll
        for (int k = 0; k < 2 * kSuper; ++k) bb[k] = tb[2 * s * kSuper + k];
#pragma unroll
        for (int k = 0; k < kSuper; ++k) {
            const float4 bl = bb[2 * k], bh = bb[2 * k + 1];
            l.x = fminf(l.x, bl.x); l.y = fminf(l.y, bl.y); l.z = fminf(l.z, bl.z);
            h.x = fmaxf(h.x, bh.x); h.y = fmaxf(h.y, bh.y); h.z = fmaxf(h.z, bh.z);
        }
        sbx[2 * s] = l;
        sbx[2 * s + 1] = h;
    }
}

#ifndef ICP4R_KD_KEYS
#define ICP4R_KD_KEYS 1  // kd levels read the quantised keys from a scratch copy, not the points
#endif

// The source of pair p is ordered by its target's kd tree (src_order_kernel) rather than its own.
__device__ __forceinline__ bool src_by_tgt_tree(const PairArgs& a, const WorkArgs& w, int p) {
    const int m = a.tgt_n[p];
    // (src_order_kernel places at most kKdMaxN sources; a larger source gets its own index)
    return w.src_by_tgt && w.kdn && (w.kd_index & 1) && m > 0 && m <= kKdMaxN && w.t_stride <= kKdMaxN &&
           a.src_n[p] <= kKdMaxN;
}

// One cloud's index (the target or the source of pair p) by one workgroup: index_kernel, and the
// source column of index_refine_kernel when the target's Morton sort is multi-workgroup (w.mo_hist).
__device__ __forceinline__ void index_cloud(IndexShared& shu, const PairArgs& a, const WorkArgs& w, int p, bool is_tgt) {
    if (w.state[p].phase == kPhaseInvalid) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = is_tgt ? a.tgt_n[p] : a.src_n[p];
    if (n <= 0) return;
    const float4* pts = is_tgt ? a.tgt + a.tgt_off[p] : a.src + a.src_off[p];
    if (!is_tgt && src_by_tgt_tree(a, w, p)) return;  // src_order_kernel orders it
    if ((w.kd_index & (is_tgt ? 1 : 2)) && n <= kKdMaxN && (!is_tgt || w.t_stride <= kKdMaxN)) {
#if ICP4R_WG_TICKS  // diagnostic build: every cloud's build start / end and XCC / CU (tools/experiments/idx_ticks.py)
        uint64_t* it = (w.ticks && tid == 0) ? w.ticks + 32 + 12 * (int64_t)gridDim.x + 8 * (int64_t)p + (is_tgt ? 0 : 4) : nullptr;
        if (it) {
            it[0] = __builtin_amdgcn_s_memrealtime();
            it[2] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                    ((uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
        }
#endif
        uint64_t* tk = (w.ticks && p == 0 && is_tgt && tid == 0) ? w.ticks + 12 : nullptr;
        uint32_t* kdn = (is_tgt && w.kdn && w.src_by_tgt) ? w.kdn + (int64_t)p * kKdnStride : nullptr;
        if (kdn)
            for (int k = tid; k < kKdnStride; k += kIdxWG) kdn[k] = 0u;  // (kd_order syncs before writing)
        // the quantised keys' scratch (3 x kKdMaxN u16): the pair's query-record area, unused until
        // the source order / first search writes it (compile-time ICP4R_KD_KEYS=0: the levels re-read the points)
        // (targets only: a pair's source build may run beside it on the same area)
        uint16_t* gk = (ICP4R_KD_KEYS && is_tgt && w.qv && (int64_t)w.x_stride * (int64_t)sizeof(float4) >= 3 * kKdMaxN * 2)
                           ? reinterpret_cast<uint16_t*>(w.qv + (int64_t)p * w.x_stride)
                           : nullptr;
        if (n <= kKdMaxN / 2)
            kd_order<8>(shu.kd, [&](int i) { return pts[i]; }, n, is_tgt ? w.leaf : 16, tk, kdn, gk);
        else
            kd_order<16>(shu.kd, [&](int i) { return pts[i]; }, n, is_tgt ? w.leaf : 16, tk, kdn, gk);
        const uint16_t* ord = shu.kd.L[0];
        if (is_tgt) {
            // sorted targets, padding (+inf coordinates, .w = the last target's index: never a match,
            // never a second-nearest duplicate), and block boxes reduced over `leaf` adjacent lanes
            float4* ts = w.tsort + (int64_t)p * w.t_stride;
            int32_t* tinv = w.tinv + (int64_t)p * w.t_stride;
            float4* tb = w.tbox + (int64_t)p * 2 * w.b_stride;
            const float lastw = __uint_as_float((uint32_t)ord[n - 1]);
            const int B = w.leaf;
            // The coordinates by sorted position come through LDS, not a gather pts[ord[pos]] (16-B
            // reads of 64-B lines: 4.6x the cloud fetched): every position's point writes its inverse
            // (tinv, here coalesced by point), each thread re-reads its own points in index order, and
            // a quarter of the positions at a time is staged in the free axis lists L[1..2] (x, y, z
            // rows) and written out by position.  (t_stride <= kKdMaxN here and a multiple of 64, so
            // the position guard is wave-uniform: the shuffles below see every lane.)
            uint16_t* inv = shu.kd.L[1];
#pragma unroll
            for (int k = 0; k < kKdPer; ++k) {
                const int pos = tid + k * kIdxWG;
                if (pos < n) inv[ord[pos]] = (uint16_t)pos;
            }
            __syncthreads();
            float px[kKdPer], py[kKdPer], pz[kKdPer];
            uint32_t pos2[kKdPer / 2];  // the thread's points' positions, two per dword (0xffff: none)
#pragma unroll
            for (int k = 0; k < kKdPer; ++k) {
                const float4 c = pts[min(tid + k * kIdxWG, n - 1)];
                px[k] = c.x;
                py[k] = c.y;
                pz[k] = c.z;
            }
#pragma unroll
            for (int k = 0; k < kKdPer; ++k) {
                const int i = tid + k * kIdxWG;
                const uint32_t ps = i < n ? (uint32_t)inv[i] : 0xffffu;
                if (i < n) tinv[i] = (int32_t)ps;
                if ((k & 1) == 0)
                    pos2[k >> 1] = ps;
                else
                    pos2[k >> 1] |= ps << 16;
            }
            constexpr int kQ = kKdMaxN / 4;  // positions per quarter: 3 rows of kQ floats (24 KB of L[1..2])
            static_assert(3 * kQ * 4 <= 2 * kKdMaxN * 2, "staging rows in L[1], L[2]");
            float* rx = reinterpret_cast<float*>(&shu.kd.L[1][0]);
            float* ry = rx + kQ;
            float* rz = ry + kQ;
#pragma unroll 1
            for (int q = 0; q < 4; ++q) {
                __syncthreads();  // (inv / the previous quarter's rows read)
#pragma unroll
                for (int k = 0; k < kKdPer / 2; ++k) asm volatile("" : "+v"(pos2[k]));  // (nothing hoisted)
#pragma unroll
                for (int k = 0; k < kKdPer; ++k) {
                    const uint32_t r = ((pos2[k >> 1] >> (16 * (k & 1))) & 0xffffu) - (uint32_t)(q * kQ);
                    if (r < (uint32_t)kQ) {
                        rx[r] = px[k];
                        ry[r] = py[k];
                        rz[r] = pz[k];
                    }
                }
                __syncthreads();
#pragma unroll
                for (int kk = 0; kk < kQ / kIdxWG; ++kk) {
                    const int k = q * (kQ / kIdxWG) + kk;
                    const int pos = tid + k * kIdxWG;
                    if (pos < (int)w.t_stride) {
                        float4 v = make_float4(INFINITY, INFINITY, INFINITY, lastw);
                        float4 l = v, h = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
                        if (pos < n) {
                            const int o = pos - q * kQ;
                            v = make_float4(rx[o], ry[o], rz[o], __uint_as_float((uint32_t)ord[pos]));
                            l = v;
                            h = v;
                        }
                        ts[pos] = v;
                        l.x = seg_minf(l.x, B); h.x = seg_maxf(h.x, B);
                        l.y = seg_minf(l.y, B); h.y = seg_maxf(h.y, B);
                        l.z = seg_minf(l.z, B); h.z = seg_maxf(h.z, B);
                        if ((lane & (B - 1)) == 0) {
                            const int b = pos / B;
                            l.w = 0.f;
                            h.w = 0.f;
                            tb[2 * b] = l;
                            tb[2 * b + 1] = h;
                            shu.kd.u.bbox[2 * b] = l;
                            shu.kd.u.bbox[2 * b + 1] = h;
                        }
                    }
                }
            }
            __syncthreads();
            float4* sbx = w.sbox + (int64_t)p * 2 * w.sb_stride;
            for (int sb = tid; sb < w.sb_stride; sb += kIdxWG) {
                float4 l = make_float4(INFINITY, INFINITY, INFINITY, 0.f), h = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
                for (int b = sb * kSuper; b < (sb + 1) * kSuper; ++b) {
                    const float4 bl = shu.kd.u.bbox[2 * b], bh = shu.kd.u.bbox[2 * b + 1];
                    l.x = fminf(l.x, bl.x); l.y = fminf(l.y, bl.y); l.z = fminf(l.z, bl.z);
                    h.x = fmaxf(h.x, bh.x); h.y = fmaxf(h.y, bh.y); h.z = fmaxf(h.z, bh.z);
                }
                sbx[2 * sb] = l;
                sbx[2 * sb + 1] = h;
            }
            if (tk) tk[3] = __builtin_amdgcn_s_memrealtime();
        } else {
            int32_t* sp = w.sperm + (int64_t)p * w.x_stride;
            for (int pos = tid; pos < n; pos += kIdxWG) sp[pos] = ord[pos];
        }
#if ICP4R_WG_TICKS
        __syncthreads();
        if (it) it[1] = __builtin_amdgcn_s_memrealtime();
#endif
        return;
    }
    if (is_tgt && w.mo_hist) return;  // index_mo_hist_kernel / index_mo_scatter_kernel sort it
    uint32_t* bins = shu.mo.bins;
    float(*red)[6] = shu.mo.red;
    uint32_t* wsum = shu.mo.wsum;
    float* lo_s = shu.mo.lo_s;
    float* sc_s = shu.mo.sc_s;
    // Large clouds (the scan-to-map target): every pass over the cloud keeps kMoPer points per thread
    // in flight (a load-use loop had waited out one round trip per 512 points: 3 x 128 of them for a
    // 65k-point map, ~140 us of a single registration)
    constexpr int kMoPer = 16;
    auto sweep = [&](auto&& f) {
        for (int i0 = 0; i0 < n; i0 += kIdxWG * kMoPer) {
            float4 v[kMoPer];
#pragma unroll
            for (int e = 0; e < kMoPer; ++e) v[e] = pts[min(i0 + e * kIdxWG + tid, n - 1)];
#pragma unroll
            for (int e = 0; e < kMoPer; ++e)
                if (i0 + e * kIdxWG + tid < n) f(i0 + e * kIdxWG + tid, v[e]);
        }
    };
    // 1. bounding box (a target's from init_kernel's validation pass: one pass over the cloud fewer)
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    if (is_tgt && w.tbb) {
        for (int k = 0; k < 3; ++k) {
            mn[k] = w.tbb[(int64_t)p * 8 + k];
            mx[k] = w.tbb[(int64_t)p * 8 + 3 + k];
        }
    } else {
        sweep([&](int, const float4& v) {
            mn[0] = fminf(mn[0], v.x); mn[1] = fminf(mn[1], v.y); mn[2] = fminf(mn[2], v.z);
            mx[0] = fmaxf(mx[0], v.x); mx[1] = fmaxf(mx[1], v.y); mx[2] = fmaxf(mx[2], v.z);
        });
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // (DPP: no ds_bpermute round trips)
        mn[k] = wave_minf(mn[k]);
        mx[k] = wave_maxf(mx[k]);
    }
    if (lane == 0)
        for (int k = 0; k < 3; ++k) {
            red[wave][k] = mn[k];
            red[wave][3 + k] = mx[k];
        }
    for (int b = tid; b < kCellBins; b += kIdxWG) bins[b] = 0;
    __syncthreads();
    if (tid < 3) {
        float l = INFINITY, h = -INFINITY;
        for (int v = 0; v < kIdxWaves; ++v) {
            l = fminf(l, red[v][tid]);
            h = fmaxf(h, red[v][3 + tid]);
        }
        const float cells = tid == 2 ? 16.0f : 32.0f;
        lo_s[tid] = l;
        sc_s[tid] = h > l ? cells / (h - l) : 0.0f;
    }
    __syncthreads();
    float lo[3] = {lo_s[0], lo_s[1], lo_s[2]}, sc[3] = {sc_s[0], sc_s[1], sc_s[2]};
    // 2. histogram of cell codes
    sweep([&](int, const float4& v) { atomicAdd(&bins[cell_code(v.x, v.y, v.z, lo, sc)], 1u); });
    __syncthreads();
    // 3. exclusive scan: thread t owns bins [16 t, 16 t + 16)
    constexpr int per = kCellBins / kIdxWG;
    uint32_t loc[per], run = 0;
#pragma unroll
    for (int k = 0; k < per; ++k) {
        loc[k] = run;
        run += bins[tid * per + k];
    }
    uint32_t incl = run;
    incl = wave_scan_incl(incl);  // (DPP)
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (int v = 0; v < wave; ++v) wbase += wsum[v];
    const uint32_t tbase = wbase + incl - run;
#pragma unroll
    for (int k = 0; k < per; ++k) bins[tid * per + k] = tbase + loc[k];
    __syncthreads();
    // 4. scatter
    if (is_tgt) {
        float4* ts = w.tsort + (int64_t)p * w.t_stride;
        int32_t* tinv = w.tinv + (int64_t)p * w.t_stride;
        sweep([&](int i, const float4& v) {
            const uint32_t pos = atomicAdd(&bins[cell_code(v.x, v.y, v.z, lo, sc)], 1u);
            ts[pos] = make_float4(v.x, v.y, v.z, __uint_as_float((uint32_t)i));
            tinv[i] = (int32_t)pos;
        });
        index_boxes(w, p, n);
    } else {
        int32_t* sp = w.sperm + (int64_t)p * w.x_stride;
        sweep([&](int i, const float4& v) {
            const uint32_t pos = atomicAdd(&bins[cell_code(v.x, v.y, v.z, lo, sc)], 1u);
            sp[pos] = i;
        });
    }
}


// Multi-workgroup Morton sort of a large target (the C5 submap: 65k points), for few pairs: the
// one-workgroup sort above spends ~125 us of a single registration in its three sweeps over the
// cloud.  Workgroup g of pair p owns points [g * kMoChunk, (g + 1) * kMoChunk): one sweep, 16 points
// per thread in flight.  index_mo_hist_kernel writes each workgroup's cell histogram (row p * G + g
// of w.mo_hist); index_mo_scatter_kernel gives every workgroup the exclusive prefix over (cell,
// workgroup) — the cells of all rows before its cell, plus its cell in the rows before its own —
// and scatters its points there.  The quantisation (w.tbb, from init_kernel) is the one-workgroup
// sort's.  Only for plans whose index_refine_kernel re-orders every chunk afterwards (it writes tinv
// and the boxes of every real block); the scatter writes the padding and the empty tail's boxes.
constexpr int kMoChunk = kIdxWG * 16;

__device__ __forceinline__ void mo_quant(const WorkArgs& w, int p, float* lo, float* sc) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float l = w.tbb[(int64_t)p * 8 + k], h = w.tbb[(int64_t)p * 8 + 3 + k];
        lo[k] = l;
        sc[k] = h > l ? (k == 2 ? 16.0f : 32.0f) / (h - l) : 0.0f;
    }
}

__global__ __launch_bounds__(kIdxWG) void index_mo_hist_kernel(PairArgs a, WorkArgs w) {
    __shared__ uint32_t bins[kCellBins];
    const int g = blockIdx.x, p = blockIdx.y, tid = threadIdx.x;
    const int m = a.tgt_n[p];
    if (w.state[p].phase == kPhaseInvalid || m <= 0 || g * kMoChunk >= m) return;
    const float4* pts = a.tgt + a.tgt_off[p];
    float lo[3], sc[3];
    mo_quant(w, p, lo, sc);
    for (int b = tid; b < kCellBins; b += kIdxWG) bins[b] = 0;
    const int i0 = g * kMoChunk;
    float4 v[kMoChunk / kIdxWG];
#pragma unroll
    for (int e = 0; e < kMoChunk / kIdxWG; ++e) v[e] = pts[min(i0 + e * kIdxWG + tid, m - 1)];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < kMoChunk / kIdxWG; ++e)
        if (i0 + e * kIdxWG + tid < m) atomicAdd(&bins[cell_code(v[e].x, v[e].y, v[e].z, lo, sc)], 1u);
    __syncthreads();
    // the row as u16 counts (a workgroup's cell holds at most kMoChunk points), 8 cells per 16-B store
    static_assert(kMoChunk < 65536, "u16 cell counts");
    uint4* row = reinterpret_cast<uint4*>(w.mo_hist + ((int64_t)p * w.mo_groups + g) * kCellBins);
    const uint4* b4 = reinterpret_cast<const uint4*>(bins);
    for (int k = tid; k < kCellBins / 8; k += kIdxWG) {
        const uint4 lo4 = b4[2 * k], hi4 = b4[2 * k + 1];
        row[k] = make_uint4(lo4.x | lo4.y << 16, lo4.z | lo4.w << 16, hi4.x | hi4.y << 16, hi4.z | hi4.w << 16);
    }
}

__global__ __launch_bounds__(kIdxWG) void index_mo_scatter_kernel(PairArgs a, WorkArgs w) {
    __shared__ uint32_t bins[kCellBins];
    __shared__ uint32_t wsum[kIdxWaves];
    const int g = blockIdx.x, p = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m = a.tgt_n[p];
    if (w.state[p].phase == kPhaseInvalid || m <= 0 || g * kMoChunk >= m) return;
    const int ng = (m + kMoChunk - 1) / kMoChunk;  // rows of this pair
    const float4* pts = a.tgt + a.tgt_off[p];
    const int i0 = g * kMoChunk;
    float4 v[kMoChunk / kIdxWG];  // this workgroup's points, in flight while the prefix is formed
#pragma unroll
    for (int e = 0; e < kMoChunk / kIdxWG; ++e) v[e] = pts[min(i0 + e * kIdxWG + tid, m - 1)];
    // thread t owns cells [per * t, per * (t + 1)): per cell its count over every row (tot) and over the
    // rows before g (bef); u16 counts, eight cells per 16-B read, kMoRows rows' reads in flight at once
    // (a row at a time had waited out one L2 round trip per row: ~15 us of a 65k-point sort)
    constexpr int per = kCellBins / kIdxWG;
    constexpr int kMoRows = 3;
    static_assert(per % 8 == 0, "whole 16-B reads of the rows");
    uint32_t tot[per], bef[per];
#pragma unroll
    for (int k = 0; k < per; ++k) tot[k] = bef[k] = 0u;
    const uint16_t* rows = w.mo_hist + (int64_t)p * w.mo_groups * kCellBins + tid * per;
    for (int r0 = 0; r0 < ng; r0 += kMoRows) {
        uint4 c[kMoRows][per / 8];
#pragma unroll
        for (int j = 0; j < kMoRows; ++j) {
            const uint4* rr = reinterpret_cast<const uint4*>(rows + (int64_t)min(r0 + j, ng - 1) * kCellBins);
#pragma unroll
            for (int q = 0; q < per / 8; ++q) c[j][q] = rr[q];
        }
#pragma unroll
        for (int j = 0; j < kMoRows; ++j) {
            const uint32_t use = r0 + j < ng ? 0xffffffffu : 0u, into_bef = r0 + j < g ? 0xffffffffu : 0u;
#pragma unroll
            for (int q = 0; q < per / 8; ++q) {
                const uint32_t u[4] = {c[j][q].x & use, c[j][q].y & use, c[j][q].z & use, c[j][q].w & use};
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    const uint32_t cnt = (u[h >> 1] >> (16 * (h & 1))) & 0xffffu;
                    tot[8 * q + h] += cnt;
                    bef[8 * q + h] += cnt & into_bef;
                }
            }
        }
    }
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < per; ++k) {  // bef[k] := exclusive prefix of cell k inside the thread + its rows before g
        const uint32_t t = tot[k];
        bef[k] += run;
        run += t;
    }
    uint32_t incl = run;
    incl = wave_scan_incl(incl);  // (DPP)
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t tbase = incl - run;
    for (int q = 0; q < wave; ++q) tbase += wsum[q];
    int32_t* rep = w.mo_rep ? w.mo_rep + (int64_t)p * kCellBins : nullptr;
#pragma unroll
    for (int k = 0; k < per; ++k) {
        bins[tid * per + k] = tbase + bef[k];
        if (rep && g == 0 && tot[k] == 0) rep[tid * per + k] = -1;  // (the others: a point's index, below)
    }
    __syncthreads();
    float lo[3], sc[3];
    mo_quant(w, p, lo, sc);
    float4* ts = w.tsort + (int64_t)p * w.t_stride;
#pragma unroll
    for (int e = 0; e < kMoChunk / kIdxWG; ++e) {
        const int i = i0 + e * kIdxWG + tid;
        if (i < m) {
            const uint32_t cell = cell_code(v[e].x, v[e].y, v[e].z, lo, sc);
            const uint32_t pos = atomicAdd(&bins[cell], 1u);
            ts[pos] = make_float4(v[e].x, v[e].y, v[e].z, __uint_as_float((uint32_t)i));
            if (rep) rep[cell] = i;  // (any of the cell's points: the last store wins)
        }
    }
    if (g != ng - 1) return;
    // the tail: padding (+inf coordinates, .w = a real index: never a match) and the boxes of the
    // blocks and superblocks past the last real block (index_refine_kernel writes the real ones)
    for (int64_t pos = m + tid; pos < w.t_stride; pos += kIdxWG)
        ts[pos] = make_float4(INFINITY, INFINITY, INFINITY, __uint_as_float((uint32_t)(m - 1)));
    const int nb = (m + w.leaf - 1) / w.leaf, nsb = (nb + kSuper - 1) / kSuper;
    const float4 el = make_float4(INFINITY, INFINITY, INFINITY, 0.f), eh = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
    float4* tb = w.tbox + (int64_t)p * 2 * w.b_stride;
    for (int64_t b = nb + tid; b < w.b_stride; b += kIdxWG) {
        tb[2 * b] = el;
        tb[2 * b + 1] = eh;
    }
    float4* sbx = w.sbox + (int64_t)p * 2 * w.sb_stride;
    for (int64_t s = nsb + tid; s < w.sb_stride; s += kIdxWG) {
        sbx[2 * s] = el;
        sbx[2 * s + 1] = eh;
    }
}

// src_order_kernel: one workgroup per pair whose target has the kd order (src_by_tgt_tree).  Every
// source point descends the target's kd tree (the quantised key of the node's axis against the key of
// the first point right of the split; equal keys sit on both sides, so they may go either way — the
// order only decides how well the search prunes), and a counting sort by the leaf reached gives the
// source order (sperm): consecutive queries fall in the same or neighbouring target leaves, so
// query runs stay compact, and the leaf's first target seeds the query's first search (nn_key with
// d² = +inf, read by the first pass).  It replaces the source's own kd build (index_kernel).
constexpr int kSoWG = 512;
// query records {index | sorted position << kNtPosShift, ...} and nn_t[i].w (nt_pack, below)
constexpr int kNtPosShift = 14;
constexpr int kNtIdxMask = (1 << kNtPosShift) - 1;

struct SoShared {
    uint32_t nodes[kKdNodes];
    uint32_t bins[kKdMaxN / 16];
    uint32_t wsum[kSoWG / 64];
    float qz[6];
    uint32_t sl[kKdMaxN];  // stage_first: a quarter of the sorted positions' records
};
__device__ void src_order_pair(const PairArgs& a, const WorkArgs& w, int p, SoShared& so) {
    uint32_t* nodes = so.nodes;
    uint32_t* bins = so.bins;
    uint32_t* wsum = so.wsum;
    float* qz = so.qz;
    uint32_t* sl = so.sl;
    if (w.state[p].phase == kPhaseInvalid || !src_by_tgt_tree(a, w, p)) return;
    const int n = a.src_n[p], m = a.tgt_n[p];
    if (n <= 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#if ICP4R_WG_TICKS  // diagnostic build: this pair's source-order start / end (the index stamps' source slots)
    uint64_t* it = (w.ticks && tid == 0) ? w.ticks + 32 + 12 * (int64_t)gridDim.x + 8 * (int64_t)p + 4 : nullptr;
    if (it) {
        it[0] = __builtin_amdgcn_s_memrealtime();
        it[2] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                ((uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
    }
#endif
    const int B = w.leaf;
    const int nb = (m + B - 1) / B;  // <= kKdMaxN / 16
    const uint32_t* kd = w.kdn + (int64_t)p * kKdnStride;
    {
        uint32_t nv[kKdNodes / kSoWG];  // every load before the first store
#pragma unroll
        for (int k = 0; k < kKdNodes / kSoWG; ++k) nv[k] = kd[8 + tid + k * kSoWG];
#pragma unroll
        for (int k = 0; k < kKdNodes / kSoWG; ++k) nodes[tid + k * kSoWG] = nv[k];
    }
    if (tid < 6) qz[tid] = __uint_as_float(kd[tid]);
    for (int b = tid; b < kKdMaxN / 16; b += kSoWG) bins[b] = 0u;
    __syncthreads();
    const float lo[3] = {qz[0], qz[1], qz[2]}, sc[3] = {qz[3], qz[4], qz[5]};
    // Every thread's points (i = tid + e * kSoWG) descend in groups of kSoGrp: their loads all in
    // flight together and the descents interleaved level by level (independent LDS chains) — a
    // point-at-a-time loop had waited out a global round trip and 9 dependent LDS reads per point.
    // The points are X (the guess-transformed sources the first pass searches; init_kernel wrote
    // them), in index order: the leaves stay in registers (two per dword) for the scatter.
    const float4* X = w.X + (int64_t)p * w.x_stride;
    constexpr int kSoPer = kKdMaxN / kSoWG, kSoGrp = 8;
    static_assert(kSoPer % kSoGrp == 0 && kSoPer % 2 == 0, "point groups");
    uint32_t lv[kSoPer / 2];
#pragma unroll
    for (int g = 0; g < kSoPer; g += kSoGrp) {
        float4 v[kSoGrp];
#pragma unroll
        for (int e = 0; e < kSoGrp; ++e) v[e] = X[min(tid + (g + e) * kSoWG, n - 1)];
        int key3[kSoGrp][3], node[kSoGrp], sp[kSoGrp];
#pragma unroll
        for (int e = 0; e < kSoGrp; ++e) {
            key3[e][0] = min(kKdBins - 1, max(0, (int)((v[e].x - lo[0]) * sc[0])));
            key3[e][1] = min(kKdBins - 1, max(0, (int)((v[e].y - lo[1]) * sc[1])));
            key3[e][2] = min(kKdBins - 1, max(0, (int)((v[e].z - lo[2]) * sc[2])));
            node[e] = 1;
            sp[e] = 0;
        }
        for (int lvl = 0; lvl < 11; ++lvl) {  // heap ids < kKdNodes = 2^11
            uint32_t nd[kSoGrp];  // the group's node reads all issued, then branch-free steps
#pragma unroll
            for (int e = 0; e < kSoGrp; ++e) nd[e] = nodes[min(node[e], kKdNodes - 1)];
#pragma unroll
            for (int e = 0; e < kSoGrp; ++e) {
                const bool inner = node[e] < kKdNodes && (nd[e] >> 31);
                const uint32_t ax = (nd[e] >> 11) & 3u;
                const int k = ax == 0u ? key3[e][0] : (ax == 1u ? key3[e][1] : key3[e][2]);
                const bool right = k >= (int)(nd[e] & 2047u);
                sp[e] = (inner && right) ? (int)((nd[e] >> 13) & 0x3fffu) : sp[e];
                node[e] = inner ? 2 * node[e] + (right ? 1 : 0) : kKdNodes;  // a leaf: done
            }
        }
#pragma unroll
        for (int e = 0; e < kSoGrp; ++e) {
            const uint32_t leaf = (uint32_t)min(sp[e] / B, nb - 1);
            if (tid + (g + e) * kSoWG < n) atomicAdd(&bins[leaf], 1u);
            if ((e & 1) == 0)
                lv[(g + e) >> 1] = leaf;
            else
                lv[(g + e) >> 1] |= leaf << 16;
        }
    }
    __syncthreads();
#if ICP4R_WG_TICKS
    if (it) it[3] = __builtin_amdgcn_s_memrealtime();
#endif
    {  // exclusive scan of the nb bins: thread t owns bins [2t, 2t + 2)
        constexpr int per = kKdMaxN / 16 / kSoWG;
        uint32_t loc[per], run = 0;
#pragma unroll
        for (int k = 0; k < per; ++k) {
            loc[k] = run;
            run += bins[tid * per + k];
        }
        uint32_t incl = run;
        incl = wave_scan_incl(incl);  // (DPP)
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t base = 0;
        for (int v = 0; v < wave; ++v) base += wsum[v];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < per; ++k) bins[tid * per + k] = base + incl - run + loc[k];
    }
    __syncthreads();
    int32_t* spm = w.sperm + (int64_t)p * w.x_stride;
    NNKey* key = w.nn_key + (int64_t)p * w.x_stride;
    const float4* ts = w.tsort + (int64_t)p * w.t_stride;
    if (w.stage_first) {
        // The batched search's first-pass query records in sorted order: {X_i, U = +inf} and
        // {i | its position << kNtPosShift, the seed = its leaf's first target position} — the
        // search takes them as they are instead of gathering X through sperm at every work item
        // (a chain of dependent global round trips in front of each pair's first search).  Every
        // record is written in position order (scattered 24-B record stores had cost more than the
        // search saved), from LDS, a quarter of the positions at a time: each thread puts its own
        // points' records (x, y, z, i | leaf << 14) at their positions in the quarter, then the
        // quarter is stored coalesced.  (A gather of X by sorted position instead fetched 4x
        // the cloud: 16-B reads of 64-B lines.)
        // (the coordinates read again, from the L2: kept from the descent they cost occupancy)
        float px[kSoPer], py[kSoPer], pz[kSoPer];
#pragma unroll
        for (int g = 0; g < kSoPer; ++g) {
            const float4 v = X[min(tid + g * kSoWG, n - 1)];
            px[g] = v.x;
            py[g] = v.y;
            pz[g] = v.z;
        }
        uint32_t pos2[kSoPer / 2];  // the points' sorted positions, two per dword
#pragma unroll
        for (int g = 0; g < kSoPer; ++g) {
            const int i = tid + g * kSoWG;
            const uint32_t leaf = (lv[g >> 1] >> (16 * (g & 1))) & 0xffffu;
            const uint32_t ps = i < n ? atomicAdd(&bins[leaf], 1u) : 0xffffu;
            if ((g & 1) == 0)
                pos2[g >> 1] = ps;
            else
                pos2[g >> 1] |= ps << 16;
        }
        constexpr int kQ = kKdMaxN / 4;  // positions per quarter: 4 rows of kQ words in sl's 32 KB
        float* rx = reinterpret_cast<float*>(sl);  // (rows, not 16-B records: a record's 4-register
        float* ry = rx + kQ;                       //  tuples, hoisted out of the quarter loop,
        float* rz = ry + kQ;                       //  took 64 registers)
        uint32_t* rw = sl + 3 * kQ;
        float4* qv = w.qv + (int64_t)p * w.x_stride;
        uint2* qm = w.qm + (int64_t)p * w.x_stride;
        for (int q0 = 0; q0 < n; q0 += kQ) {
            __syncthreads();  // (the previous quarter's records read)
#pragma unroll
            for (int k = 0; k < kSoPer / 2; ++k) asm volatile("" : "+v"(pos2[k]), "+v"(lv[k]));  // (nothing derived from them hoisted: registers)
#pragma unroll
            for (int g = 0; g < kSoPer; ++g) {
                const uint32_t ps = (pos2[g >> 1] >> (16 * (g & 1))) & 0xffffu;
                const uint32_t leaf = (lv[g >> 1] >> (16 * (g & 1))) & 0xffffu;
                const uint32_t r = ps - (uint32_t)q0;
                if (r < (uint32_t)kQ) {
                    rx[r] = px[g];
                    ry[r] = py[g];
                    rz[r] = pz[g];
                    rw[r] = (uint32_t)(tid + g * kSoWG) | (leaf << kNtPosShift);
                }
            }
            __syncthreads();
#pragma unroll
            for (int e = 0; e < kQ / kSoWG; ++e) {
                const int pos = q0 + tid + e * kSoWG;
                if (pos >= n) continue;
                const int o = tid + e * kSoWG;
                const uint32_t e8 = rw[o];
                const uint32_t i = e8 & kNtIdxMask, leaf = e8 >> kNtPosShift;
                spm[pos] = (int32_t)i;
                qv[pos] = make_float4(rx[o], ry[o], rz[o], INFINITY);
                qm[pos] = make_uint2(i | ((uint32_t)pos << kNtPosShift), leaf * (uint32_t)B);
            }
        }
#if ICP4R_WG_TICKS
        __syncthreads();
        if (it) it[1] = __builtin_amdgcn_s_memrealtime();
#endif
        return;
    }
#pragma unroll
    for (int g = 0; g < kSoPer; g += kSoGrp) {
        float sw[kSoGrp];  // the leaves' first targets' index bits (first-pass seeds), loads in flight together
#pragma unroll
        for (int e = 0; e < kSoGrp; ++e) {
            const uint32_t leaf = (lv[(g + e) >> 1] >> (16 * ((g + e) & 1))) & 0xffffu;
            sw[e] = ts[leaf * B].w;
        }
#pragma unroll
        for (int e = 0; e < kSoGrp; ++e) {
            const int i = tid + (g + e) * kSoWG;
            if (i >= n) continue;
            const uint32_t leaf = (lv[(g + e) >> 1] >> (16 * ((g + e) & 1))) & 0xffffu;
            const uint32_t pos = atomicAdd(&bins[leaf], 1u);
            spm[pos] = i;
            key[i] = make_key(INFINITY, __float_as_uint(sw[e]));  // first-pass seed: the leaf's first target
        }
    }
#if ICP4R_WG_TICKS
    __syncthreads();
    if (it) it[1] = __builtin_amdgcn_s_memrealtime();
#endif
}

__global__ __launch_bounds__(kSoWG) void src_order_kernel(PairArgs a, WorkArgs w) {
    __shared__ SoShared so;
    src_order_pair(a, w, xcd_remap(blockIdx.x, gridDim.x), so);
}

#ifndef ICP4R_FUSE_SRC_ORDER
#define ICP4R_FUSE_SRC_ORDER 1  // targets-only grids order the pair's source in the same workgroup
#endif
static_assert(sizeof(SoShared) <= sizeof(IndexShared) && kSoWG == kIdxWG, "the source order reuses the index build's workgroup");
__global__ __launch_bounds__(kIdxWG, 4) void index_kernel(PairArgs a, WorkArgs w) {
    __shared__ IndexShared shu;
    // grid (pairs, 2): target and source of every pair; (pairs, 1): targets only, every source
    // ordered by its target's tree — by this workgroup right after the build (ICP4R_FUSE_SRC_ORDER:
    // one launch and one kernel boundary fewer, the tree read back while it is in this XCD's L2)
    const int g = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
    const int p = gridDim.y == 2 ? g >> 1 : g;
    const bool is_tgt = gridDim.y == 2 ? (g & 1) == 0 : true;
    index_cloud(shu, a, w, p, is_tgt);
    if (ICP4R_FUSE_SRC_ORDER && gridDim.y == 1) {
        __syncthreads();  // the tree (kdn) and sorted targets written; the LDS free
        src_order_pair(a, w, p, *reinterpret_cast<SoShared*>(&shu));
    }
}

// One cloud's index alone (as the target of pair p: no source column, no source order) — the GICP
// source's own index for its k-NN covariances, built on buffers of its own beside the target's chain.
__global__ __launch_bounds__(kIdxWG, 4) void index_cloud_kernel(PairArgs a, WorkArgs w) {
    __shared__ IndexShared shu;
    index_cloud(shu, a, w, xcd_remap(blockIdx.x, gridDim.x), true);
}

// index_refine_kernel: targets too large for the in-LDS kd build (the C5 scan-to-map submap) are
// Morton-sorted by index_kernel, then every 8192-position chunk of that order is re-ordered as a
// balanced kd-tree on its own (one workgroup per chunk, the same builder): superblocks and blocks —
// the units the search prunes with — become kd subtrees and leaves, only the chunk boundaries (every
// 64 superblocks) stay Morton cuts.  Block and superblock boxes of the chunk are recomputed.
__global__ __launch_bounds__(kIdxWG, 4) void index_refine_kernel(PairArgs a, WorkArgs w) {
    __shared__ IndexShared shu;
    const int c = blockIdx.x, p = blockIdx.y;
    if (w.mo_hist && c == (int)gridDim.x - 1) {  // (multi-workgroup Morton sort: no index_kernel launch)
        index_cloud(shu, a, w, p, false);         // the last column builds the pair's source index
        return;
    }
    if (w.state[p].phase == kPhaseInvalid) return;
    const int m = a.tgt_n[p];
    if (m <= 0 || (m <= kKdMaxN && w.t_stride <= kKdMaxN)) return;  // index_kernel's kd path did it
    const int c0 = c * kKdMaxN;
    if (c0 >= m) return;
    const int len = min(kKdMaxN, m - c0);
    const int tid = threadIdx.x, lane = tid & 63;
    float4* ts = w.tsort + (int64_t)p * w.t_stride + c0;
    kd_order<16>(shu.kd, [&](int i) { return ts[i]; }, len, w.leaf, nullptr);
    const uint16_t* ord = shu.kd.L[0];
    float4 v[kKdPer];  // the chunk in its new order (read before anything is overwritten)
#pragma unroll
    for (int k = 0; k < kKdPer; ++k) {
        const int pos = tid + k * kIdxWG;
        v[k] = pos < len ? ts[ord[pos]] : make_float4(INFINITY, INFINITY, INFINITY, 0.f);
    }
    __syncthreads();
    int32_t* tinv = w.tinv + (int64_t)p * w.t_stride;
    float4* tb = w.tbox + (int64_t)p * 2 * w.b_stride;
    const int B = w.leaf;
    const int nbc = (len + B - 1) / B;  // blocks of the chunk (the last may be partial)
#pragma unroll
    for (int k = 0; k < kKdPer; ++k) {
        const int pos = tid + k * kIdxWG;
        const bool real = pos < len;
        if (real) {
            ts[pos] = v[k];
            tinv[__float_as_uint(v[k].w)] = c0 + pos;
        }
        float4 l = real ? v[k] : make_float4(INFINITY, INFINITY, INFINITY, 0.f);
        float4 h = real ? v[k] : make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
        l.x = seg_minf(l.x, B); h.x = seg_maxf(h.x, B);
        l.y = seg_minf(l.y, B); h.y = seg_maxf(h.y, B);
        l.z = seg_minf(l.z, B); h.z = seg_maxf(h.z, B);
        if ((lane & (B - 1)) == 0 && pos / B < nbc) {
            const int b = pos / B;
            l.w = 0.f;
            h.w = 0.f;
            tb[2 * (c0 / B + b)] = l;
            tb[2 * (c0 / B + b) + 1] = h;
            shu.kd.u.bbox[2 * b] = l;
            shu.kd.u.bbox[2 * b + 1] = h;
        }
    }
    __syncthreads();
    float4* sbx = w.sbox + (int64_t)p * 2 * w.sb_stride;
    const int nsbc = (nbc + kSuper - 1) / kSuper, sb0 = c0 / (B * kSuper);
    for (int sb = tid; sb < nsbc; sb += kIdxWG) {
        float4 l = make_float4(INFINITY, INFINITY, INFINITY, 0.f), h = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
        for (int b = sb * kSuper; b < min((sb + 1) * kSuper, nbc); ++b) {
            const float4 bl = shu.kd.u.bbox[2 * b], bh = shu.kd.u.bbox[2 * b + 1];
            l.x = fminf(l.x, bl.x); l.y = fminf(l.y, bl.y); l.z = fminf(l.z, bl.z);
            h.x = fmaxf(h.x, bh.x); h.y = fmaxf(h.y, bh.y); h.z = fmaxf(h.z, bh.z);
        }
        sbx[2 * (sb0 + sb)] = l;
        sbx[2 * (sb0 + sb) + 1] = h;
    }
}

// ---------------------------------------------------------------------------------------------
// nn_pruned_kernel<Q, B>: exact 1-NN with block pruning.  Each wave owns 64*Q source points that
// are contiguous in Morton order (a compact region), keeps their best key in VGPRs, and walks the
// target superblocks outward from the one holding its seed match.  A (super)block is swept only if
// some query's box lower bound can reach its current best; the sweep itself is the scalar-cache
// stream of nn_sweep with the comparison on the full (d², index) key, so the answer is exactly the
// brute-force one (PCL semantics, lowest index among ties) whatever the visiting order.
//
// Pruning is conservative in float: the bound is computed in float and shrunk by 2^-16 before the
// `<=` test, which covers the few-ulp rounding of both the bound and l2_simple's d².  Seeds: the
// previous NN of the same query (iterations > 0 and the fitness pass: the source moved by one small
// increment, so the old match is nearly as close); iteration 0: the target at the same relative
// Morton position.

// lane l's value of v, wave-uniform (v_readlane; l uniform)
__device__ __forceinline__ float rdlane(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

template <int Q>
__device__ __forceinline__ bool box_needed(const v4f lo, const v4f hi, const float (&x)[Q], const float (&y)[Q],
                                           const float (&z)[Q], const NNKey (&best)[Q]) {
    bool need = false;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const float gx = fmaxf(fmaxf(lo.x - x[q], x[q] - hi.x), 0.0f);
        const float gy = fmaxf(fmaxf(lo.y - y[q], y[q] - hi.y), 0.0f);
        const float gz = fmaxf(fmaxf(lo.z - z[q], z[q] - hi.z), 0.0f);
        const float lb = __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, gx * gx));
        need = need || (lb * kLbShrink <= key_d2(best[q]));
    }
    return __any(need);
}

// Coarse (wave-uniform) test: distance between the (super)block box and the box of all the wave's
// queries against the largest best d² of the wave — a few VALU ops on uniform values instead of
// Q per-query tests; only (super)blocks that pass it get the per-query test.
__device__ __forceinline__ bool box_maybe(const v4f lo, const v4f hi, const float (&qlo)[3], const float (&qhi)[3],
                                          float qmax) {
    const float gx = fmaxf(fmaxf(lo.x - qhi[0], qlo[0] - hi.x), 0.0f);
    const float gy = fmaxf(fmaxf(lo.y - qhi[1], qlo[1] - hi.y), 0.0f);
    const float gz = fmaxf(fmaxf(lo.z - qhi[2], qlo[2] - hi.z), 0.0f);
    const float lb = __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, gx * gx));
    return lb * kLbShrink <= qmax;
}

template <int Q, int B>
__device__ __forceinline__ void sweep_block(cv4f_ptr blk, const float (&x)[Q], const float (&y)[Q], const float (&z)[Q],
                                            NNKey (&best)[Q]) {
#pragma unroll
    for (int t = 0; t < B; t += 4) {
        const v4f c[4] = {blk[t], blk[t + 1], blk[t + 2], blk[t + 3]};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t ti = __float_as_uint(c[u].w);
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const NNKey kn = make_key(l2_simple(x[q], y[q], z[q], c[u].x, c[u].y, c[u].z), ti);
                best[q] = kn < best[q] ? kn : best[q];
            }
        }
    }
}

// Seed keys for the chunked pruned search (chunks > 1): every query's key := its seed evaluated at
// the query's current position — the previous match (iterations > 0 / fitness pass) or, in the
// first pass, the target at the same relative sorted position (as the unchunked kernel seeds
// inline).  The chunk searches then start from this key and merge into it with a u64 atomicMin:
// the seed is a real candidate, so min(seed, chunk minima) is the exact (d², index) minimum.
__global__ __launch_bounds__(256) void nn_seed_kernel(PairArgs a, WorkArgs w, int fitness_pass, int first) {
    const int p = blockIdx.y;
    const int phase = uload(&w.state[p].phase);
    if (fitness_pass ? (phase == kPhaseInvalid) : (phase != kPhaseActive)) return;
    const int n = uload(a.src_n + p), m = uload(a.tgt_n + p);
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= n) return;
    const int o = w.sperm[(int64_t)p * w.x_stride + s];
    const float4 v = w.X[(int64_t)p * w.x_stride + o];
    NNKey* key = w.nn_key + (int64_t)p * w.x_stride;
    const NNKey k0 = key[o];
    const float4* tsg = w.tsort + (int64_t)p * w.t_stride;
    uint32_t j;
    if (first && !seed_key(k0, m)) {
        j = __float_as_uint(tsg[((int64_t)s * m) / n].w);
        if (w.mo_rep) {  // a multi-workgroup Morton target: a target in the query's own cell, if any
            float lo[3], sc[3];
            mo_quant(w, p, lo, sc);
            const int32_t r = w.mo_rep[(int64_t)p * kCellBins + cell_code(v.x, v.y, v.z, lo, sc)];
            if (r >= 0 && r < m) j = (uint32_t)r;
        }
    } else {
        j = min((uint32_t)key_idx(k0), (uint32_t)(m - 1));
    }
    const float4 t = a.tgt[uload(a.tgt_off + p) + j];
    key[o] = make_key(l2_simple(v.x, v.y, v.z, t.x, t.y, t.z), j);
}

// Streamed pruned search (single pairs, small batches, targets beyond LDS — C1, C2, C5): one wave
// per 64·Q queries of a pair (Morton/kd-contiguous), blocks streamed through the scalar cache.
// grid.z = chunks: chunk c searches superblocks [c·cs, (c+1)·cs) only (cs <= 64, one lane per
// superblock for the wave's candidate mask), so a single pair fills the GPU — C5's 8 Morton chunks of
// 8192 map points, each a kd tree, or C2's target in quarters — and a wave whose query box cannot
// reach a chunk leaves after one ballot.  With chunks > 1 the seed is nn_seed_kernel's key and the
// chunk minima merge by atomicMin (correspondence records: corr_kernel afterwards).
template <int Q, int B>
__global__ __launch_bounds__(kNNWG) void nn_pruned_kernel(PairArgs a, WorkArgs w, int fitness_pass, int first, int cs) {
    const int chunks = gridDim.z, c = blockIdx.z;
    const int g = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
    const int p = g / gridDim.x, qb = g - p * gridDim.x;
    const int phase = uload(&w.state[p].phase);
    if (fitness_pass ? (phase == kPhaseInvalid) : (phase != kPhaseActive)) return;
    const int n = uload(a.src_n + p), m = uload(a.tgt_n + p);
    const int nb = (m + B - 1) / B, nsb = (nb + kSuper - 1) / kSuper;
    const int sb_lo = c * cs, sb_n = min(cs, nsb - sb_lo);
    if (sb_n <= 0) return;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int base = (qb * (kNNWG / 64) + wave) * (64 * Q);
    if (base >= n) return;
    const float4* X = w.X + (int64_t)p * w.x_stride;
    const int32_t* sperm = w.sperm + (int64_t)p * w.x_stride;
    NNKey* key = w.nn_key + (int64_t)p * w.x_stride;
    const float4* tgt = a.tgt + uload(a.tgt_off + p);
    const float4* tsg = w.tsort + (int64_t)p * w.t_stride;
    float x[Q], y[Q], z[Q];
    NNKey best[Q], seed[Q];
    int orig[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int s0 = base + lane + q * 64;
        const int s = min(s0, n - 1);  // lanes past the end repeat the last query (not written)
        const int o = sperm[s];
        orig[q] = s0 < n ? o : -1;
        const float4 v = X[o];
        x[q] = v.x;
        y[q] = v.y;
        z[q] = v.z;
        const NNKey k0 = key[o];  // chunked: nn_seed_kernel's key; else the previous key / first-pass seed
        if (chunks > 1) {
            best[q] = k0;
        } else {
            const uint32_t j = (first && !seed_key(k0, m)) ? __float_as_uint(tsg[((int64_t)s * m) / n].w)
                                                           : min((uint32_t)key_idx(k0), (uint32_t)(m - 1));
            const float4 t = tgt[j];
            best[q] = make_key(l2_simple(x[q], y[q], z[q], t.x, t.y, t.z), j);
        }
        seed[q] = best[q];
    }
    // the wave's query box and its largest seed distance (uniform; best only shrinks from here on)
    float qlo[3], qhi[3], qmax = 0.0f;
    qlo[0] = qhi[0] = x[0];
    qlo[1] = qhi[1] = y[0];
    qlo[2] = qhi[2] = z[0];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        qlo[0] = fminf(qlo[0], x[q]); qhi[0] = fmaxf(qhi[0], x[q]);
        qlo[1] = fminf(qlo[1], y[q]); qhi[1] = fmaxf(qhi[1], y[q]);
        qlo[2] = fminf(qlo[2], z[q]); qhi[2] = fmaxf(qhi[2], z[q]);
        qmax = fmaxf(qmax, key_d2(best[q]));
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // DPP reductions, wave-uniform results (every lane active here)
        qlo[k] = wave_minf(qlo[k]);
        qhi[k] = wave_maxf(qhi[k]);
    }
    qmax = wave_maxf(qmax);
    // the chunk's superblocks: lane l holds superblock sb_lo + l; one ballot gives the candidates
    v4f isl, ish;
    {
        const v4f* sbv = reinterpret_cast<const v4f*>(w.sbox + (int64_t)p * 2 * w.sb_stride);
        const int sbl = sb_lo + min(lane, sb_n - 1);
        isl = sbv[2 * sbl];
        ish = sbv[2 * sbl + 1];
    }
    const uint64_t cmask = __ballot(lane < sb_n && box_maybe(isl, ish, qlo, qhi, qmax));
    unsigned long long tests = (unsigned long long)sb_n;  // box tests (lane-level: one query against one box)
    int swept = 0;
    // visiting order: outward from the seed's superblock (the first lane's seed) when it lies in the
    // chunk, else from the chunk end nearest to it
    const int seed_pos = w.tinv[(int64_t)p * w.t_stride + __builtin_amdgcn_readfirstlane((uint32_t)best[0])];
    const int sb0 = __builtin_amdgcn_readfirstlane(seed_pos) / (B * kSuper) - sb_lo;
    uint64_t um = sb0 <= 0 ? cmask : sb0 < 64 ? (cmask >> sb0) << sb0 : 0ull, dm = cmask & ~um;
    const cv4f_ptr ts = as_const(tsg);
    const cv4f_ptr tb = as_const(w.tbox + (int64_t)p * 2 * w.b_stride);
    for (bool upnext = true; um | dm; upnext = !upnext) {
        int l;
        if (um && (upnext || !dm)) {
            l = __builtin_ctzll(um);
            um &= um - 1;
        } else {
            l = 63 - __builtin_clzll(dm);
            dm &= ~(1ull << l);
        }
        const v4f slo = {rdlane(isl.x, l), rdlane(isl.y, l), rdlane(isl.z, l), 0.f};
        const v4f shi = {rdlane(ish.x, l), rdlane(ish.y, l), rdlane(ish.z, l), 0.f};
        tests += 64 * Q;
        if (!box_needed<Q>(slo, shi, x, y, z, best)) continue;
        const int sb = sb_lo + l;
        for (int b = sb * kSuper; b < (sb + 1) * kSuper; ++b) {  // blocks past nb have empty boxes
            const v4f blo = tb[2 * b], bhi = tb[2 * b + 1];
            ++tests;
            if (!box_maybe(blo, bhi, qlo, qhi, qmax)) continue;
            tests += 64 * Q;
            if (!box_needed<Q>(blo, bhi, x, y, z, best)) continue;
            sweep_block<Q, B>(ts + (int64_t)b * B, x, y, z, best);
            ++swept;
        }
    }
    if (lane == 0) {
        count_add(w.evals, 0, (unsigned long long)swept * B * (unsigned long long)min(n - base, 64 * Q));
        count_add(w.evals, 1, tests);
    }
    if (chunks > 1) {  // merge; corr_kernel writes the correspondence records after every chunk
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (orig[q] >= 0 && best[q] < seed[q])
                atomicMin(reinterpret_cast<unsigned long long*>(key + orig[q]), (unsigned long long)best[q]);
        return;
    }
    if (w.corr != nullptr && !fitness_pass) {  // PCL numerics: the update's correspondence arrays
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (orig[q] >= 0) write_corr(w, a, p, orig[q], x[q], y[q], z[q], best[q], tgt);
    }
#pragma unroll
    for (int q = 0; q < Q; ++q)
        if (orig[q] >= 0) key[orig[q]] = best[q];
}

// ---------------------------------------------------------------------------------------------
// The batched exact 1-NN (many pairs, targets <= kLdsTargets): three launches per NN pass.
//
//  nn_cache_test_kernel  (passes after the first, CACHE only) the cached-neighbour test of every
//                        query, elementwise at full occupancy: hits get their key / correspondence
//                        record; misses are flagged by Morton position in the pair's bitmap (w.need)
//                        and counted per pair (w.miss_cnt).
//  nn_order_kernel       one workgroup: the pairs that need a search, heaviest first (pair work list
//                        w.plist, w.plist_n), and the search's work-queue counter reset.
//  nn_lds_kernel<CACHE>  persistent (one workgroup per CU): takes pairs from the work list; per
//                        pair it stages the Morton-sorted target set in LDS and searches the queries
//                        that need it (all of them in the first pass / without CACHE).
//
// Search (per pair, one 1024-thread workgroup, the target set in LDS — 128 KB; block / superblock
// boxes stream through the scalar cache).  Each wave owns a Morton-contiguous run of queries and,
// instead of sweeping every block that ANY of its queries might need (nn_pruned_kernel), tests
// blocks per query and appends the (query, block) pairs that pass to a per-wave ring of work items;
// every 64 items are evaluated one per lane (16 targets from LDS each) and merged with an LDS
// atomicMin on the (d², index) key.  The answer is the same exact minimum (PCL semantics, lowest
// index among ties).
//
// CACHE (cached-neighbour test, exact): a search also returns L_i, a lower bound on the distance
// from X_i to every target other than its nearest one j (the exact second-nearest distance: the
// search prunes against the second-best key instead of the best, and an LDS atomicMin keeps the
// smallest key that lost a comparison).  Every kernel that moves X_i by δ_i lowers L_i by δ_i
// (triangle inequality, move_lb).  The next pass first evaluates d_j only: if
// L_i² (1 − m) > d_j² (1 + m) every other target is strictly farther in float too, so (d_j², j)
// IS the brute-force answer — no tie is possible — and the query needs no search.  ICP's increments
// shrink geometrically, so after the first few iterations most queries pass.  The margin m = 1e-4
// is ~500x the float rounding of the test (l2_simple: <= 5 ulp; the bounds are rounded down).
//
// Why persistent + a work list: a late pass leaves most pairs with no miss at all and a few (slowly
// converging) pairs with thousands; one workgroup per pair paid a dispatch gap per pair and let
// the heavy pairs that happened to share a CU set the launch time.
constexpr int kLdsTargets = 8192;
constexpr int kLdsLeaf = 16;
constexpr int kLdsWG = 1024;
constexpr int kLdsWaves = kLdsWG / 64;
constexpr int kLdsQ = 1;  // queries per lane (2 measured no faster: smaller runs prune better)
constexpr int kRing = 128;  // work items per wave (<= 63 pending + 64 appended per query slot)
constexpr float kCacheMargin = 1.0e-4f;
constexpr int kNeedWords = kCacheMaxN / 32;  // bitmap words per pair (one bit per Morton position)
// miss_cnt[p]: the pass' misses, | kMissUnranked when the test left them unplaced (the pair's miss list
// sq / sm and bitmap, for the search to place) instead of in rank order in qv / qm
constexpr int32_t kMissUnranked = 1 << 30;
constexpr int32_t kMissCount = kMissUnranked - 1;
static_assert(kNeedWords <= kLdsWG, "compaction: one bitmap word per thread");

// An LDS address held in a VGPR: a wave-uniform LDS address otherwise sits in an SGPR and every
// ds_read of a row pays its own v_mov; from a VGPR base the row's reads take immediate offsets.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(3))) T* lds_vbase(const T* p) {
    const auto* l = (const __attribute__((address_space(3))) T*)p;
    uint32_t a = (uint32_t)(uintptr_t)l, v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(a));
    return (const __attribute__((address_space(3))) T*)(uintptr_t)v;
}

// Per lane: bit `lane` of the wave mask m set ? if1 : if0 (one v_cndmask on the mask itself)
__device__ __forceinline__ uint32_t lane_select(uint64_t m, uint32_t if0, uint32_t if1) {
    uint32_t r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(m));
    return r;
}

// The 16 targets of LDS block b (lds_swz order) into cs: slot t sits at byte A ^ (t << 4) with
// A = the block's base | (b & 15) << 4 — one v_xor per read instead of an xor, shift and or.
__device__ __forceinline__ void lds_block(const v4f* tl, int b, v4f (&cs)[16]) {
    const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) v4f*)tl;
    const uint32_t A = (base + ((uint32_t)b << 8)) | (((uint32_t)b & 15u) << 4);
#pragma unroll
    for (int t = 0; t < 16; ++t) cs[t] = *(const __attribute__((address_space(3))) v4f*)(uintptr_t)(A ^ ((uint32_t)t << 4));
}

// An LDS target slot is {key, x, y, z}: the key (original index << 13 | LDS position) first, so a
// drain's (d², key) pair forms in the aligned register pair of the slot's first two words (d²
// overwrites x, dead once dx is formed) — with the key last, every evaluation paid a v_mov to pair
// them (a 64-bit VGPR operand must start on an even register).
#ifndef ICP4R_TL_KEYFIRST
#define ICP4R_TL_KEYFIRST 1
#endif
__device__ __forceinline__ v4f tl_slot(const v4f t, uint32_t k) {
    return ICP4R_TL_KEYFIRST ? (v4f){__uint_as_float(k), t.x, t.y, t.z} : (v4f){t.x, t.y, t.z, __uint_as_float(k)};
}
__device__ __forceinline__ float tl_x(const v4f c) { return ICP4R_TL_KEYFIRST ? c.y : c.x; }
__device__ __forceinline__ float tl_y(const v4f c) { return ICP4R_TL_KEYFIRST ? c.z : c.y; }
__device__ __forceinline__ float tl_z(const v4f c) { return ICP4R_TL_KEYFIRST ? c.w : c.z; }
__device__ __forceinline__ uint32_t tl_key(const v4f c) { return __float_as_uint(ICP4R_TL_KEYFIRST ? c.x : c.w); }

// The second-smallest d² of a block after one more evaluation: s2 ≥ b (the current best's d²)
// holds throughout, so min(s2, max(b, d)) — "d below the best: the old best; else min(s2, d)" —
// is the median of the three (one v_med3_u32; d² bits order as unsigned: never negative).
__device__ __forceinline__ uint32_t second_d2(uint32_t b, uint32_t d, uint32_t s2) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(d), "v"(s2));
    return r;
}

// The batched search's box tests against a bound pre-multiplied by kLbGrow (> 1 / kLbShrink with
// margin): lb <= bnd·kLbGrow rejects only what lb·kLbShrink <= bnd rejects, one multiply fewer per
// test.  The per-axis gap v - clamp(v, lo, hi) (a med3) has the magnitude of max(lo - v, v - hi, 0)
// bit for bit (IEEE subtraction is sign-symmetric); a box staged as FLT_MAX (empty) gives +inf.
constexpr float kLbGrow = 1.00002f;
template <typename P>
__device__ __forceinline__ float pt_lb(const P b, float x, float y, float z) {
    const float gx = x - __builtin_amdgcn_fmed3f(x, b[0], b[3]);
    const float gy = y - __builtin_amdgcn_fmed3f(y, b[1], b[4]);
    const float gz = z - __builtin_amdgcn_fmed3f(z, b[2], b[5]);
    return __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, gx * gx));
}
// lower bound of the distance between boxes [lo, hi] and [qlo, qhi] (squared; empty: +inf)
__device__ __forceinline__ float box_lb(const v4f lo, const v4f hi, const float (&qlo)[3], const float (&qhi)[3]) {
    const float gx = fmaxf(fmaxf(lo.x - qhi[0], qlo[0] - hi.x), 0.0f);
    const float gy = fmaxf(fmaxf(lo.y - qhi[1], qlo[1] - hi.y), 0.0f);
    const float gz = fmaxf(fmaxf(lo.z - qhi[2], qlo[2] - hi.z), 0.0f);
    return __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, gx * gx));
}

#ifndef ICP4R_SKIP_SEED
#define ICP4R_SKIP_SEED 1  // the lane's seed block (evaluated whole up front) is never queued again
#endif
#ifndef ICP4R_SB_EXPAND
#define ICP4R_SB_EXPAND 1  // a reached superblock's blocks tested for the lanes that reach it only
#endif
#ifndef ICP4R_SB_BATCH
#define ICP4R_SB_BATCH 1  // candidate superblocks tested together per traversal step
#endif
constexpr int kSbBatch = ICP4R_SB_BATCH;

static_assert(kSbBatch >= 1 && kSbBatch <= 5, "six bits per superblock in a 32-bit pack");
struct LdsNN {
    v4f tl[kLdsTargets];                               // 128 KB: the pair's targets, index order
    alignas(16) float bx[kLdsTargets / kLdsLeaf][6];   // 12 KB: block boxes lo.xyz, hi.xyz (empty: FLT_MAX)
    float sbx[kLdsTargets / kLdsLeaf / kSuper][6];     // 1.5 KB: superblock boxes
    union {
        unsigned long long best[kLdsWaves][64];        // 8 KB: best (d², index << 13 | position) key per query
        struct {                                       // staging: the miss bitmap and its word prefixes
            uint32_t bits[kNeedWords];
            int32_t pre[kNeedWords];
        } cz;
    } r;
    uint32_t sec[kLdsWaves][64];                       // 4 KB: second-smallest d² bits (CACHE search)
    uint16_t items[kLdsWaves][kRing + 64];             // 6 KB: (query lane << 9) | block; + a spare slot per lane
    int32_t wsum[kLdsWaves];                           // staging: bitmap popcounts per wave
    int32_t cur;                                       // the pair this workgroup works on
    unsigned long long selm[kLdsWaves];                // staging (reach_all): superblocks per wave's queries
    int32_t fin;                                       // (claim-ahead) waves done with their runs, all items
    int32_t nx[2][5];                                  // (claim-ahead) item k's {index, item, n, m, misses} in nx[k & 1]
};


// LDS slot of sorted target position p: the slot inside its 16-target block XOR the block's low
// bits — an involution per block (bank spreading for the drain, see nn_lds_kernel)
__device__ __forceinline__ int lds_swz(int p) { return p ^ ((p >> 4) & (kLdsLeaf - 1)); }

// nn_t[i].w packs the NN's sorted target position (bits 0..13) and the query's sorted source position
// (bits 14..27): the test reads one record for the miss bitmap's bit and for the search record it
// writes (sq / sm: the next search's seed is that target position, no index lookup).  Sizes:
// <= kCacheMaxN = 2^14 sources, <= 8192 targets on the batched plan.
static_assert(kCacheMaxN <= (1 << kNtPosShift) && kLdsTargets <= (1 << kNtPosShift) && kLdsMaxSources == (1 << kNtPosShift),
              "nn_t.w / query record packing");
__device__ __forceinline__ float nt_pack(int tpos, int pos) {
    return __uint_as_float((uint32_t)tpos | ((uint32_t)pos << kNtPosShift));
}
__device__ __forceinline__ uint32_t nt_tpos(float w) { return __float_as_uint(w) & kNtIdxMask; }
__device__ __forceinline__ uint32_t nt_pos(float w) { return __float_as_uint(w) >> kNtPosShift; }

// LDS target record .w during the batched search: original index << 13 | sorted position.  Keys
// compare (d², original index) exactly as before (the index is unique and the position follows
// it), and the winner's slot in LDS comes back with its key.
constexpr int kLdsPosBits = 13;
static_assert(kLdsTargets <= (1 << kLdsPosBits), "LDS key packing");
__device__ __forceinline__ uint32_t lk_idx(NNKey k) { return (uint32_t)k >> kLdsPosBits; }
__device__ __forceinline__ uint32_t lk_pos(NNKey k) { return (uint32_t)k & ((1u << kLdsPosBits) - 1); }

// A missed query's search record, appended to its pair's miss list at slot k (in the order the
// test found them): {X.xyz, U} and {its index | its NN's sorted target position << 14, its sorted
// position}.  The search stages these by rank instead of gathering X, U and a seed per query.
__device__ __forceinline__ void put_miss(const WorkArgs& w, int p, int k, uint32_t sp, int i, float x, float y,
                                         float z, float U, uint32_t tpos) {
    const int64_t slot = (int64_t)p * w.x_stride + k;
    w.sq[slot] = make_float4(x, y, z, U);
    // (one 8-B store: stored as two dwords, the second was merged with the LDS record's into a flat
    // store that every miss of the fused test paid)
    *reinterpret_cast<uint64_t*>(&w.sm[slot]) = (uint64_t)((uint32_t)i | (tpos << kNtPosShift)) | ((uint64_t)sp << 32);
}

// Slot of this lane's record in an append list shared by the workgroup (ctr: an LDS counter): one
// LDS atomic per wave.  Every lane of the wave must call it.
__device__ __forceinline__ int wave_append(bool flag, int32_t* ctr) {
    const uint64_t mask = __ballot(flag);
    if (mask == 0) return -1;
    const int lane = threadIdx.x & 63;
    int base = 0;
    if (lane == 0) base = atomicAdd(ctr, __builtin_popcountll(mask));
    base = __builtin_amdgcn_readfirstlane(base);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
    return flag ? base + (int)rank : -1;
}

// Bounds on the second-nearest distance of X_i (L in X_i.w, U in nn_u[i]):
//  L (.x): lower bound on |X_i - t_k| for every target k other than the NN — the cache test's;
//  U (.y): upper bound on the second-nearest distance — the next search's initial pruning bound.
// From the second-smallest d² a search saw (every other target has float d² >= sec; the true
// distance is within sqrt(d²)(1 -/+ 3u)), rounded outwards by 1e-6 (>> the sqrt's own rounding).
__device__ __forceinline__ float2 lu_from_sec(float sec_d2) {
    const float r = sqrtf(sec_d2);
    return make_float2(r * 0.999999f, r * 1.000001f);
}

// The bounds after X_i moved from o to v (float points): L - |v - o|, U + |v - o|, roundings covered.
__device__ __forceinline__ float2 move_lu(float2 lu, float ox, float oy, float oz, float vx, float vy, float vz) {
    const float dx = vx - ox, dy = vy - oy, dz = vz - oz;
    const float d = sqrtf(dx * dx + dy * dy + dz * dz) * 1.00001f;
    return make_float2(fmaxf((lu.x - d) * 0.999999f, 0.0f), (lu.y + d) * 1.000001f);
}

__device__ __forceinline__ bool cache_hit(float L, float dj2) {
    return L * L * (1.0f - kCacheMargin) > dj2 * (1.0f + kCacheMargin);
}

template <int WT = 0>
__device__ __forceinline__ void write_corr_t(const WorkArgs& w, const PairArgs& a, int p, int i, float sx, float sy,
                                             float sz, float d2, const float4 t) {
    float4* C = w.corr + ((int64_t)p * w.x_stride + i) * 2;
    const float wt = a.kp.huber_delta < INFINITY ? (float)huber_w(d2, a.kp.huber_delta) : 1.0f;
    st_v4<WT>(C, make_float4(sx, sy, sz, wt));
    st_v4<WT>(C + 1, make_float4(t.x, t.y, t.z, d2));
}

// With the cached-neighbour state a pass's keys are read only by the finish kernel's fitness (the
// fitness pass) and by the F64 update (load_nn); the PCL-numerics update folds X and nn_t.
__device__ __forceinline__ bool keys_read(const PairArgs& a, int fitness_pass) {
    return fitness_pass || a.kp.numerics != kNumericsPCL;
}

__device__ __forceinline__ bool pass_wants(int phase, int fitness_pass) {
    return fitness_pass ? (phase != kPhaseInvalid) : (phase == kPhaseActive);
}

// The update that follows an NN pass clears the pair's miss bitmap and count (the next test kernel
// ORs into them; nn_light_kernel's work items all read the bitmap, so none of them can clear it).
__device__ __forceinline__ void clear_need(const WorkArgs& w, int p, int n, int tid, int nthreads) {
    if (!w.need) return;
    uint32_t* gneed = w.need + (int64_t)p * w.need_stride;
    for (int k = tid; k < (n + 31) >> 5; k += nthreads) gneed[k] = 0u;
    if (tid == 0) w.miss_cnt[p] = 0;
}

// ---- nn_cache_test_kernel: grid (chunks of kTestWG * kTestPer queries, npairs), XCD-aware.
constexpr int kTestWG = 256;
constexpr int kTestPer = 8;

__global__ __launch_bounds__(kTestWG) void nn_cache_test_kernel(PairArgs a, WorkArgs w, int fitness_pass) {
    __shared__ uint32_t need[kNeedWords];
    __shared__ int32_t wmiss[kTestWG / 64];
    __shared__ int32_t mbase;  // this workgroup's first slot in the pair's miss list
    const int chunks = gridDim.x;
    const int g = xcd_remap(blockIdx.x + chunks * blockIdx.y, chunks * gridDim.y);
    const int p = g / chunks, chunk = g - p * chunks;
    if (!pass_wants(uload(&w.state[p].phase), fitness_pass)) return;
    const int n = uload(a.src_n + p);
    const int i0 = chunk * kTestWG * kTestPer;
    if (i0 >= n) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nwords = (n + 31) >> 5;
    for (int k = tid; k < nwords; k += kTestWG) need[k] = 0;
    __syncthreads();
    float4* X = w.X + (int64_t)p * w.x_stride;
    NNKey* key = w.nn_key + (int64_t)p * w.x_stride;
    float* uu = w.nn_u + (int64_t)p * w.x_stride;
    const float4* nt = w.nn_t + (int64_t)p * w.x_stride;
    const float4* ts = w.tsort + (int64_t)p * w.t_stride;
    // In the iteration passes the previous update's transformCloud(T_inc) is applied here (the
    // update defers it: X_i is read and written once per iteration, and the bounds move with it).
    const bool xform = !fitness_pass;
    float T[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) T[q] = xform ? uload(&w.state[p].T_inc[q]) : 0.0f;
    // Every load is coalesced (the NN's coordinates come from nn_t, not a gather from the target
    // cloud) and issued before the first store (a load after a store waits behind it on vmcnt).
    float4 v[kTestPer], t[kTestPer];
    float U[kTestPer];
#pragma unroll
    for (int e = 0; e < kTestPer; ++e) {
        const int i = min(i0 + e * kTestWG + tid, n - 1);
        v[e] = X[i];  // .w = L
        t[e] = nt[i];
        U[e] = uu[i];
    }
    int hits = 0, misses = 0;
    bool miss[kTestPer];
#pragma unroll
    for (int e = 0; e < kTestPer; ++e) {
        const int i = i0 + e * kTestWG + tid;
        const bool valid = i < n;
        if (xform) {
            float4 o = v[e];
            xform_pt(T, v[e].x, v[e].y, v[e].z, o.x, o.y, o.z);  // PCL transformCloud, in place
            const float2 Lm = move_lu(make_float2(v[e].w, U[e]), v[e].x, v[e].y, v[e].z, o.x, o.y, o.z);
            o.w = Lm.x;
            v[e] = o;
            U[e] = Lm.y;
            if (valid) {
                X[i] = o;
                uu[i] = Lm.y;
            }
        }
        const float d2 = l2_simple(v[e].x, v[e].y, v[e].z, t[e].x, t[e].y, t[e].z);
        const bool hit = valid & cache_hit(v[e].w, d2);  // '&': a conditional use would sink the load
        const uint32_t sp = nt_pos(t[e].w);
        miss[e] = valid && !hit;
        if (hit) {
            // the finish kernel's fitness reads the keys (their d²; the index from the sorted target)
            if (keys_read(a, fitness_pass)) key[i] = make_key(d2, __float_as_uint(ts[nt_tpos(t[e].w)].w));
            ++hits;
        } else if (valid) {
            atomicOr(&need[sp >> 5], 1u << (sp & 31));
            ++misses;
        }
    }
    // this thread's misses -> slots [mbase + the workgroup's prefix, ...) of the pair's miss list
    int incl = misses;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off, 64);
        if (lane >= off) incl += o;
    }
    if (lane == 63) wmiss[wave] = incl;
    hits = wave_sum(hits);
    if (lane == 0) {
        count_add(w.evals, 0, (unsigned long long)hits);
        count_add(w.evals, 2, (unsigned long long)hits);
        count_add(w.evals, 3, (unsigned long long)hits);
    }
    __syncthreads();
    int wbase = 0, tot = 0;
    for (int q = 0; q < kTestWG / 64; ++q) {
        wbase += q < wave ? wmiss[q] : 0;
        tot += wmiss[q];
    }
    if (tid == 0) {
        mbase = tot ? atomicAdd(w.miss_cnt + p, tot) : 0;
        count_add(w.evals, 3, (unsigned long long)tot);
    }
    __syncthreads();
    int k = mbase + wbase + incl - misses;
#pragma unroll
    for (int e = 0; e < kTestPer; ++e)
        if (miss[e]) put_miss(w, p, k++, nt_pos(t[e].w), i0 + e * kTestWG + tid, v[e].x, v[e].y, v[e].z, U[e], nt_tpos(t[e].w));
    uint32_t* gneed = w.need + (int64_t)p * w.need_stride;
    for (int q = tid; q < nwords; q += kTestWG)
        if (need[q]) atomicOr(gneed + q, need[q]);
}

// ---- nn_order_kernel: one workgroup.  Pairs to search, bucketed by floor(log2(work)) heaviest
// first (longest-processing-time-first for the persistent search; the order inside a bucket is
// arbitrary and cannot change any result).  all = 1: every pair the pass wants (first pass / no
// CACHE), work = its source count.
constexpr int kOrderWG = 1024;
constexpr int kOrderBuckets = 32;
constexpr int kPartBits = 10;  // work item = pair << kPartBits | part (parts of >= 64 misses)
static_assert(kCacheMaxN / 64 <= (1 << kPartBits), "part field");

#ifndef ICP4R_ITEMS_PER_CU
#define ICP4R_ITEMS_PER_CU 1  // the work list's target items per CU when heavy pairs are cut (round 6: 1 +0.6 % over 2; 3, 4 slower)
#endif
struct OrderShared {
    int32_t bcnt[kOrderBuckets], boff[kOrderBuckets];
    unsigned long long tot;
};

// The work list of a pass, built by WG threads of one workgroup: by nn_order_kernel, or (FUSED) by
// the last workgroup of the fold_update_kernel launch that ran the pass's cached-neighbour test,
// from the per-pair work words (owork) the other workgroups published — written and read with
// agent-scope (L1-bypassing, write-through) accesses only, so no cache can hold a stale copy.
template <int WG, bool FUSED>
__device__ __forceinline__ void order_items_body(const PairArgs& a, const WorkArgs& w, int npairs, int fitness_pass,
                                                 int all, int ncu, OrderShared& sh) {
    const int tid = threadIdx.x;
    if (tid < kOrderBuckets) sh.bcnt[tid] = 0;
    if (tid == 0) sh.tot = 0;
    __syncthreads();
    auto work_load = [&](int p) -> int {
        if (FUSED) return __hip_atomic_load(w.owork + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kMissCount;
        return !pass_wants(w.state[p].phase, fitness_pass) ? 0 : all ? a.src_n[p] : (w.miss_cnt[p] & kMissCount);
    };
    // the thread's first kOrderReg pairs' work loaded once, all in flight (the three passes below
    // had each waited out their loads: one dependent round trip per pass)
    constexpr int kOrderReg = 4;
    int wreg[kOrderReg];
#pragma unroll
    for (int k = 0; k < kOrderReg; ++k) wreg[k] = tid + k * WG < npairs ? work_load(tid + k * WG) : 0;
    auto work = [&](int p) -> int {
        const int k = (p - tid) / WG;
        return k < kOrderReg ? wreg[k] : work_load(p);
    };
    if (!all && w.part_size > 0) {  // the pass' total work, for the part size below
        unsigned long long t = 0;
        for (int p = tid; p < npairs; p += WG) t += (unsigned long long)work(p);
        t = wave_sum(t);
        if ((tid & 63) == 0) atomicAdd(&sh.tot, t);
    }
    __syncthreads();
    int32_t* bcnt = sh.bcnt;
    int32_t* boff = sh.boff;
    const unsigned long long tot_s = sh.tot;
    // a heavy pair's misses are cut into parts of part_size (first pass: one part, all queries), so
    // the few slowly converging pairs with thousands of misses spread over several CUs
    // (at least part_size, and large enough that the pass has about 2 items per CU: a part costs a
    // target staging, so only the heavy tail of a light pass is worth cutting)
    constexpr unsigned long long kIpc = ICP4R_ITEMS_PER_CU;
    const int ps = (!all && w.part_size > 0) ? max(w.part_size, (int)((tot_s + kIpc * ncu - 1) / (kIpc * ncu))) : (1 << 30);
    auto heavy_parts = [&](int c) { return (c + ps - 1) / ps; };
    auto heavy_size = [&](int c, int k) { return min(ps, c - k * ps); };
    for (int p = tid; p < npairs; p += WG) {
        const int c = work(p);
        if (w.ticks) w.ticks[32 + p] = (uint64_t)c;  // debug: this pass' work per pair (tools/experiments/miss_hist.py)
        if (c <= 0) continue;
        for (int k = 0, np = heavy_parts(c); k < np; ++k) atomicAdd(&bcnt[31 - __builtin_clz((uint32_t)heavy_size(c, k))], 1);
    }
    __syncthreads();
    if (tid == 0) {
        int run = 0;
        for (int b = kOrderBuckets - 1; b >= 0; --b) {
            boff[b] = run;
            run += bcnt[b];
        }
        *w.plist_n = run;
        *w.queue = 0;
        w.plist_n[2] = ps == (1 << 30) ? 0 : ps;  // nn_lds_kernel: misses per part (0: whole pairs)
    }
    __syncthreads();
    for (int p = tid; p < npairs; p += WG) {
        const int c = work(p);
        if (c > 0)
            for (int k = 0, np = heavy_parts(c); k < np; ++k)
                w.plist[atomicAdd(&boff[31 - __builtin_clz((uint32_t)heavy_size(c, k))], 1)] = (p << kPartBits) | k;
    }
}
// (order_items_body: inlined where a call would spill the caller's live registers — fold_update_res_kernel
// takes its kernel arguments' addresses otherwise)
template <int WG, bool FUSED>
__device__ void order_items(const PairArgs& a, const WorkArgs& w, int npairs, int fitness_pass, int all, int ncu,
                            OrderShared& sh) {
    order_items_body<WG, FUSED>(a, w, npairs, fitness_pass, all, ncu, sh);
}

__global__ __launch_bounds__(kOrderWG) void nn_order_kernel(PairArgs a, WorkArgs w, int npairs, int fitness_pass,
                                                            int all, int ncu) {
    __shared__ OrderShared sh;
    order_items<kOrderWG, false>(a, w, npairs, fitness_pass, all, ncu, sh);
}

// Counters of the LDS search runs (device work counts; per-wave events and clocks for
// plan option phase_ticks = 1 — tools/experiments/nn_events.py)
struct RunStats {
    unsigned long long evals = 0, tests = 0;
    uint32_t ev_runs = 0, ev_q = 0, ev_sbv = 0, ev_sbp = 0, ev_blk = 0, ev_push = 0, ev_drain = 0, ev_items = 0;
    uint64_t ck_setup = 0, ck_trav = 0, ck_write = 0;
};
// The LDS arrays a search reads: one pair's staged targets (.w = original index << 13 | position)
// and block / superblock boxes (empty: FLT_MAX).
struct LdsTile {
    v4f* tl;
    float (*bx)[6];
    float (*sbx)[6];
};

// Stage pair p's sorted targets and boxes for an LDS search (every superblock of the pair: nsb <= 64)
// and load lane l's superblock box into isl / ish (kept in registers for every run).  Every load is
// issued before the first store: a load-store loop waited out one global round trip per target (8
// per thread, ~10-20 us per item under load).  The caller's barrier makes the LDS visible.
// A pair's tile in registers (every load issued, nothing waited for): tile_load, then tile_store.
template <int WG>
struct TileRegs {
    v4f tv[kLdsTargets / WG];
    v4f blo, bhi, isl, ish;
};
template <int WG>
__device__ __forceinline__ void tile_load(const WorkArgs& w, int p, int nsb, TileRegs<WG>& r, uint64_t M = ~0ull) {
    const int tid = threadIdx.x, lane = tid & 63;
    const v4f* tsg = reinterpret_cast<const v4f*>(w.tsort + (int64_t)p * w.t_stride);
    const int nt = nsb * kSuper * kLdsLeaf;
    constexpr int kPerT = kLdsTargets / WG;
    static_assert(kLdsTargets % WG == 0, "targets per thread");
    // M: the superblocks to stage; the others load target 0 (one line for the whole wave) into slots
    // no search reads.  A wave's 64 positions lie in one superblock: the test is scalar.
    static_assert(kLdsLeaf * kSuper % 64 == 0 && WG % (kLdsLeaf * kSuper) == 0, "wave-uniform superblock");
    const int wsb = __builtin_amdgcn_readfirstlane(tid / (kLdsLeaf * kSuper));
#pragma unroll
    for (int k = 0; k < kPerT; ++k) {
        const bool on = M == ~0ull || ((M >> (wsb + k * (WG / (kLdsLeaf * kSuper)))) & 1ull);
        r.tv[k] = tsg[on ? min(tid + k * WG, nt - 1) : 0];
    }
    const v4f* tb = reinterpret_cast<const v4f*>(w.tbox + (int64_t)p * 2 * w.b_stride);
    const v4f* sbg = reinterpret_cast<const v4f*>(w.sbox + (int64_t)p * 2 * w.sb_stride);
    static_assert(kLdsTargets / kLdsLeaf / kSuper * (kSuper + 1) <= WG, "one box per thread");
    const int nbx = nsb * (kSuper + 1);
    const int bq = min(tid, nbx - 1);
    const bool blk = bq < nsb * kSuper;
    const int kb = blk ? bq : bq - nsb * kSuper;
    r.blo = blk ? tb[2 * kb] : sbg[2 * kb];
    r.bhi = blk ? tb[2 * kb + 1] : sbg[2 * kb + 1];
    const int sbl = min(lane, nsb - 1);  // (in flight across the caller's barrier)
    r.isl = sbg[2 * sbl];
    r.ish = sbg[2 * sbl + 1];
}
template <int WG>
__device__ __forceinline__ void tile_store(const LdsTile& sh, int nsb, const TileRegs<WG>& r) {
    const int tid = threadIdx.x;
    const int nt = nsb * kSuper * kLdsLeaf;
    constexpr int kPerT = kLdsTargets / WG;
#pragma unroll
    for (int k = 0; k < kPerT; ++k) {
        int i = tid + k * WG;
        // (opaque: the slot addresses are formed here, not hoisted out of a caller's item loop as
        // invariants — kept live across the search they pushed its other values into scratch)
        asm volatile("" : "+v"(i));
        if (i < nt) sh.tl[lds_swz(i)] = tl_slot(r.tv[k], (__float_as_uint(r.tv[k].w) << kLdsPosBits) | (uint32_t)i);
    }
    const int nbx = nsb * (kSuper + 1);
    if (tid < nbx) {
        const bool blk = tid < nsb * kSuper;
        const int kb = blk ? tid : tid - nsb * kSuper;
        const bool empty = !(r.blo.x <= r.bhi.x);  // (+inf, -inf): a box no point reaches
        float* d = blk ? sh.bx[kb] : sh.sbx[kb];
        d[0] = empty ? FLT_MAX : r.blo.x; d[1] = empty ? FLT_MAX : r.blo.y; d[2] = empty ? FLT_MAX : r.blo.z;
        d[3] = empty ? FLT_MAX : r.bhi.x; d[4] = empty ? FLT_MAX : r.bhi.y; d[5] = empty ? FLT_MAX : r.bhi.z;
    }
}

// Stage pair p's sorted targets and boxes for an LDS search (every superblock of the pair: nsb <= 64)
// and load lane l's superblock box into isl / ish (kept in registers for every run).  Every load is
// issued before the first store: a load-store loop waited out one global round trip per target (8
// per thread, ~10-20 us per item under load).  The caller's barrier makes the LDS visible.
template <int WG>
__device__ __forceinline__ void stage_tile(const LdsTile& sh, const WorkArgs& w, int p, int nsb, v4f& isl, v4f& ish,
                                           uint64_t M = ~0ull) {
    TileRegs<WG> r;
    tile_load<WG>(w, p, nsb, r, M);
    tile_store<WG>(sh, nsb, r);
    isl = r.isl;
    ish = r.ish;
}

// The superblocks an item's queries can reach (plan option stage_sel): a lane-per-superblock test of
// each query against lds_runs' initial pruning bound.  lds_runs reads a target only (a) in a query's
// seed block, or (b) in a block it queued, whose superblock passed pt_lb(superblock, q) <= bnd_q for
// that query; and bnd_q = min(seed block's second-smallest d², U²·1.00001) · kLbGrow never exceeds
// B_q = (U²·1.00001) · kLbGrow (the same float expressions: rounding is monotone), nor grows.  So
// every target the search reads lies in a superblock with pt_lb <= B_q for some query of the item,
// or in a seed's superblock — the mask below holds both (idle lanes shadow a run's first query, so
// they read its seed).  A U that is not finite stages everything.  Wave w tests queries w, w + NW, …
// (uniform loads); the caller ORs the waves' masks.  Items of more than kSelExact queries: per run of 64.
constexpr int kSelExact = 64;
template <int WG>
__device__ __forceinline__ uint64_t reach_mask(const float4* qv, const uint2* qm, int nlist, int m, int nsb,
                                               const v4f isl, const v4f ish) {
    constexpr int NW = WG / 64;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const float b[6] = {isl.x, isl.y, isl.z, ish.x, ish.y, ish.z};  // (an empty box passes: a superset)
    const bool mine = lane < nsb;
    uint64_t mk = 0;
    if (nlist > kSelExact) {
        // larger items: 64 consecutive queries (a compact run of sorted positions) at a time, tested as
        // their bounding box against their largest bound — box_lb(sb, box) <= pt_lb(sb, q) <= B_q <= max B
        // for every query q in the box (the same per-axis gaps, monotone float arithmetic): a superset
        const v4f lo4 = isl, hi4 = ish;
        for (int j0 = wave * 64; j0 < nlist; j0 += NW * 64) {
            const int j = min(j0 + lane, nlist - 1);
            const float4 q = qv[j];
            const uint32_t sd = qm[j].y;
            const float B = __uint_as_float(__float_as_uint(q.w * q.w * 1.00001f)) * kLbGrow;
            if (__ballot(!(B < INFINITY)) != 0ull) return ~0ull;
            float qlo[3] = {q.x, q.y, q.z}, qhi[3] = {q.x, q.y, q.z};
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                qlo[k] = wave_minf(qlo[k]);
                qhi[k] = wave_maxf(qhi[k]);
            }
            const float bmax = wave_maxf(B);
            mk |= __ballot(mine && box_lb(lo4, hi4, qlo, qhi) <= bmax);
            unsigned long long s = 1ull << (min(sd, (uint32_t)(m - 1)) / (uint32_t)(kLdsLeaf * kSuper));
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) s |= __shfl_xor(s, off, 64);
            mk |= s;
        }
        return mk;
    }
    for (int j0 = wave; j0 < nlist; j0 += 4 * NW) {
        float4 q[4];
        uint32_t sd[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int j = min(j0 + e * NW, nlist - 1);
            q[e] = qv[j];
            sd[e] = qm[j].y;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float B = __uint_as_float(__float_as_uint(q[e].w * q[e].w * 1.00001f)) * kLbGrow;
            mk |= (B < INFINITY) ? __ballot(mine && pt_lb(b, q[e].x, q[e].y, q[e].z) <= B) : ~0ull;
            mk |= 1ull << (min(sd[e], (uint32_t)(m - 1)) / (uint32_t)(kLdsLeaf * kSuper));
        }
    }
    return mk;
}

// The superblock mask of a small item (stage_sel): reach_mask over the workgroup's waves, ORed through
// selm (kLdsWaves words of LDS); ends with a barrier.  stage_tile then loads the targets of the named
// superblocks only (a late pass's item of a few misses stages a few KB instead of the whole 128-KB
// tile, for one more round trip: the queries and superblock boxes before the targets).
template <int WG>
__device__ __forceinline__ uint64_t reach_all(unsigned long long* selm, const WorkArgs& w, int p, int nsb, int m,
                                              const float4* qv, const uint2* qm, int nlist) {
    const int tid = threadIdx.x, lane = tid & 63;
    const v4f* sbg = reinterpret_cast<const v4f*>(w.sbox + (int64_t)p * 2 * w.sb_stride);
    const int sbl = min(lane, nsb - 1);
    const uint64_t mk = reach_mask<WG>(qv, qm, nlist, m, nsb, sbg[2 * sbl], sbg[2 * sbl + 1]);
    if (lane == 0) selm[tid >> 6] = mk;
    __syncthreads();
    uint64_t M = 0;
#pragma unroll
    for (int v = 0; v < WG / 64; ++v) M |= selm[v];
    // (uniform: scalar registers, not two VGPRs live across the staging)
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(M >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)M);
}

// The exact LDS search of one query list [0, nlist) of pair p (qv / qm: {x, y, z, U}, {source index |
// sorted position << 14, seed target position}, in sorted-position order) against the staged tile,
// by the workgroup's kLdsWaves waves (this wave: its runs, with bestl / secl / ring its LDS state).
// CACHE: the second-nearest distance too (X.w = L, nn_u = U, nn_t = the NN's coordinates | positions);
// want_key: the (d², index) key; corr: the correspondence record (plans without the cached state).
template <bool CACHE>
__device__ __forceinline__ void lds_runs(const LdsTile& sh, unsigned long long* bestl, uint32_t* secl, uint16_t* ring,
                                         const float4* qv, const uint2* qm, int nlist, int m, int nsb, const v4f isl,
                                         const v4f ish, const PairArgs& a, const WorkArgs& w, int p, int64_t xs0,
                                         float4* X, NNKey* key, bool want_key, bool corr, RunStats& rs) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    // Queries per wave run: the list is cut into R rounds of kLdsWaves equal position-contiguous
    // runs of at most 64 (R = ceil(nlist / (kLdsWaves * 64))), so every wave gets the same share —
    // a short list (the misses of a late pass) spreads over all waves, and the traversal,
    // latency-bound per wave, runs on small runs whose tight query box prunes most superblocks.
    const int rounds = max(1, (nlist + kLdsWaves * 64 - 1) / (kLdsWaves * 64));
    const int per = (nlist + kLdsWaves * rounds - 1) / (kLdsWaves * rounds);
    const int stride = kLdsWaves * per;
    // the run's records (idle lanes shadow the run's first query: they never queue work and
    // never widen the run's box); the next run's are loaded while this one is searched
    auto fetch = [&](int b, float4& v, uint2& mq) {
        const int s = (b + lane < min(b + per, nlist)) ? b + lane : b;
        v = qv[s];
        mq = qm[s];
    };
    float4 nv = make_float4(0.f, 0.f, 0.f, 0.f);
    uint2 nm = make_uint2(0u, 0u);
    if (wave * per < nlist) fetch(wave * per, nv, nm);
    for (int base = wave * per; base < nlist; base += stride) {
        const int cend = min(base + per, nlist);
        const uint64_t ck0 = __builtin_readcyclecounter();
        ++rs.ev_runs;
        rs.ev_q += (uint32_t)(cend - base);
        const float x = nv.x, y = nv.y, z = nv.z, uu = nv.w;
        const bool live = base + lane < cend;
        const int orig = (int)(nm.x & kNtIdxMask);
        const int spos = (int)(nm.x >> kNtPosShift);
        const int pj = min((int)nm.y, m - 1);
        __builtin_amdgcn_sched_barrier(0);  // the current record consumed before the prefetch
        if (base + stride < nlist) fetch(base + stride, nv, nm);
        float bnd;  // pruning bound: best d² (plain search) / second-best d² (CACHE search);
                    // -1 on idle lanes (never queue work, never widen the coarse bound)
        const int seed_pos0 = __builtin_amdgcn_readfirstlane(pj);
        const int seed_blk = pj / kLdsLeaf;
        [[maybe_unused]] const uint32_t lane9 = (uint32_t)lane << 9;  // ring item: query lane << 9 | block
        {
            // seed: the previous match (first pass: the target at the same relative position)
            // and the rest of its 16-target block, evaluated up front from LDS — tight initial
            // bounds, so the coarse rs.tests below already prune with them
            NNKey lo = ~0ull;       // the smallest key seen
            uint32_t s2 = ~0u;      // the smallest d² of every other target seen (bits)
            v4f cs[kLdsLeaf];
            lds_block(sh.tl, pj / kLdsLeaf, cs);
            __builtin_amdgcn_sched_barrier(0);  // all 16 reads in flight before the first use
#pragma unroll
            for (int t = 0; t < kLdsLeaf; ++t) {
                const v4f c = cs[t];
                const float d2 = l2_simple(x, y, z, tl_x(c), tl_y(c), tl_z(c));
                const NNKey kn = make_key(d2, tl_key(c));
                if (CACHE) s2 = second_d2((uint32_t)(lo >> 32), __float_as_uint(d2), s2);
                lo = kn < lo ? kn : lo;
            }
            bestl[lane] = lo;
            if (CACHE) {
                // U of the previous search, moved since: an upper bound of the second-nearest
                // distance even if no evaluated target attains it (all-query passes: +inf)
                const uint32_t sec0 = min(s2, __float_as_uint(uu * uu * 1.00001f));
                secl[lane] = sec0;
                bnd = live ? __uint_as_float(sec0) * kLbGrow : -1.0f;
            } else {
                bnd = live ? key_d2(lo) * kLbGrow : -1.0f;
            }
            rs.evals += 64 * kLdsLeaf;  // the wave's lanes (counted once by lane 0)
        }
        float qlo[3] = {x, y, z}, qhi[3] = {x, y, z};
#pragma unroll
        for (int k = 0; k < 3; ++k) {  // DPP reductions (no LDS round trips), wave-uniform results
            qlo[k] = wave_minf(qlo[k]);
            qhi[k] = wave_maxf(qhi[k]);
        }
        const float qmax = wave_maxf(bnd);

        // Evaluate `cnt` (<= 64) queued items from ring[head..]: lane L takes item head + L.
        uint32_t head = 0, tail = 0;
        auto drain = [&](uint32_t cnt) {
            ++rs.ev_drain;
            rs.ev_items += cnt;
            const bool act = (uint32_t)lane < cnt;
            const uint32_t it = ring[(head + lane) & (kRing - 1)];
            const int owner = act ? (int)(it >> 9) : 0;
            const int b = act ? (int)(it & 0x1ffu) : 0;
            // the query's coordinates from its owner lane
            const float qx = __shfl(x, owner, 64), qy = __shfl(y, owner, 64), qz = __shfl(z, owner, 64);
            if (act) {
                NNKey k1 = ~0ull;
                uint32_t s2 = ~0u;  // second-smallest d² of the block (bits; >= k1's throughout)
                // block b's targets sit XOR-swizzled (lds_swz): at step t lane L reads slot
                // t ^ (b_L & 15), so lanes on different blocks spread over the 64 banks instead of
                // all hitting the 4 banks of slot t (a 64-way conflict: every block is 256 B)
                // all 16 reads issued before the first compare (the compiler otherwise keeps two
                // in flight: 8 dependent LDS round trips per drain)
                v4f cs[kLdsLeaf];
                lds_block(sh.tl, b, cs);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = 0; t < kLdsLeaf; ++t) {
                    const v4f c = cs[t];
                    const float d2 = l2_simple(qx, qy, qz, tl_x(c), tl_y(c), tl_z(c));
                    const NNKey kn = make_key(d2, tl_key(c));
                    if (CACHE) s2 = second_d2((uint32_t)(k1 >> 32), __float_as_uint(d2), s2);
                    k1 = kn < k1 ? kn : k1;
                }
                if (CACHE) {
                    // every key but the final winner loses exactly one comparison: keep the smallest loser
                    const NNKey old = atomicMin(&bestl[owner], k1);
                    const uint32_t cand =
                        k1 < old ? min((uint32_t)(old >> 32), s2) : (k1 == old ? s2 : (uint32_t)(k1 >> 32));
                    atomicMin(&secl[owner], cand);
                } else {
                    atomicMin(&bestl[owner], k1);
                }
            }
            head += cnt;
            rs.evals += (unsigned long long)cnt * kLdsLeaf;
            // tighter bounds for the rs.tests
            bnd = !live ? -1.0f : (CACHE ? __uint_as_float(secl[lane]) : key_d2(bestl[lane])) * kLbGrow;
        };
        // coarse test of every superblock at once (lane = superblock; nsb <= 64 here): the boxes
        // sit in the lanes' registers for the whole item (isl / ish)
        const uint64_t cmask = __ballot(lane < nsb && box_lb(isl, ish, qlo, qhi) <= qmax);
        rs.tests += nsb;
        const int sb0 = seed_pos0 / (kLdsLeaf * kSuper);
        // the candidate superblocks outward from the seed's, alternating up / down (only set bits
        // of cmask are visited: a scalar loop over all nsb cost ~10 SALU per superblock per run)
        uint64_t um = sb0 < 64 ? (cmask >> sb0) << sb0 : 0ull, dm = cmask & ~um;
        bool upnext = true;
        auto next_sb = [&]() -> int {
            if (!(um | dm)) return -1;
            int sb;
            if (um && (upnext || !dm)) {
                sb = __builtin_ctzll(um);
                um &= um - 1;
            } else {
                sb = 63 - __builtin_clzll(dm);
                dm &= ~(1ull << sb);
            }
            upnext = !upnext;
            return sb;
        };
        // Candidates are taken kSbBatch at a time: their per-query superblock rs.tests run as
        // independent chains (the traversal is bound by dependent latency, not by issue); then
        // every superblock some lane may reach has its 8 blocks tested for every lane in one
        // straight-line sequence (boxes broadcast from LDS, 8 independent rs.tests in flight), and
        // the non-empty ones are queued.  A test may use a bound a drain has since tightened:
        // that only queues more work, never loses a target.
        const uint64_t ck1 = __builtin_readcyclecounter();
#if ICP4R_SB_EXPAND
        // A superblock some lane may reach has its 8 blocks tested for those lanes only: the c
        // lanes that passed are compacted (ds_permute: rank k -> lane k), and each round rs.tests 8
        // of them against the 8 blocks at once — lane L takes passed lane r0 + L / 8 and block
        // L % 8, with that query's coordinates and bound pulled from its lane (ds_bpermute).  The
        // (query, block) pairs that pass are queued with one ballot per round.  (Testing all 64
        // lanes against all 8 blocks spent 80 VALU per superblock on the ~5 lanes that need it.)
        const int blk8 = lane & (kSuper - 1);
        for (;;) {
            // kSbBatch candidates tested together (independent LDS reads and test chains), then
            // the ones some lane may reach processed in order
            int sbs[kSbBatch];
            uint64_t ms[kSbBatch];
#pragma unroll
            for (int j = 0; j < kSbBatch; ++j) sbs[j] = next_sb();
            if (sbs[0] < 0) break;
#pragma unroll
            for (int j = 0; j < kSbBatch; ++j) {
                const auto* sbb = lds_vbase(&sh.sbx[sbs[j] < 0 ? 0 : sbs[j]][0]);
                ms[j] = sbs[j] < 0 ? 0ull : __ballot(pt_lb(sbb, x, y, z) <= bnd);
                rs.ev_sbv += sbs[j] < 0 ? 0 : 1;
            }
            rs.tests += 64 * kSbBatch;
#pragma unroll
            for (int j = 0; j < kSbBatch; ++j) {
            const int sb = sbs[j];
            const uint64_t m = ms[j];
            if (m == 0) continue;
            ++rs.ev_sbp;
            const int c = __builtin_popcountll(m);
            // this lane's tag: its lane id, and its seed block if that lies in sb (never queued:
            // it was evaluated whole up front)
            const int rel = seed_blk - sb * kSuper;
            const uint32_t tag = (uint32_t)lane | ((ICP4R_SKIP_SEED && (uint32_t)rel < (uint32_t)kSuper) ? (8u | (uint32_t)rel) << 6 : 0u);
            const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            // passed lanes go to lane rank, the others to distinct lanes >= c (no collisions)
            const uint32_t dst = lane_select(m, (uint32_t)c + (uint32_t)lane - rk, rk);
            const uint32_t packed = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)tag);
            // this lane's block box (8 rows, each read by 8 lanes: broadcast)
            const auto* brow = lds_vbase(&sh.bx[sb * kSuper + blk8][0]);
            float bb[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) bb[k] = brow[k];
            rs.tests += 8 * c;
            for (int r0 = 0; r0 < c; r0 += 8) {
                const int srcl = r0 + (lane >> 3);
                const uint32_t tg = (uint32_t)__builtin_amdgcn_ds_bpermute(srcl << 2, (int)packed);
                const int owner = (int)(tg & 63u);
                const float qx = __shfl(x, owner, 64), qy = __shfl(y, owner, 64), qz = __shfl(z, owner, 64);
                const float qb = __shfl(bnd, owner, 64);
                const bool ok = srcl < c && (tg >> 6) != (8u | (uint32_t)blk8) && pt_lb(bb, qx, qy, qz) <= qb;
                const uint64_t pm = __ballot(ok);
                if (pm == 0) continue;
                rs.ev_blk += __builtin_popcountll(pm);
                const uint32_t slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)pm, tail));
                const uint32_t at = lane_select(pm, (uint32_t)(kRing + lane), slot & (kRing - 1));
                ring[at] = (uint16_t)(((uint32_t)owner << 9) | (uint32_t)(sb * kSuper + blk8));
                tail += (uint32_t)__builtin_popcountll(pm);
                if (tail - head >= 64) drain(64);
            }
            }
        }
#else
        for (;;) {
            uint32_t sbpack = 0, valid = 0;
#pragma unroll
            for (int j = 0; j < kSbBatch; ++j) {
                const int sbj = next_sb();
                if (sbj >= 0) {
                    sbpack |= (uint32_t)sbj << (6 * j);
                    valid |= 1u << j;
                }
            }
            if (!valid) break;
            uint32_t pass = 0;
#pragma unroll
            for (int j = 0; j < kSbBatch; ++j) {
                const int sbj = (sbpack >> (6 * j)) & 63;
                // the lanes that may reach this superblock (its box broadcast from LDS)
                const auto* sbb = lds_vbase(&sh.sbx[sbj][0]);
                if (__ballot(pt_lb(sbb, x, y, z) <= bnd) != 0) pass |= 1u << j;
            }
            pass &= valid;
            const int nv = __builtin_popcount(valid);
            rs.ev_sbv += nv;
            rs.tests += 64 * nv;
            for (; pass; pass &= pass - 1) {
                const int sb = (sbpack >> (6 * __builtin_ctz(pass))) & 63;
                ++rs.ev_sbp;
                // the lane's seed block was evaluated whole up front: never queued again
                const int rel = seed_blk - sb * kSuper;
                uint64_t nmk[kSuper];
#pragma unroll
                for (int h = 0; h < kSuper; h += 4) {
                    // 4 rows of 24 B from a multiple of 4 rows (16-B aligned): six ds_read_b128 at
                    // immediate offsets from one VGPR base
                    const auto* b4 = (const __attribute__((address_space(3))) v4f*)lds_vbase(&sh.bx[sb * kSuper + h][0]);
                    v4f r4[6];
#pragma unroll
                    for (int i = 0; i < 6; ++i) r4[i] = b4[i];
                    float bb[4][6];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int c = 0; c < 6; ++c) bb[j][c] = r4[(6 * j + c) >> 2][(6 * j + c) & 3];
                    // (two ballots: a ballot of the '&&' went through a VGPR select, 3 VALU more)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        nmk[h + j] = __ballot(pt_lb(bb[j], x, y, z) <= bnd) & (ICP4R_SKIP_SEED ? __ballot(rel != h + j) : ~0ull);
                }
                rs.tests += 64 * kSuper;
#pragma unroll
                for (int k = 0; k < kSuper; ++k) {  // (unrolled: a rolled loop with one drain
                    const uint64_t mask = nmk[k];  //  copy measured 9 % slower)
                    if (mask == 0) continue;
                    ++rs.ev_blk;
                    // every lane writes (no exec-mask branch): lanes that do not need the block
                    // write their own spare slot past the ring (the mask itself is the select)
                    const uint32_t slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)mask, tail));
                    const uint32_t at = lane_select(mask, (uint32_t)(kRing + lane), slot & (kRing - 1));
                    ring[at] = (uint16_t)(lane9 | (uint32_t)(sb * kSuper + k));
                    tail += (uint32_t)__builtin_popcountll(mask);
                    if (tail - head >= 64) drain(64);
                }
            }
        }
#endif
        if (tail != head) drain(tail - head);
        const uint64_t ck2 = __builtin_readcyclecounter();
        // the winner's coordinates come from its LDS slot (the key carries its position)
        const NNKey kb = bestl[lane];
        const uint32_t tpos = lk_pos(kb);
        const v4f t = sh.tl[lds_swz((int)tpos)];
        if (live) {
            const NNKey ko = make_key(key_d2(kb), lk_idx(kb));  // (d², original index): PCL's answer
            if (want_key) st_sc<2>(&key[orig], ko);
            if (CACHE) {  // the update reads X, nn_t: no correspondence record
                const float2 lu = lu_from_sec(__uint_as_float(secl[lane]));
                st_v4<2>(&X[orig], make_float4(x, y, z, lu.x));  // .w = L
                st_sc<2>(&w.nn_u[xs0 + orig], lu.y);
                st_v4<2>(&w.nn_t[xs0 + orig], make_float4(tl_x(t), tl_y(t), tl_z(t), nt_pack((int)tpos, spos)));
            } else if (corr) {
                write_corr_t(w, a, p, orig, x, y, z, key_d2(kb), make_float4(tl_x(t), tl_y(t), tl_z(t), 0.f));
            }
        }
        const uint64_t ck3 = __builtin_readcyclecounter();
        rs.ck_setup += ck1 - ck0;
        rs.ck_trav += ck2 - ck1;
        rs.ck_write += ck3 - ck2;
    }
}

// Claim-ahead (ICP4R_CLAIM_AHEAD): the next work item's index, pair word, sizes and miss count are
// fetched by lane 0 of the first wave of the workgroup to finish its runs of the current item —
// three dependent round trips (the queue add, the list, the pair's sizes) that then overlap the
// slower waves' runs instead of sitting between two items.  The claim is at most one item's runs
// early (the list is heaviest first: the last items are the smallest).
#ifndef ICP4R_CLAIM_AHEAD
#define ICP4R_CLAIM_AHEAD 1
#endif
__device__ __forceinline__ void claim_item(const PairArgs& a, const WorkArgs& w, int npl, int32_t* nx) {
    const int idx = atomicAdd(w.queue, 1);
    int item = 0, n = 0, m = 0, mc = 0;
    if (idx < npl) {
        item = w.plist[idx];
        const int p = item >> kPartBits;
        n = a.src_n[p];
        m = a.tgt_n[p];
        mc = w.miss_cnt ? w.miss_cnt[p] : 0;
    }
    nx[0] = idx;
    nx[1] = item;
    nx[2] = n;
    nx[3] = m;
    nx[4] = mc;
}

// ---- nn_lds_kernel<CACHE>: persistent search over the pair work list.
// CACHE: per searched query the exact second-nearest distance too, stored as the cached-neighbour
// state: L in X_i.w, U in nn_u[i], the NN's coordinates in nn_t[i] with .w = its index | the query's
// sorted position << 14 (nt_pack) — the position is what the next test flags a miss at.
template <bool CACHE>
__global__ __launch_bounds__(kLdsWG) void nn_lds_kernel(PairArgs a, WorkArgs w, int fitness_pass, int first, int ranked) {
    static_assert(kLdsQ == 1, "one query per lane");
    __shared__ LdsNN sh;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool corr = w.corr != nullptr && !fitness_pass;
    // keys: without the cached-neighbour state the next search's seed and the records read them
    const bool want_key = !CACHE || keys_read(a, fitness_pass);
    const int npl = uload(w.plist_n);
    // work counters; debug event counters and per-phase clocks of every wave (plan option phase_ticks = 1:
    // summed over the registration in ticks[16..26], and per pass in pass_ticks[0..10];
    // tools/experiments/nn_events.py): wave-uniform adds, stored once at the end
    RunStats rs;
#if ICP4R_CLAIM_AHEAD
    if (tid == 0) {
        claim_item(a, w, npl, sh.nx[0]);
        sh.fin = 0;
    }
    __syncthreads();
    for (int it = 0;; ++it) {
        const int32_t* nx = sh.nx[it & 1];
        const int idx = __builtin_amdgcn_readfirstlane(nx[0]);
        if (idx >= npl) break;  // uniform: every wave read the same word
        const bool tk = w.ticks != nullptr && tid == 0;
        uint64_t tk0 = tk ? __builtin_amdgcn_s_memrealtime() : 0, tk1 = tk0, tk2 = tk0;
        const int item = __builtin_amdgcn_readfirstlane(nx[1]);
        const int p = item >> kPartBits, part = item & ((1 << kPartBits) - 1);
        const int n = __builtin_amdgcn_readfirstlane(nx[2]), m = __builtin_amdgcn_readfirstlane(nx[3]);
#else
    for (;;) {
        if (tid == 0) sh.cur = atomicAdd(w.queue, 1);
        __syncthreads();
        const int idx = sh.cur;
        if (idx >= npl) break;  // uniform: every wave read the same sh.cur
        // debug (plan option phase_ticks = 1): per-pair compaction / staging / search wall time, summed over
        // the pairs of the launch into ticks[8..10], pairs in ticks[11]
        const bool tk = w.ticks != nullptr && tid == 0;
        uint64_t tk0 = tk ? __builtin_amdgcn_s_memrealtime() : 0, tk1 = tk0, tk2 = tk0;
        const int item = w.plist[idx];
        const int p = item >> kPartBits, part = item & ((1 << kPartBits) - 1);
        const int n = uload(a.src_n + p), m = uload(a.tgt_n + p);
#endif
        const int nb = (m + kLdsLeaf - 1) / kLdsLeaf, nsb = (nb + kSuper - 1) / kSuper;
        const int64_t xs0 = (int64_t)p * w.x_stride;
        float4* X = w.X + xs0;
        NNKey* key = w.nn_key + xs0;
        // (the parts of a heavy pair run concurrently on other workgroups: each stages at its own
        // absolute ranks [lo, hi) and reads back from qv + lo)
        float4* qv = w.qv + xs0;
        uint2* qm = w.qm + xs0;

        // Stage the item's queries into qv / qm in list order, so every run below reads its
        // queries with one coalesced load that is issued a run ahead:
        //  * all queries (first pass / no cached state): sorted position k -> sperm[k]; X gathered,
        //    U = +inf, the seed = the target at the same relative position (or the source-order
        //    kernel's seed, or the previous key's target);
        //  * the test's misses with rank [lo, lo + part_size) (this item's part), in sorted position
        //    order: the records the test appended to the pair's miss list (sq / sm), each put at its
        //    rank in the miss bitmap.  The update kernel clears the bitmap (other parts may still be
        //    reading it).
        int nlist;
#if ICP4R_CLAIM_AHEAD
        const int mc = (CACHE && !first && ranked) ? __builtin_amdgcn_readfirstlane(nx[4]) : kMissUnranked;
#else
        const int mc = (CACHE && !first && ranked) ? uload(w.miss_cnt + p) : kMissUnranked;
#endif
        bool sel = false;  // a small ranked item: stage the superblocks its queries can reach only
        if (!(mc & kMissUnranked)) {
            // the fused test put the pair's misses in rank order already (pair_cache_test)
            const int ps = uload(w.plist_n + 2);  // the order kernel's part size for this pass
            const int lo = ps > 0 ? part * ps : 0;
            const int hi = ps > 0 ? lo + ps : (1 << 30);
            nlist = min(hi, mc) - lo;
            qv += lo;
            qm += lo;
            sel = nlist <= w.stage_sel;
        } else if (CACHE && !first) {
            const uint32_t* gneed = w.need + (int64_t)p * w.need_stride;
            const int ps = uload(w.plist_n + 2);  // the order kernel's part size for this pass
            const int lo = ps > 0 ? part * ps : 0;
            const int hi = ps > 0 ? lo + ps : (1 << 30);
            const int nwords = (n + 31) >> 5;
            const uint32_t f = tid < nwords ? gneed[tid] : 0u;
            const int c = __builtin_popcount(f);
            int incl = c;
incl = (int)wave_scan_incl((uint32_t)incl);  // (DPP)
            if (lane == 63) sh.wsum[wave] = incl;
            __syncthreads();
            int base = 0, total = 0;
            for (int v = 0; v < kLdsWaves; ++v) {
                const int s = sh.wsum[v];
                base += v < wave ? s : 0;
                total += s;
            }
            if (tid < nwords) {
                sh.r.cz.bits[tid] = f;
                sh.r.cz.pre[tid] = base + incl - c;
            }
            nlist = min(hi, total) - lo;
            __syncthreads();
            // every record of the pair's miss list (in the test's order) goes to its rank: the
            // rank of sorted position sp = its word's prefix + the set bits below it
            const float4* sq = w.sq + xs0;
            const uint2* sm = w.sm + xs0;
            auto get = [&](int k, float4& v, uint2& mm) {
                k = min(k, total - 1);
                v = sq[k];
                mm = sm[k];
            };
            auto put = [&](int k, const float4& v, const uint2& mm) {
                const uint32_t sp = min(mm.y, (uint32_t)(n - 1));
                const int r = sh.r.cz.pre[sp >> 5] + __builtin_popcount(sh.r.cz.bits[sp >> 5] & ((1u << (sp & 31)) - 1u));
                if (k < total && r >= lo && r < hi) {
                    qv[r] = v;
                    qm[r] = make_uint2((mm.x & kNtIdxMask) | (sp << kNtPosShift), mm.x >> kNtPosShift);
                }
            };
#pragma nounroll
            for (int k0 = tid; k0 < total; k0 += 4 * kLdsWG) {
                float4 v0, v1, v2, v3;  // (named, not an array: an array here went to scratch)
                uint2 m0, m1, m2, m3;
                get(k0, v0, m0);  // all loads of the round issued together
                get(k0 + kLdsWG, v1, m1);
                get(k0 + 2 * kLdsWG, v2, m2);
                get(k0 + 3 * kLdsWG, v3, m3);
                put(k0, v0, m0);
                put(k0 + kLdsWG, v1, m1);
                put(k0 + 2 * kLdsWG, v2, m2);
                put(k0 + 3 * kLdsWG, v3, m3);
            }
            qv += lo;  // this item's slice, read back by the runs
            qm += lo;
        } else if (first && w.stage_first && src_by_tgt_tree(a, w, p)) {
            nlist = n;  // src_order_kernel wrote the records
        } else {
            const int32_t* sperm = w.sperm + xs0;
            const int32_t* tinv = w.tinv + (int64_t)p * w.t_stride;
            for (int k0 = 0; k0 < n; k0 += 4 * kLdsWG) {
                int o[4];
                float4 v[4];
                NNKey pk[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = sperm[min(k0 + e * kLdsWG + tid, n - 1)];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[e] = X[o[e]];
                    pk[e] = key[o[e]];
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = k0 + e * kLdsWG + tid;
                    if (k >= n) continue;
                    // seed: the previous match (no cached state), the source-order kernel's leaf, or
                    // the target at the same relative position
                    const bool prev = !first || seed_key(pk[e], m);
                    const int seed = prev ? tinv[min((uint32_t)key_idx(pk[e]), (uint32_t)(m - 1))]
                                          : (int)(((int64_t)k * m) / n);
                    qv[k] = make_float4(v[e].x, v[e].y, v[e].z, INFINITY);
                    qm[k] = make_uint2((uint32_t)o[e] | ((uint32_t)k << kNtPosShift), (uint32_t)seed);
                }
            }
            nlist = n;
        }
        if (tk) tk1 = __builtin_amdgcn_s_memrealtime();

        // Stage the pair's sorted targets into LDS (.w = original index << 13 | position) and the block
        // and superblock boxes, and load every lane's superblock box (isl / ish: lane l holds
        // superblock l's box for every run of the item; nsb <= 64 on this plan).  Every load is issued
        // before the first store: a load-store loop waited out one global round trip per target
        // (8 per thread, ~10-20 us per item under load).
        const LdsTile tv{sh.tl, sh.bx, sh.sbx};
        v4f isl, ish;
        const uint64_t M = sel ? reach_all<kLdsWG>(sh.selm, w, p, nsb, m, qv, qm, nlist) : ~0ull;
        stage_tile<kLdsWG>(tv, w, p, nsb, isl, ish, M);
        __syncthreads();  // LDS targets; qv / qm (global, this workgroup's) visible to every wave
        if (tk) tk2 = __builtin_amdgcn_s_memrealtime();
        unsigned long long* bestl = sh.r.best[wave];
        uint32_t* secl = sh.sec[wave];
        uint16_t* ring = sh.items[wave];
        lds_runs<CACHE>(tv, bestl, secl, ring, qv, qm, nlist, m, nsb, isl, ish, a, w, p, xs0, X, key, want_key, corr, rs);
#if ICP4R_CLAIM_AHEAD
        // the first wave done claims the next item (sh.nx[(it + 1) & 1]: item it - 1's words, read by
        // every wave before this item's staging barrier)
        if (lane == 0 && atomicAdd(&sh.fin, 1) == it * kLdsWaves) claim_item(a, w, npl, sh.nx[(it + 1) & 1]);
#endif
        __syncthreads();  // LDS (targets, per-wave state, sh.cur) is reused by the next pair
        if (tk) {
            unsigned long long* tt = reinterpret_cast<unsigned long long*>(w.ticks);
            atomicAdd(tt + 8, (unsigned long long)(tk1 - tk0));
            atomicAdd(tt + 9, (unsigned long long)(tk2 - tk1));
            atomicAdd(tt + 10, (unsigned long long)(__builtin_amdgcn_s_memrealtime() - tk2));
            atomicAdd(tt + 11, 1ull);
            if (w.pass_ticks) {  // the same walls in this pass' own slots
                unsigned long long* pt = reinterpret_cast<unsigned long long*>(w.pass_ticks);
                atomicAdd(pt + 11, (unsigned long long)(tk1 - tk0));
                atomicAdd(pt + 12, (unsigned long long)(tk2 - tk1));
                atomicAdd(pt + 13, (unsigned long long)(__builtin_amdgcn_s_memrealtime() - tk2));
                atomicAdd(pt + 14, 1ull);
            }
        }
    }
    if (lane == 0) {
        count_add(w.evals, 0, rs.evals);
        count_add(w.evals, 1, rs.tests);
        if (w.ticks) {
            unsigned long long* tt = reinterpret_cast<unsigned long long*>(w.ticks);
            const unsigned long long ev[11] = {rs.ev_runs, rs.ev_q,     rs.ev_sbv,   rs.ev_sbp,  rs.ev_blk,  rs.ev_push,
                                               rs.ev_drain, rs.ev_items, rs.ck_setup, rs.ck_trav, rs.ck_write};
            for (int k = 0; k < 11; ++k) atomicAdd(tt + 16 + k, ev[k]);
            if (w.pass_ticks)
                for (int k = 0; k < 11; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(w.pass_ticks) + k, ev[k]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// nn_tile_kernel: the pruned plan's search (single pairs, small batches, targets of any size — the
// C1 / C2 pairs and the C5 scan-to-map target) with the batched search's LDS machinery.  Grid:
// (target tiles of kLdsTargets sorted positions, query parts of kLdsWG sorted sources, pairs).  A
// workgroup stages its tile (targets and block / superblock boxes) in LDS and searches its queries
// against it, one query per lane in runs of 64 consecutive sorted sources: the tile's superblocks
// tested against the run's box at once, a reached superblock's 8 blocks tested for every lane, the
// non-empty (lane, block) items queued per wave and drained 64 at a time (16 targets from LDS per
// lane).  A query starts from its current key — nn_seed_kernel's seed, or another tile's minimum read
// at the start (any key read is an upper bound: keys only fall) — and merges its tile minimum into it
// with a u64 atomicMin (exact: the lexicographic (d², index) minimum whatever the order of tiles).
// corr_kernel writes the correspondence records afterwards.  Replaces the scalar-cache stream of
// nn_pruned_kernel, whose every block visit evaluated the block for all 64 lanes of a wave.
struct TileShared {
    v4f tl[kLdsTargets];                              // 128 KB: the tile's targets (.w = index << 13 | position)
    alignas(16) float bx[kLdsTargets / kLdsLeaf][6];  // block boxes (empty: FLT_MAX)
    float sbx[kLdsTargets / kLdsLeaf / kSuper][6];    // superblock boxes
    unsigned long long best[kLdsWaves][64];           // per query: best local key
    uint16_t items[kLdsWaves][kRing + 64];            // (query lane << 9) | block; + a spare slot per lane
};
constexpr int kTileMaxM = 1 << (32 - kLdsPosBits);  // target indices that fit the local key

//
// One tile (every target of the pass fits one tile: C1, C2), `first` >= 0: the workgroup owns its
// queries' whole search, so the seed (the previous match; first pass: the target at the same
// relative sorted position — nn_seed_kernel's rule) is evaluated here, the key is stored, not merged,
// and the correspondence record is written from the winner's LDS slot — one launch per NN pass
// instead of three (seed, search, records), two kernel boundaries fewer per ICP iteration.
__global__ __launch_bounds__(kLdsWG) void nn_tile_kernel(PairArgs a, WorkArgs w, int fitness_pass, int first, int qrun) {
    __shared__ TileShared sh;
    const bool own = first >= 0;  // (single tile: launched with gridDim.x == 1)
    const int tile = blockIdx.x, part = blockIdx.y, p = blockIdx.z;
    const unsigned long long tk_entry = w.pass_ticks ? __builtin_amdgcn_s_memrealtime() : 0;
#if defined(ICP4R_DIAG_TILE) && ICP4R_DIAG_TILE == 1  // (timing diagnostic only: later passes do nothing — wrong results)
    if (first == 0 && !fitness_pass) return;
#endif
    const int phase = uload(&w.state[p].phase);
    if (fitness_pass ? (phase == kPhaseInvalid) : (phase != kPhaseActive)) return;
    const int n = uload(a.src_n + p), m = uload(a.tgt_n + p);
    const int t0 = tile * kLdsTargets, q0 = part * kLdsWaves * qrun;  // (qrun queries per wave: 64, 32, 16, 8)
    if (t0 >= m || q0 >= n) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tm = min(kLdsTargets, m - t0);
    const int nb = (tm + kLdsLeaf - 1) / kLdsLeaf, nsb = (nb + kSuper - 1) / kSuper;
    const int64_t xs0 = (int64_t)p * w.x_stride;
    unsigned long long evals = 0, tests = 0;
    // debug (plan option phase_ticks = 1): workgroup (0, 0, 0)'s stamps in the pass' slots 0..4, and
    // over every workgroup the earliest start (slot 6, as its complement) and the latest end (slot 5)
    unsigned long long* tk = (w.pass_ticks && tid == 0) ? reinterpret_cast<unsigned long long*>(w.pass_ticks) : nullptr;
    const bool tk0 = tk && tile == 0 && part == 0 && p == 0;
    const unsigned long long tk_in = tk ? __builtin_amdgcn_s_memrealtime() : 0;
    if (tk0) tk[0] = tk_in;
    if (tk0) tk[7] = tk_entry;
    if (tk) atomicMax(tk + 6, ~tk_in);

    // Stage the tile (whole superblocks: tsort is padded to them), every load before the first store,
    // with the query's chain of dependent loads beside it: the query's sorted position goes out first,
    // then the tile, then its point and key (behind the position only: the tile's loads stay in
    // flight), the seed target, and the tile's LDS stores while that last load is out.  (The chain had
    // started after the staging barrier: ~1.2 us of a 2k pass' 5.4 per workgroup; behind the tile's
    // loads it would wait for them at its first step.)
    const int r0 = q0 + wave * qrun;  // this wave's run: sorted sources [r0, r0 + qrun)
    const bool wrun = r0 < n;         // (wave-uniform)
    const bool live = wrun && lane < qrun && r0 + lane < n;
    const int sq = live ? r0 + lane : min(r0, n - 1);
    // (unconditional loads, clamped: a load under a branch merges into a copy that waits for it)
    const int o = w.sperm[xs0 + sq];  // idle lanes shadow the run's first query
    __builtin_amdgcn_sched_barrier(0);  // (the order of issue above and below is the point)
    const v4f* tsg = reinterpret_cast<const v4f*>(w.tsort + (int64_t)p * w.t_stride + t0);
    const v4f* tb = reinterpret_cast<const v4f*>(w.tbox + (int64_t)p * 2 * w.b_stride) + 2 * (t0 / kLdsLeaf);
    const v4f* sbg = reinterpret_cast<const v4f*>(w.sbox + (int64_t)p * 2 * w.sb_stride) + 2 * (t0 / (kLdsLeaf * kSuper));
    const int nt = nsb * kSuper * kLdsLeaf;
    constexpr int kPerT = kLdsTargets / kLdsWG;
    v4f tv[kPerT];
#pragma unroll
    for (int k = 0; k < kPerT; ++k) tv[k] = tsg[min(tid + k * kLdsWG, nt - 1)];
    const int nbx = nsb * (kSuper + 1);
    const int bq = min(tid, nbx - 1);
    const bool blk = bq < nsb * kSuper;
    const int bk = blk ? bq : bq - nsb * kSuper;
    const v4f blo = blk ? tb[2 * bk] : sbg[2 * bk], bhi = blk ? tb[2 * bk + 1] : sbg[2 * bk + 1];
    const int sbl = min(lane, nsb - 1);
    const v4f isl = sbg[2 * sbl], ish = sbg[2 * sbl + 1];
    __builtin_amdgcn_sched_barrier(0);

    unsigned long long* bestl = sh.best[wave];
    uint16_t* ring = sh.items[wave];
    NNKey* key = w.nn_key + xs0;
    float x = 0.f, y = 0.f, z = 0.f;
    NNKey init = 0;
    // the fitness pass with w.fit_xform (own plans): the query is final * input_i, formed here as
    // fitness_prep_kernel did (Registration::getFitnessScore's transformPointCloud) and written to X
    const bool fitx = own && fitness_pass && w.fit_xform;
    float4 v = fitx ? a.src[uload(a.src_off + p) + o] : w.X[xs0 + o];
    NNKey k0 = key[o];
    uint32_t j = 0;
    float4 t;
    {
        if (fitx) {
            float T[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) T[q] = uload(&w.state[p].final_T[q]);
            xform_pt(T, v.x, v.y, v.z, v.x, v.y, v.z);
            if (live) st_v4<4>(w.X + xs0 + o, v);
        }
        if (own && first == 0 && !fitness_pass && w.defer_xform) {
            // the previous update's transformCloud(T_inc), deferred to here (one read and write of X
            // per pass instead of a pass over the cloud by the update's one workgroup); every query
            // belongs to one lane of one workgroup of the single tile, which writes it back
            float T[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) T[q] = uload(&w.state[p].T_inc[q]);
            xform_pt(T, v.x, v.y, v.z, v.x, v.y, v.z);
            if (live) st_v4<4>(w.X + xs0 + o, v);
        }
        x = v.x;
        y = v.y;
        z = v.z;
        // the seed (nn_seed_kernel's rule, own: evaluated at the query's current position); loaded on
        // every plan for the same reason (the multi-tile plan does not use it)
        j = (own && first && !seed_key(k0, m)) ? __float_as_uint(w.tsort[(int64_t)p * w.t_stride + ((int64_t)sq * m) / n].w)
                                               : min((uint32_t)key_idx(k0), (uint32_t)(m - 1));
        t = a.tgt[uload(a.tgt_off + p) + j];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < kPerT; ++k) {
        const int i = tid + k * kLdsWG;
        if (i < nt) {
            sh.tl[lds_swz(i)] = tl_slot(tv[k], (__float_as_uint(tv[k].w) << kLdsPosBits) | (uint32_t)i);
        }
    }
    if (tid < nbx) {
        const bool empty = !(blo.x <= bhi.x);
        float* d = blk ? sh.bx[bk] : sh.sbx[bk];
        d[0] = empty ? FLT_MAX : blo.x; d[1] = empty ? FLT_MAX : blo.y; d[2] = empty ? FLT_MAX : blo.z;
        d[3] = empty ? FLT_MAX : bhi.x; d[4] = empty ? FLT_MAX : bhi.y; d[5] = empty ? FLT_MAX : bhi.z;
    }
    __builtin_amdgcn_sched_barrier(0);
    if (wrun) {
        if (own) k0 = make_key(l2_simple(x, y, z, t.x, t.y, t.z), j);
        // the current key in the tile's encoding, ranked after every real target of the same (d², index)
        init = make_key(key_d2(k0), ((uint32_t)key_idx(k0) << kLdsPosBits) | ((1u << kLdsPosBits) - 1));
        bestl[lane] = init;  // (sh.best: not staged)
    }
    if (tk0) tk[2] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (tk0) tk[1] = __builtin_amdgcn_s_memrealtime();
    if (!wrun) return;  // (no barrier follows)
    float bnd = live ? key_d2(k0) * kLbGrow : -1.0f;
    float qlo[3] = {x, y, z}, qhi[3] = {x, y, z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        qlo[k] = wave_minf(qlo[k]);
        qhi[k] = wave_maxf(qhi[k]);
    }
    const float qmax = wave_maxf(bnd);
    const uint32_t lane9 = (uint32_t)lane << 9;
    uint32_t head = 0, tail = 0;
    auto drain = [&](uint32_t cnt) {
        const bool act = (uint32_t)lane < cnt;
        const uint32_t it = ring[(head + lane) & (kRing - 1)];
        const int owner = act ? (int)(it >> 9) : 0;
        const int b = act ? (int)(it & 0x1ffu) : 0;
        const float qx = __shfl(x, owner, 64), qy = __shfl(y, owner, 64), qz = __shfl(z, owner, 64);
        if (act) {
            NNKey k1 = ~0ull;
            v4f cs[kLdsLeaf];
            lds_block(sh.tl, b, cs);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < kLdsLeaf; ++t) {
                const v4f c = cs[t];
                const NNKey kn = make_key(l2_simple(qx, qy, qz, tl_x(c), tl_y(c), tl_z(c)), tl_key(c));
                k1 = kn < k1 ? kn : k1;
            }
            atomicMin(&bestl[owner], k1);
        }
        head += cnt;
        evals += (unsigned long long)cnt * kLdsLeaf;
        bnd = live ? key_d2(bestl[lane]) * kLbGrow : -1.0f;
    };
    // the tile's superblocks some query may reach, visited in order (the run's neighbourhood is
    // unknown here: no seed inside the tile)
    uint64_t cm = __ballot(lane < nsb && box_lb(isl, ish, qlo, qhi) <= qmax);
    tests += nsb;
    for (; cm; cm &= cm - 1) {
        const int sb = __builtin_ctzll(cm);
        const auto* sbb = lds_vbase(&sh.sbx[sb][0]);
        tests += 64;
        if (__ballot(pt_lb(sbb, x, y, z) <= bnd) == 0) continue;
        uint64_t nmk[kSuper];
#pragma unroll
        for (int h = 0; h < kSuper; h += 4) {
            const auto* b4 = (const __attribute__((address_space(3))) v4f*)lds_vbase(&sh.bx[sb * kSuper + h][0]);
            v4f r4[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) r4[i] = b4[i];
            float bb[4][6];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int c = 0; c < 6; ++c) bb[j][c] = r4[(6 * j + c) >> 2][(6 * j + c) & 3];
#pragma unroll
            for (int j = 0; j < 4; ++j) nmk[h + j] = __ballot(pt_lb(bb[j], x, y, z) <= bnd);
        }
        tests += 64 * kSuper;
#pragma unroll
        for (int k = 0; k < kSuper; ++k) {
            const uint64_t mask = nmk[k];
            if (mask == 0) continue;
            const uint32_t slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)mask, tail));
            const uint32_t at = lane_select(mask, (uint32_t)(kRing + lane), slot & (kRing - 1));
            ring[at] = (uint16_t)(lane9 | (uint32_t)(sb * kSuper + k));
            tail += (uint32_t)__builtin_popcountll(mask);
            if (tail - head >= 64) drain(64);
        }
    }
    if (tail != head) drain(tail - head);
    const NNKey kb = bestl[lane];
    if (tk0) tk[3] = __builtin_amdgcn_s_memrealtime();
#if defined(ICP4R_DIAG_TILE) && ICP4R_DIAG_TILE == 2  // (timing diagnostic only: no result stores in later passes — wrong results)
    if (first == 0 && !fitness_pass) {
        if (lane == 0 && kb == 0x1234) key[0] = kb;  // (keeps the search from being optimised away)
        return;
    }
#endif
    if (own) {
        // the seed target lies in the tile and its block's bound cannot prune it, so the winner is a
        // real LDS slot; the sentinel position (kb == init) is handled all the same
        const NNKey ko = kb < init ? make_key(key_d2(kb), lk_idx(kb)) : k0;
        if (live) {
            st_sc<4>(key + o, ko);
            if (w.corr != nullptr && !fitness_pass) {  // PCL numerics: the update's correspondence records
                const float4 t = kb < init ? [&] {
                    const v4f c = sh.tl[lds_swz((int)lk_pos(kb))];
                    return make_float4(tl_x(c), tl_y(c), tl_z(c), 0.f);
                }() : a.tgt[uload(a.tgt_off + p) + key_idx(k0)];
                write_corr_t<4>(w, a, p, o, x, y, z, key_d2(ko), t);
            }
        }
    } else if (live && kb < init) {
        atomicMin(&key[o], make_key(key_d2(kb), lk_idx(kb)));
    }
    if (lane == 0) {
        count_add(w.evals, 0, evals);
        count_add(w.evals, 1, tests);
    }
    if (tk) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        if (tk0) tk[4] = t;
        atomicMax(tk + 5, t);
    }
}

// ---------------------------------------------------------------------------------------------
// Sequential folds over an LDS chunk, one lane per chain: acc = acc + f[k] for k in [0, len), in
// that order — exactly the reference loop.  Groups of 32 floats are read 32 elements ahead in two
// explicit register sets (a/b ping-pong) so the chain runs at the dependent-add latency instead of
// waiting on each LDS round trip.  TAcc = float (the float chains) or double (MSE / fitness: the
// float values are widened, as PCL's double accumulators do).
template <typename TAcc>
__device__ __forceinline__ void add_group(TAcc& acc, const float4 (&g)[8]) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        acc = acc + (TAcc)g[u].x;
        acc = acc + (TAcc)g[u].y;
        acc = acc + (TAcc)g[u].z;
        acc = acc + (TAcc)g[u].w;
    }
}

__device__ __forceinline__ void load_group(float4 (&g)[8], const float* f) {
#pragma unroll
    for (int u = 0; u < 8; ++u) g[u] = *reinterpret_cast<const float4*>(f + 4 * u);
}

// The last < 32 elements of a chain segment: groups of 8 loaded one group ahead, then up to 7 loaded
// together (a dependent scalar loop would wait out one LDS round trip per element — the panel ends of
// pass B cut segments at arbitrary positions).  f needs no alignment.
template <typename TAcc>
__device__ __forceinline__ TAcc fold_tail(const float* f, int len, TAcc acc) {
    int k = 0;
    if (len >= 4) {
        float a0 = f[0], a1 = f[1], a2 = f[2], a3 = f[3];
        for (; k + 4 <= len; k += 4) {
            const int nx = (k + 8 <= len) ? k + 4 : k;  // the next group, or a harmless re-read
            const float b0 = f[nx], b1 = f[nx + 1], b2 = f[nx + 2], b3 = f[nx + 3];
            __builtin_amdgcn_sched_barrier(0);
            acc = acc + (TAcc)a0;
            acc = acc + (TAcc)a1;
            acc = acc + (TAcc)a2;
            acc = acc + (TAcc)a3;
            a0 = b0;
            a1 = b1;
            a2 = b2;
            a3 = b3;
        }
    }
    const int r = len - k;  // 0..3, loaded together
    const float v0 = f[k], v1 = f[k + (r > 1 ? 1 : 0)], v2 = f[k + (r > 2 ? 2 : 0)];
    if (r > 0) acc = acc + (TAcc)v0;
    if (r > 1) acc = acc + (TAcc)v1;
    if (r > 2) acc = acc + (TAcc)v2;
    return acc;
}

// acc + x.x + x.y + x.z + x.w in that order, each IEEE add as v_add_f32 does it, with acc kept in one
// register (the tied operand): the allocator had used a consumed group register as the running sum,
// then copied the next group into place with 16 v_mov per round.
__device__ __forceinline__ float chain_add4(float acc, const float4& x) {
    asm("v_add_f32 %0, %1, %0\n\t"
        "v_add_f32 %0, %2, %0\n\t"
        "v_add_f32 %0, %3, %0\n\t"
        "v_add_f32 %0, %4, %0"
        : "+v"(acc)
        : "v"(x.x), "v"(x.y), "v"(x.z), "v"(x.w));
    return acc;
}

// A panel chain's step over one chunk row (len <= T floats, T a multiple of 8; 16-B aligned): groups
// of 16 floats in two register sets that trade roles (the next group's four ds_read_b128 issued before
// this group's 16 dependent adds, as long as the LDS round trip; no register copies: one set carried
// into the next round had cost 16 v_mov and a full lgkmcnt wait per 16 adds, ~15 cycles per add
// against ~7), the rest through fold_tail — half fold_seq's registers: the panel fold lanes share
// their waves' allocation with the fillers.
__device__ __forceinline__ float fold_row(const float* f, int len, float acc) {
    int k = 0;
    if (len >= 32) {
        float4 a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = *reinterpret_cast<const float4*>(f + 4 * u);
        for (; k + 32 <= len; k += 32) {
#pragma unroll
            for (int u = 0; u < 4; ++u) b[u] = *reinterpret_cast<const float4*>(f + k + 16 + 4 * u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc = chain_add4(acc, a[u]);
            }
            const int nx = (k + 48 <= len) ? k + 32 : k;  // the next group, or a harmless re-read
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] = *reinterpret_cast<const float4*>(f + nx + 4 * u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc = chain_add4(acc, b[u]);
            }
        }
        if (k + 16 <= len) {  // a holds f[k, k + 16)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc = chain_add4(acc, a[u]);
            }
            k += 16;
        }
    }
    return k < len ? fold_tail<float>(f + k, len - k, acc) : acc;
}

#ifndef ICP4R_FOLD_AHEAD
#define ICP4R_FOLD_AHEAD 2  // groups of 32 floats in flight ahead of the adds (1 or 2)
#endif
template <typename TAcc>
__device__ __forceinline__ TAcc fold_seq(const float* f, int len, TAcc acc) {
    int k = 0;
    if (ICP4R_FOLD_AHEAD >= 2 && len >= 96) {
        // three register groups in rotation, two loads in flight while a group is summed: 6.4-6.7
        // cycles per dependent add on gfx950 vs 7.6-9.0 with one group ahead (tools/experiments/chain_bench.hip)
        float4 a[8], b[8], c[8];
        load_group(a, f);
        load_group(b, f + 32);
        for (; k + 96 <= len; k += 96) {
            // the loads past this round re-read group 0 harmlessly when nothing follows
            const int n1 = (k + 128 <= len) ? k + 96 : 0, n2 = (k + 160 <= len) ? k + 128 : 0;
            load_group(c, f + k + 64);
            __builtin_amdgcn_sched_barrier(0);
            add_group(acc, a);
            load_group(a, f + n1);
            __builtin_amdgcn_sched_barrier(0);
            add_group(acc, b);
            load_group(b, f + n2);
            __builtin_amdgcn_sched_barrier(0);
            add_group(acc, c);
        }
        // a, b hold [k, k + 32) and [k + 32, k + 64) when they exist
        if (k + 32 <= len) {
            add_group(acc, a);
            k += 32;
            if (k + 32 <= len) {
                add_group(acc, b);
                k += 32;
            }
        }
        return k < len ? fold_tail<TAcc>(f + k, len - k, acc) : acc;
    }
    if (len >= 32) {
        float4 a[8], b[8];
        load_group(a, f);
        int apos = 0;  // where `a` was loaded from
        // sched_barrier: keep each prefetch ahead of the adds it overlaps (the scheduler would
        // otherwise sink the loads down to their first use and expose the LDS latency again)
        for (; k + 64 <= len; k += 64) {
            load_group(b, f + k + 32);
            __builtin_amdgcn_sched_barrier(0);
            add_group(acc, a);
            apos = (k + 96 <= len) ? k + 64 : k;  // next group, or a harmless re-read
            load_group(a, f + apos);
            __builtin_amdgcn_sched_barrier(0);
            add_group(acc, b);
        }
        if (k + 32 <= len) {
            if (apos != k) load_group(a, f + k);
            add_group(acc, a);
            k += 32;
        }
    }
    return k < len ? fold_tail<TAcc>(f + k, len - k, acc) : acc;
}

// fold_seq with the chain switched at element xa (a wave-uniform multiple of 32): groups before it go
// to acc, the rest to acc2 — a panel end of pass B inside a chunk (the fillers padded the ending
// panel to xa with +0).  One three-group rotation over the whole row: the loads stay in flight across
// the switch, which is a scalar branch per group.
template <typename TAcc>
__device__ __forceinline__ void fold_seq_switch(const float* f, int len, int xa, TAcc& acc, TAcc& acc2) {
    xa = __builtin_amdgcn_readfirstlane(xa);
    auto add = [&](int k, const float4 (&g)[8]) __attribute__((always_inline)) {
        if (k < xa)
            add_group(acc, g);
        else
            add_group(acc2, g);
    };
    int k = 0;
    if (len >= 96) {
        float4 a[8], b[8], c[8];
        load_group(a, f);
        load_group(b, f + 32);
        for (; k + 96 <= len; k += 96) {
            const int n1 = (k + 128 <= len) ? k + 96 : 0, n2 = (k + 160 <= len) ? k + 128 : 0;
            load_group(c, f + k + 64);
            __builtin_amdgcn_sched_barrier(0);
            add(k, a);
            load_group(a, f + n1);
            __builtin_amdgcn_sched_barrier(0);
            add(k + 32, b);
            load_group(b, f + n2);
            __builtin_amdgcn_sched_barrier(0);
            add(k + 64, c);
        }
        if (k + 32 <= len) {
            add(k, a);
            k += 32;
            if (k + 32 <= len) {
                add(k, b);
                k += 32;
            }
        }
    } else {
        for (; k + 32 <= len; k += 32) {
            float4 a[8];
            load_group(a, f + k);
            add(k, a);
        }
    }
    if (k < len) {  // the last < 32 elements belong to the second chain (xa <= the last group's start)
        if (k < xa)
            acc = fold_tail<TAcc>(f + k, len - k, acc);
        else
            acc2 = fold_tail<TAcc>(f + k, len - k, acc2);
    }
}

// Elements [lo, hi) (0 <= lo <= hi <= 32, wave-uniform) of the 32-float window g (16-B aligned), in
// order: the window in one round trip, the adds behind scalar branches.
template <typename TAcc>
__device__ __forceinline__ TAcc fold_window(const float* g, int lo, int hi, TAcc acc) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(g + 4 * u);
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        if (4 * u + 0 >= lo && 4 * u + 0 < hi) acc = acc + (TAcc)v[u].x;
        if (4 * u + 1 >= lo && 4 * u + 1 < hi) acc = acc + (TAcc)v[u].y;
        if (4 * u + 2 >= lo && 4 * u + 2 < hi) acc = acc + (TAcc)v[u].z;
        if (4 * u + 3 >= lo && 4 * u + 3 < hi) acc = acc + (TAcc)v[u].w;
    }
    return acc;
}

// fold_seq over row[a, b) of a 16-B aligned LDS row (a, b wave-uniform): the partial 32-float windows
// at either end in one round trip each, the whole windows between them by fold_seq.
#ifndef ICP4R_SPAN_WINDOW
#define ICP4R_SPAN_WINDOW 0
#endif
template <typename TAcc>
__device__ __forceinline__ TAcc fold_span(const float* row, int a, int b, TAcc acc) {
    if (!ICP4R_SPAN_WINDOW) {  // up to 3 leading elements until row + a is aligned, then fold_seq
        const int a4 = min(b, (a + 3) & ~3);
        if (a < a4) acc = fold_tail<TAcc>(row + a, a4 - a, acc);
        return a4 < b ? fold_seq<TAcc>(row + a4, b - a4, acc) : acc;
    }
    if (b <= a) return acc;
    const int w0 = a & ~31;
    if (b <= w0 + 32) return fold_window<TAcc>(row + w0, a - w0, b - w0, acc);
    if (a > w0) acc = fold_window<TAcc>(row + w0, a - w0, 32, acc);
    const int m0 = a > w0 ? w0 + 32 : w0, m1 = b & ~31;
    if (m1 > m0) acc = fold_seq<TAcc>(row + m0, m1 - m0, acc);
    return b > m1 ? fold_window<TAcc>(row + m1, 0, b - m1, acc) : acc;
}

// The double chains (PCL's MSE sum and getFitnessScore) over values the fillers stored as doubles:
// the widening (exact) is done by the filler waves, so the fold lane only adds — a v_cvt_f64_f32 in
// front of every dependent v_add_f64 had put the chain at ~13.5 cycles per element.  Groups of 16
// doubles (8 x b128), three in rotation as in fold_seq.
__device__ __forceinline__ void load_group_d(double2 (&g)[8], const double* f) {
#pragma unroll
    for (int u = 0; u < 8; ++u) g[u] = *reinterpret_cast<const double2*>(f + 2 * u);
}
__device__ __forceinline__ void add_group_d(double& acc, const double2 (&g)[8]) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        acc = acc + g[u].x;
        acc = acc + g[u].y;
    }
}
__device__ __forceinline__ double fold_seq_d(const double* f, int len, double acc) {
    int k = 0;
    if (len >= 48) {
        double2 a[8], b[8], c[8];
        load_group_d(a, f);
        load_group_d(b, f + 16);
        for (; k + 48 <= len; k += 48) {
            // the loads past this round re-read group 0 harmlessly when nothing follows
            const int n1 = (k + 64 <= len) ? k + 48 : 0, n2 = (k + 80 <= len) ? k + 64 : 0;
            load_group_d(c, f + k + 32);
            __builtin_amdgcn_sched_barrier(0);
            add_group_d(acc, a);
            load_group_d(a, f + n1);
            __builtin_amdgcn_sched_barrier(0);
            add_group_d(acc, b);
            load_group_d(b, f + n2);
            __builtin_amdgcn_sched_barrier(0);
            add_group_d(acc, c);
        }
        // a, b hold [k, k + 16) and [k + 16, k + 32) when they exist
        if (k + 16 <= len) {
            add_group_d(acc, a);
            k += 16;
            if (k + 16 <= len) {
                add_group_d(acc, b);
                k += 16;
            }
        }
    }
    for (; k < len; ++k) acc = acc + f[k];
    return acc;
}

// Brute-force path: the correspondence arrays from the merged NN keys (the pruned kernel writes
// them itself).
__global__ __launch_bounds__(256) void corr_kernel(PairArgs a, WorkArgs w) {
    const int p = blockIdx.y;
    if (uload(&w.state[p].phase) != kPhaseActive) return;
    const int n = uload(a.src_n + p);
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 s = w.X[(int64_t)p * w.x_stride + i];
    write_corr(w, a, p, i, s.x, s.y, s.z, w.nn_key[(int64_t)p * w.x_stride + i], a.tgt + uload(a.tgt_off + p));
}

// ---------------------------------------------------------------------------------------------
// The 3x3 solve and convergence test of one pair (thread 0), shared by both numerics.
struct SolveShared {
    double mom[20];
    double sigma[9], ms[3], md[3];
    SvdWork svd;
    float sigmaf[9];  // PCL numerics: sigma as Eigen's GEMM leaves it (one_over_n applied per panel)
    float mean[6];
    float one_over_n;
    int32_t bnd[16];  // pass B with rejected correspondences: the group's panel starts (point index)
    int32_t wsum[16];  // (its scan's per-wave counts)
    double mse_sum;
    float T_inc[16];
    int32_t flag;  // 0 continue, 1 error (no transform), 2 converged after this transform
};

template <int NUM> struct MomLayout;
template <> struct MomLayout<kNumericsPCL> {  // |C| only: every other sum is a sequential fold
    static constexpr int N = 1, CNT = 0;
};
template <> struct MomLayout<kNumericsF64> {  // Σ w·d·sᵀ [9], Σ w·s [3], Σ w·d [3], Σ w, Σ d², |C|
    static constexpr int N = 18, MSE = 16, CNT = 17;
};

// (solve_pair_body: always inlined — fold_update_res_kernel keeps its pair in registers across the solve,
// and a call would spill every caller-saved one of them; solve_pair: the other kernels' call)
template <int NUM>
__device__ __forceinline__ void solve_pair_body(SolveShared& sh, PairState& st, const KParams& kp) {
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
    // the pair state this serial solve reads, loaded up front (in flight during the SVD): each had
    // been a dependent global load on thread 0's critical path
    float F[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) F[k] = st.final_T[k];
    ConvState cs;
    cs.prev_mse = st.prev_mse;
    cs.similar = st.similar;
    cs.state = st.conv_state;
    const int32_t iters = st.iterations + 1;
    float* Tinc = sh.T_inc;
    mat4_identity(Tinc);
    double mse;
    if constexpr (NUM == kNumericsPCL) {
        // Eigen umeyama, Scalar = float: sigma = one_over_n * Σ d' s'ᵀ (fold_pass_b: Eigen's blocked
        // GEMM, already scaled), float SVD, R as Matrix4f, Rt.col(3) = dst_mean; Rt.col(3) -= R * src_mean.
        // (in registers: umeyama_rotation_f32_reg is umeyama_rotation_f32 with static indices)
        float sg[9], R[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) sg[k] = sh.sigmaf[k];
        umeyama_rotation_f32_reg(sg, R);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int j = 0; j < 3; ++j) Tinc[j * 4 + i] = R[i * 3 + j];
            float rs = R[i * 3 + 0] * sh.mean[0];
            rs = R[i * 3 + 1] * sh.mean[1] + rs;
            rs = R[i * 3 + 2] * sh.mean[2] + rs;
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
    float Fn[16];
    mat4_mul_f(Tinc, F, Fn);  // final_transformation_ = transformation_ * final
#pragma unroll
    for (int k = 0; k < 16; ++k) st.final_T[k] = Fn[k];
    st.iterations = iters;
    const int conv = has_converged(kp.conv, iters, Tinc, mse, cs);
    st.prev_mse = cs.prev_mse;
    st.similar = cs.similar;
    st.conv_state = cs.state;
    if (conv) st.phase = kPhaseConverged;
    sh.flag = conv ? 2 : 0;
}
template <int NUM>
__device__ void solve_pair(SolveShared& sh, PairState& st, const KParams& kp) {
    solve_pair_body<NUM>(sh, st, kp);
}

// transformCloud(*input_transformed, *input_transformed, transformation_) by the whole workgroup.
// (With the cached-neighbour test the update defers this to the next pass's test kernel.)
// seed (w.seed_next): the next NN pass's starting key too — the current NN (its coordinates from the
// correspondence record, its index from the key) at the moved point, as nn_seed_kernel computes it.
template <int WG>
__device__ __forceinline__ void transform_pair(const WorkArgs& w, int p, int n, const float* T_lds, bool seed) {
    float Tl[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) Tl[k] = T_lds[k];
    const int64_t xs0 = (int64_t)p * w.x_stride;
    float4* X = w.X + xs0;
    NNKey* key = w.nn_key + xs0;
    const float4* C = w.corr + xs0 * 2;
    // kPer points per thread with every load in flight before the first store (a load issued after a
    // store waits behind it on vmcnt: one L2 round trip per point otherwise)
    constexpr int kPer = 4;
    for (int i0 = 0; i0 < n; i0 += WG * kPer) {
        float4 s[kPer], t[kPer];
        NNKey k0[kPer];
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const int i = min(i0 + e * WG + (int)threadIdx.x, n - 1);
            s[e] = X[i];
            if (seed) {
                t[e] = C[2 * i + 1];
                k0[e] = key[i];
            }
        }
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const int i = i0 + e * WG + (int)threadIdx.x;
            if (i >= n) break;
            xform_pt(Tl, s[e].x, s[e].y, s[e].z, s[e].x, s[e].y, s[e].z);
            X[i] = s[e];
            if (seed) key[i] = make_key(l2_simple(s[e].x, s[e].y, s[e].z, t[e].x, t[e].y, t[e].z), (uint32_t)key_idx(k0[e]));
        }
    }
}

#ifndef ICP4R_TAIL_PER
#define ICP4R_TAIL_PER 4  // fused test: points per thread per pipelined group
#endif
#ifndef ICP4R_TAIL_REV
#define ICP4R_TAIL_REV 1  // fused test: the pair's point groups last to first
#endif

// ---------------------------------------------------------------------------------------------
// The cached-neighbour test of one pair by one workgroup of WG threads (the update's fused tail, and
// the fitness pass inside fitness_prep_kernel): the same work as nn_cache_test_kernel for the pair —
// X_i's new position (FROM_SRC: T·input_i, the fitness pass' final·input; else T·X_i, the deferred
// transformCloud(T_inc)), the bounds moved by |new − old|, the test against the cached NN; a miss
// sets its bit in the pair's bitmap (built in LDS: `need`, zeroed by the caller) and appends its
// search record; the fitness pass also writes a hit's key (finish_kernel's fitness reads them).
// kPer points per thread per group, software-pipelined: the next group's loads are issued before
// this group's stores, so the stores drain while the loads are in flight (a load issued after a store
// would wait behind it on vmcnt).
// Per point: X (.w = L) and nn_t (.w = target position | sorted position) read, U read (and the
// input point, FROM_SRC); X and U written (the fitness pass: neither bounds nor X, unless the aligned
// cloud is asked for).  The iteration passes write no key: nothing reads one before the fitness pass
// — the update folds recompute d² from X and nn_t, and the next search seeds from the record.
// The miss records stay in LDS (lv / lm, the first lcap of them) and are placed at their ranks in the
// pair's query list (qv / qm) at the end; a pair with more misses than lcap leaves its whole list in
// sq / sm with its bitmap, flagged kMissUnranked, for the search to place.
// The first point group's loads (kPer points per thread: X, the NN record, U) — issued by the update
// before its solve, so their latency hides behind thread 0's SVD (they do not depend on T_inc).
template <int kPer>
struct TailFirst {
    float4 v[kPer], t[kPer];
    float U[kPer];
};
// SUMS: the tail also folds the next pass A's Σs (pair_cache_test); wave 0 folds, waves 1.. test, in
// index order.
template <int WG, int kPer, bool SUMS = false>
__device__ __forceinline__ int tail_group0(int n) {  // first (last-to-first) group's start
    constexpr int WW = SUMS ? WG - 64 : WG;
    const int kStep = WW * kPer, ngrp = (n + kStep - 1) / kStep;
    return (ICP4R_TAIL_REV && !SUMS ? ngrp - 1 : 0) * kStep;
}
template <int WG, int kPer, bool SUMS = false>
__device__ __forceinline__ void tail_prefetch(const WorkArgs& w, int p, int n, TailFirst<kPer>& f) {
    constexpr int WW = SUMS ? WG - 64 : WG;
    if (SUMS && threadIdx.x < 64) return;  // (the fold wave)
    const int wt = SUMS ? (int)threadIdx.x - 64 : (int)threadIdx.x;
    const int64_t xs = (int64_t)p * w.x_stride;
    const int i0 = tail_group0<WG, kPer, SUMS>(n);
#pragma unroll
    for (int e = 0; e < kPer; ++e) {
        const int i = min(i0 + e * WW + wt, n - 1);
        f.v[e] = w.X[xs + i];
        f.t[e] = w.nn_t[xs + i];
        f.U[e] = w.nn_u[xs + i];
    }
}

// A fold wave's issue priority (ICP4R_FOLD_PRIO): its sequential chain is one dependent add after
// another, and the SIMD's other waves (fillers, the fused test's workers) otherwise take the issue
// slots between them.
#ifndef ICP4R_FOLD_PRIO
#define ICP4R_FOLD_PRIO 1
#endif
__device__ __forceinline__ void fold_prio(bool hi) {
    if (ICP4R_FOLD_PRIO) {
        if (hi)
            __builtin_amdgcn_s_setprio(3);
        else
            __builtin_amdgcn_s_setprio(0);
    }
}

// SUMS (the update's tail, eligible pairs): the next pass A's Σs folded here, in index order, over the X
// the test writes — wave 0 lanes 0..2 fold, waves 1.. test (groups of (WG - 64) * kPer points, first
// to last, each group's new coordinates staged in `stg`: two buffers of 3 rows of kSumRow floats); the sums go to
// sums_out[0..2] (the pair state) with *sums_ok = 1.
#ifndef ICP4R_SUMS_PER
#define ICP4R_SUMS_PER 2  // the Σs tail's points per worker and group (4: 185 vs 179.5 us per update)
#endif
constexpr int kSumPer = ICP4R_SUMS_PER;
constexpr int kSumRow = 192 * kSumPer + 4;  // staged points per group (192 workers x kSumPer) + pad
constexpr int kSumBuf = 3 * kSumRow;        // one group's staging; two alternate (double buffer)
// The end of a pair's cached-neighbour test (pair_cache_test; res_update_pair's tail): the per-wave
// counts and work counters, then the miss records — lv / lm in LDS (the first lcap; beyond, sq / sm)
// — placed at their ranks in the pair's query list, or the whole list left unranked in sq / sm with
// the bitmap when it overflowed.  Returns the pair's misses.
template <int WG>
__device__ __forceinline__ int test_place(const WorkArgs& w, int p, int n, int hits, int misses, uint32_t* need,
                                          int32_t* pre, float4* lv, uint2* lm, int lcap, int32_t* wcnt, bool fitness,
                                          uint64_t* stamp) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t xs = (int64_t)p * w.x_stride;
    hits = wave_sumi(hits);
    misses = wave_sumi(misses);
    if (lane == 0) {
        wcnt[wave] = misses;
        count_add(w.evals, 0, (unsigned long long)hits);
        count_add(w.evals, 2, (unsigned long long)hits);
        count_add(w.evals, 3, (unsigned long long)(hits + misses));
        if (!fitness) {  // ... of which in an update's tail
            count_add(w.evals, 5, (unsigned long long)(hits + misses));
            count_add(w.evals, 6, (unsigned long long)hits);
        }
    }
    __syncthreads();
    if (stamp && tid == 0) *stamp = __builtin_amdgcn_s_memrealtime();  // diagnostic: the test's end
    int tot = 0;
    for (int k = 0; k < WG / 64; ++k) tot += wcnt[k];
    if (tot == 0) {
        if (tid == 0) w.miss_cnt[p] = 0;
        return 0;
    }
    const int nwords = (n + 31) >> 5;
    if (tot > lcap) {
        // more misses than LDS records (the few slowly converging pairs): the whole list goes to
        // sq / sm and the bitmap to global memory, and the search places it — a read-back of the
        // overflow here sat on this workgroup's end, which sets the update's launch time
        for (int k = tid; k < lcap; k += WG) {
            w.sq[xs + k] = lv[k];
            w.sm[xs + k] = lm[k];
        }
        uint32_t* gneed = w.need + (int64_t)p * w.need_stride;
        for (int k = tid; k < nwords; k += WG) gneed[k] = need[k];
        if (tid == 0) w.miss_cnt[p] = tot | kMissUnranked;
        return tot;
    }
    // Rank placement: the search reads its item's queries in sorted-position order (a run of 64
    // consecutive ones is a compact box), so every miss record goes to its rank in the bitmap — the
    // word's prefix + the set bits below it.  Done here, where the workgroup owns the whole bitmap,
    // instead of in the search, where it put two barriers and three dependent global round trips in
    // front of every work item.  Word prefixes: wave 0, kNeedWords / 64 words per lane.
    if (wave == 0) {
        constexpr int kW = kNeedWords / 64;
        int c[kW], sum = 0;
#pragma unroll
        for (int j = 0; j < kW; ++j) {
            const int wd = lane * kW + j;
            c[j] = wd < nwords ? __builtin_popcount(need[wd]) : 0;
            sum += c[j];
        }
        int incl = sum;
incl = (int)wave_scan_incl((uint32_t)incl);  // (DPP)
        int run = incl - sum;
#pragma unroll
        for (int j = 0; j < kW; ++j) {
            pre[lane * kW + j] = run;
            run += c[j];
        }
    }
    if (tid == 0) w.miss_cnt[p] = tot;
    __syncthreads();
    float4* qv = w.qv + xs;
    uint2* qm = w.qm + xs;
    auto get = [&](int k, float4& r, uint2& m) {  // (tot <= lcap: every record is in LDS)
        k = min(k, tot - 1);
        r = lv[k];
        m = lm[k];
    };
    // (unconditional: a slot past the list re-read record tot - 1 and writes its very bytes to its
    // very rank again)
    auto put = [&](const float4& r, const uint2& m) {
        const uint32_t sp = min(m.y, (uint32_t)(n - 1));
        const int rk = pre[sp >> 5] + __builtin_popcount(need[sp >> 5] & ((1u << (sp & 31)) - 1u));
        st_v4<1>(&qv[rk], r);
        const uint2 mm = make_uint2((m.x & kNtIdxMask) | (sp << kNtPosShift), m.x >> kNtPosShift);
        st_sc<1>(reinterpret_cast<uint64_t*>(&qm[rk]), (uint64_t)mm.x | ((uint64_t)mm.y << 32));
    };
    for (int k0 = tid; k0 < tot; k0 += 4 * WG) {
        float4 r0, r1, r2, r3;  // (named, not an array: an array went to scratch)
        uint2 m0, m1, m2, m3;
        get(k0, r0, m0);  // all loads of the round first
        get(k0 + WG, r1, m1);
        get(k0 + 2 * WG, r2, m2);
        get(k0 + 3 * WG, r3, m3);
        put(r0, m0);
        put(r1, m1);
        put(r2, m2);
        put(r3, m3);
    }
    return tot;
}

template <int WG, int kPer, bool FROM_SRC, bool SUMS = false>
__device__ __forceinline__ int pair_cache_test(const PairArgs& a, const WorkArgs& w, int p, int n, const float (&T)[16],
                                                uint32_t* need, int32_t* pre, float4* lv, uint2* lm, int lcap,
                                                int32_t* mcount, int32_t* wcnt, bool fitness, uint64_t* stamp = nullptr,
                                                const TailFirst<kPer>* first = nullptr, float* stg = nullptr,
                                                float* sums_out = nullptr, int32_t* sums_ok = nullptr) {
    static_assert(!SUMS || (WG - 64) * kPer <= kSumRow - 4, "staging rows");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int WW = SUMS ? WG - 64 : WG;  // threads that test
    const bool worker = !SUMS || wave >= 1;
    const int wt = SUMS ? tid - 64 : tid;
    const int64_t xs = (int64_t)p * w.x_stride;
    float4* X = w.X + xs;
    float* uu = w.nn_u + xs;
    const float4* nt = w.nn_t + xs;
    const float4* src = FROM_SRC ? a.src + a.src_off[p] : nullptr;
    NNKey* key = w.nn_key + xs;
    constexpr int kStep = WW * kPer;
    int hits = 0, misses = 0;
    float fs = -0.0f;  // SUMS: wave 0 lane k's Σs chain (Eigen's rowwise().sum(): from the first element)
    float4 v[kPer], t[kPer], sv[kPer];
    float U[kPer];
    auto load = [&](int i0, float4 (&vv)[kPer], float4 (&tt)[kPer], float (&UU)[kPer], float4 (&ss)[kPer]) {
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const int i = min(i0 + e * WW + wt, n - 1);
            vv[e] = X[i];
            tt[e] = nt[i];
            UU[e] = uu[i];
            if (FROM_SRC) ss[e] = src[i];
        }
    };
    // Groups are visited last to first (ICP4R_TAIL_REV): the update's pass B has just streamed the
    // pair's X and nn_t front to back, so its most recently fetched lines — the ones still in the
    // L2 / MALL — are the pair's last ones.  (The folds must run in index order; the test may run in
    // any.)
    const int ngrp = (n + kStep - 1) / kStep;
    auto grp0 = [&](int g) { return (ICP4R_TAIL_REV && !SUMS ? ngrp - 1 - g : g) * kStep; };
    if (ngrp > 0 && worker) {
        if (first && !FROM_SRC) {
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                v[e] = first->v[e];
                t[e] = first->t[e];
                U[e] = first->U[e];
            }
        } else {
            load(grp0(0), v, t, U, sv);
        }
    }
    for (int g = 0; g < ngrp; ++g) {
        const int i0 = grp0(g);
        // SUMS: group g is staged in buffer g & 1 while the fold wave folds group g - 1 from the other;
        // the fold wave reaches barrier g only after folding g - 2, whose buffer group g reuses
        float* sg = stg + (g & 1) * kSumBuf;
        if (SUMS && !worker) {  // the fold wave: the group's staged coordinates, in index order
            __syncthreads();    // group g staged
            fold_prio(true);
            if (lane < 3) fs = fold_row(sg + lane * kSumRow, min(kStep, n - i0), fs);
            fold_prio(false);
            continue;
        }
        float4 vn[kPer], tn[kPer], sn[kPer];
        float Un[kPer];
        if (g + 1 < ngrp) load(grp0(g + 1), vn, tn, Un, sn);
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const int i = i0 + e * WW + wt;
            const bool valid = i < n;
            float4 o = v[e];
            if (FROM_SRC)
                xform_pt(T, sv[e].x, sv[e].y, sv[e].z, o.x, o.y, o.z);  // final * input
            else
                xform_pt(T, v[e].x, v[e].y, v[e].z, o.x, o.y, o.z);  // PCL transformCloud, in place
            const float2 Lm = move_lu(make_float2(v[e].w, U[e]), v[e].x, v[e].y, v[e].z, o.x, o.y, o.z);
            o.w = Lm.x;
            const float d2 = l2_simple(o.x, o.y, o.z, t[e].x, t[e].y, t[e].z);
            const bool hit = valid & cache_hit(Lm.x, d2);
            // (the fitness pass: no later pass reads the bounds, and X only for the aligned output —
            // the misses' search records carry their own coordinates)
            if (valid && (!fitness || a.aligned)) st_v4<1>(&X[i], o);
            if (valid && !fitness) st_sc<1>(&uu[i], Lm.y);
            if (SUMS && valid) {
                sg[e * WW + wt] = o.x;
                sg[kSumRow + e * WW + wt] = o.y;
                sg[2 * kSumRow + e * WW + wt] = o.z;
            }
            const int k = wave_append(valid && !hit, mcount);
            if (hit) {
                // the fitness pass' keys are read for their d² only (finish_kernel): a hit's index
                // bits carry its NN's sorted position, no gather of the original index
                if (fitness) key[i] = make_key(d2, nt_tpos(t[e].w));
                ++hits;
            } else if (valid) {
                const uint32_t sp = nt_pos(t[e].w);
                atomicOr(&need[sp >> 5], 1u << (sp & 31));
                if (k < lcap) {
                    lv[k] = make_float4(o.x, o.y, o.z, Lm.y);
                    *reinterpret_cast<uint64_t*>(&lm[k]) =
                        (uint64_t)((uint32_t)i | (nt_tpos(t[e].w) << kNtPosShift)) | ((uint64_t)sp << 32);
                } else {
                    put_miss(w, p, k, sp, i, o.x, o.y, o.z, Lm.y, nt_tpos(t[e].w));
                }
                ++misses;
            }
        }
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            v[e] = vn[e];
            t[e] = tn[e];
            U[e] = Un[e];
            if (FROM_SRC) sv[e] = sn[e];
        }
        if (SUMS) __syncthreads();  // group g staged
    }
    if (SUMS && wave == 0 && lane < 3) {
        sums_out[lane] = fs;
        if (lane == 0 && *sums_ok != -1) *sums_ok = 1;
    }
    return test_place<WG>(w, p, n, hits, misses, need, pre, lv, lm, lcap, wcnt, fitness, stamp);
}

// ---------------------------------------------------------------------------------------------
// fold_update_kernel (PCL numerics): one workgroup per active pair.  Bit-exact float restatement
// of TransformationEstimationSVD (use_umeyama, Scalar = float) and calculateMSE: every sum is the
// sequential fold the reference performs, in correspondence (= source index) order, one lane per
// chain, over LDS chunks that the filler waves stage from the correspondence arrays while the
// fold lanes consume the previous chunk (double buffer: a fold never waits for a gather).
//  pass A: wave 0 lanes 0..6: Σs, Σd (Eigen 3.3 rowwise().sum(): fold from the first element ==
//          fold from -0.0f; Huber: fold of w·x from +0) and Σw (== |C| unweighted);
//          wave 1 lane 0: Σd² in double (MSE) — only when an MSE criterion is live (KParams::
//          need_mse), else wave 1 fills too.  Fillers: waves 2, 3.
//  pass B: wave 0 lanes 0..8: sigma(a, b) = Σ d'_a s'_b (float, from +0) over the float-demeaned
//          points; the fillers (waves 1..3) form the products (a*b, Huber (w*a)*b) so every chain is
//          a plain sum — IEEE addition is commutative, so p + acc == a*b + acc bit for bit.
// Rejected correspondences contribute the fold's identity (-0.0f / +0), i.e. nothing.
constexpr int kFoldWG = 256;
constexpr int kFoldWaves = kFoldWG / 64;
constexpr int kFoldChunkP = 512;  // points per LDS chunk of the fold passes

// Each fold chain's row is padded by kFoldPad floats: unpadded, rows 2 KB apart start on the same
// LDS bank, and the 7-9 fold lanes' ds_read_b128 of one column were a 7-9-way bank conflict on every
// read.  Padded by 16 B they take distinct banks.
#ifndef ICP4R_FOLD_PAD
#define ICP4R_FOLD_PAD 4
#endif
constexpr int kFoldPad = ICP4R_FOLD_PAD;
constexpr int kFoldRow = kFoldChunkP + kFoldPad;

// the fused test's LDS miss records (24 B each) after the bitmap and its prefixes, in the fold buffers
constexpr int kFoldRecs = ((2 * 9 * kFoldRow * 4 - 2 * kNeedWords * 4) / 24) & ~15;
// ... and with the Σs staging rows (pair_cache_test<SUMS>) at the buffers' end
constexpr int kFoldRecsSums = ((2 * 9 * kFoldRow * 4 - 2 * kNeedWords * 4 - 2 * kSumBuf * 4) / 24) & ~15;
struct FoldShared {
    alignas(16) float buf[2][9][kFoldRow];
    float res[8];
    int32_t cnt[kFoldWaves];
    int32_t mcount;  // tail: the pair's miss list length so far
    SolveShared s;
};

// The correspondences an update folds: the NN kernels' records C ({s.xyz, w}, {d.xyz, d²} per point),
// or, with the cached-neighbour test (C == nullptr), X_i (the searched point: the transform is
// deferred) and its NN's coordinates NT[i], d² = l2_simple(X_i, t) — the very expression the NN
// computed its key with, so the same bits.
struct FoldIn {
    const float4* C;
    const float4* X;
    const float4* NT;
    int n;
    uint64_t* tk = nullptr;  // debug (phase ticks, pair 0, thread 0): pass B's sub-phase stamps
    // key mode (WorkArgs::fold_keys, pass A only; C, NT null): the NN of X_i is TG[key_idx(K[i])], and
    // pass A writes the record pair corr_kernel would have written to Cw (pass B then reads them)
    const NNKey* K = nullptr;
    const float4* TG = nullptr;
    float4* Cw = nullptr;
};

// A running exact sum of non-negative doubles that are widened floats: S in units of 2^E (E = the
// lowest set bit's exponent over the nonzero terms so far), saturated at 2^53 — the argument of
// finish_kernel: while S < 2^53 the sequential double loop over the same terms never rounds, so its
// result is S * 2^E.  Each lane keeps its own (S, E) over the terms it is handed (no cross-lane step
// per chunk: the per-chunk wave reductions had cost as much as the float chains beside them);
// wave_exact_total combines the lanes (a lane's saturation means the whole total reaches 2^53).
constexpr uint64_t kExactSat = 1ull << 53;
__device__ __forceinline__ uint64_t exact_rescale(uint64_t S, int sh) {  // S * 2^sh, saturated (sh >= 0)
    return S == 0 ? 0 : ((sh >= 53 || (S >> (53 - sh)) != 0) ? kExactSat : (S << sh));
}
__device__ __forceinline__ void lane_exact_add(double x, uint64_t& S, int& E) {
    if (!(x > 0.0)) return;
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const int ex = (int)((b >> 52) & 0x7ff);
    const uint64_t mant = (b & ((1ull << 52) - 1)) | (1ull << 52);
    const int lo = ex - 1075 + (int)__builtin_ctzll(mant);
    if (lo < E) {  // re-express S in the finer unit (exact while it stays below 2^53)
        S = E == INT_MAX ? 0 : exact_rescale(S, E - lo);
        E = lo;
    }
    // x / 2^E = mant >> (E + 1075 - ex), a shift by at most ctz(mant): exact; below 2^53 iff ex - 1023 - E <= 52
    S = min(S + ((ex - 1023 - E <= 52) ? (mant >> (E + 1075 - ex)) : kExactSat), kExactSat);
}
__device__ __forceinline__ void wave_exact_total(uint64_t& S, int& E) {  // every lane ends with the wave's
    int e = E;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) e = min(e, __shfl_xor(e, off, 64));
    uint64_t t = E == INT_MAX ? 0 : exact_rescale(S, E - e);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t = min(t + __shfl_xor(t, off, 64), kExactSat);
    S = t;
    E = e;
}

constexpr int kSliceGroup = 14;  // panels folded together (9 x 14 = 126 chains: two fold waves)
#ifndef ICP4R_FILL_BATCH
#define ICP4R_FILL_BATCH 2
#endif
constexpr int kFillBatch = ICP4R_FILL_BATCH;  // a filler's correspondences in flight per round

// Pass A of the PCL-numerics update by a workgroup of WG threads over LDS chunks of CH points
// (buf: two chunks of 9 rows of ROW floats): wave 0 lanes 0..6 fold Σs, Σd (Eigen 3.3
// rowwise().sum(): from the first element == from -0.0f; Huber: w·x from +0) and Σw; wave 1 lane 0
// the double MSE chain when an MSE criterion is live (else it fills); the other waves stage the next
// chunk.  Leaves |C|, 1/n and the centroids in s.
// sums (fold_update_kernel, eligible pairs: every correspondence kept, unweighted, no MSE criterion):
// Σs as the previous update's tail folded it over the X it wrote — the fillers read nn_t only, and
// lanes 0..2 do not fold.
template <int WG, int CH, int ROW>
__device__ __forceinline__ void fold_pass_a(const KParams& kp, const FoldIn& f, float (*buf)[9][ROW], float* res,
                                            int32_t* wcnt, SolveShared& s, const float* sums = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool weighted = kp.huber_delta < INFINITY;
    auto rec = [&](int i, float4& r0, float4& r1) {
        if (f.C) {
            r0 = f.C[2 * i];
            r1 = f.C[2 * i + 1];
        } else {
            r0 = f.X[i];
            r1 = f.NT[i];
        }
    };
    auto rec_fix = [&](float4& r0, float4& r1) {
        if (!f.C) {
            const float d2 = l2_simple(r0.x, r0.y, r0.z, r1.x, r1.y, r1.z);
            r0.w = weighted ? (float)huber_w(d2, kp.huber_delta) : 1.0f;
            r1.w = d2;
        }
    };
    const int n = f.n;
    const int nch = (n + CH - 1) / CH;
    const bool mse = kp.need_mse != 0;  // wave 1 runs the MSE chain in pass A, else it fills
    const float ident = weighted ? 0.0f : -0.0f;
    const int fill0 = mse ? 128 : 64;  // first filler thread of pass A
    int cnt = 0;
    // Fillers issue every load of their (at most kPerA) elements before the first LDS store, so a
    // chunk costs one global round trip, not one per element.
    constexpr int kPerA = (CH + (WG - 128) - 1) / (WG - 128);
    // fill: load_a issues the loads of chunk c's records (clamped: at most kPerA per filler),
    // store_a turns them into the chain rows of LDS buffer c & 1.  (Loading two chunks ahead in two
    // register sets, here and in pass B, was measured slower: C3 update 176 -> 189 us per launch at two
    // pair groups — the batched update is bound by its bytes, not by these loads' latency.)
    auto load_a = [&](int c, float4 (&r)[kPerA][2]) __attribute__((always_inline)) {
        const int base = c * CH, len = min(CH, n - base), nf = WG - fill0;
        if (f.K) {  // key mode: X and the keys in flight together, then the targets they name
            uint32_t ti[kPerA];
#pragma unroll
            for (int e = 0; e < kPerA; ++e) {
                const int i = base + min(tid - fill0 + e * nf, len - 1);
                r[e][0] = f.X[i];
                ti[e] = (uint32_t)key_idx(f.K[i]);
            }
#pragma unroll
            for (int e = 0; e < kPerA; ++e) r[e][1] = f.TG[ti[e]];
            return;
        }
#pragma unroll
        for (int e = 0; e < kPerA; ++e) {
            const int i = base + min(tid - fill0 + e * nf, len - 1);
            if (sums)  // nn_t only (X's centroid is known)
                r[e][1] = f.NT[i];
            else
                rec(i, r[e][0], r[e][1]);
        }
    };
    auto store_a = [&](int c, float4 (&r)[kPerA][2]) __attribute__((always_inline)) {  // waves 2, 3 (and 1 without the MSE chain)
        float(*b)[ROW] = buf[c & 1];
        const int base = c * CH, len = min(CH, n - base), nf = WG - fill0;
#pragma unroll
        for (int e = 0; e < kPerA; ++e) {
            const int o = tid - fill0 + e * nf;
            if (o >= len) break;
            if (sums) {  // every correspondence kept, unweighted: Σd and Σw rows only
#pragma unroll
                for (int k = 0; k < 3; ++k) b[3 + k][o] = (&r[e][1].x)[k];
                b[6][o] = 1.0f;
                ++cnt;
                continue;
            }
            rec_fix(r[e][0], r[e][1]);
            const float d2 = r[e][1].w;
            if (f.Cw) {  // corr_kernel's record pair: {s.xyz, w}, {d.xyz, d²}
                f.Cw[2 * (base + o)] = r[e][0];
                f.Cw[2 * (base + o) + 1] = r[e][1];
            }
            const float sv[6] = {r[e][0].x, r[e][0].y, r[e][0].z, r[e][1].x, r[e][1].y, r[e][1].z};
            float v[6], wt = 0.0f, dd = 0.0f;
#pragma unroll
            for (int k = 0; k < 6; ++k) v[k] = ident;
            if (!(d2 > kp.max_d2)) {
                wt = r[e][0].w;
#pragma unroll
                for (int k = 0; k < 6; ++k) v[k] = weighted ? wt * sv[k] : sv[k];
                dd = d2;
                ++cnt;
            }
#pragma unroll
            for (int k = 0; k < 6; ++k) b[k][o] = v[k];
            b[6][o] = wt;
            reinterpret_cast<double*>(b[7])[o] = (double)dd;  // (rows 7-8: the MSE chain's doubles)
        }
    };
    float acc = (lane < 6) ? ident : 0.0f;
    double dacc = 0.0;
    // The roles run as separate wave-uniform loops (the same number of barriers in each), so the
    // fold lanes' register groups and the fillers' in-flight records are never live together.
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    if (wv == 0) {
        const int lane0 = sums ? 3 : 0;
        fold_prio(true);
        for (int c = 0; c < nch; ++c) {
            __syncthreads();
            if (lane >= lane0 && lane < 7) acc = fold_seq<float>(buf[c & 1][lane], min(CH, n - c * CH), acc);
        }
        fold_prio(false);
    } else if (wv * 64 < fill0) {  // the MSE sum: its exact form, the whole wave per chunk
        uint64_t xs = 0;
        int xe = INT_MAX;
        for (int c = 0; c < nch; ++c) {
            __syncthreads();
            const double* dv = reinterpret_cast<const double*>(buf[c & 1][7]);
            const int len = min(CH, n - c * CH);
            for (int o = lane; o < len; o += 64) lane_exact_add(dv[o], xs, xe);
        }
        wave_exact_total(xs, xe);
        // -1: the span test failed (the sequential chain runs below)
        dacc = xs >= kExactSat ? -1.0 : (xe == INT_MAX ? 0.0 : ldexp((double)xs, xe));
    } else {
        if (nch > 0) {
            float4 r[kPerA][2];
            load_a(0, r);
            store_a(0, r);
        }
        for (int c = 0; c < nch; ++c) {
            __syncthreads();
            if (c + 1 < nch) {
                float4 r[kPerA][2];
                load_a(c + 1, r);
                store_a(c + 1, r);
            }
        }
    }
    // |C|: exact integer reduction of the fillers' counts
    cnt = wave_sumi(cnt);
    if (lane == 0) wcnt[wave] = cnt;
    if (wave == 0 && lane < 7) res[lane] = (sums && lane < 3) ? sums[lane] : acc;
    if (wave == 1 && lane == 0) s.mse_sum = dacc;  // 0 without the MSE chain (not used then)
    __syncthreads();
    if (tid == 0) {
        int total = 0;
        for (int k = 0; k < (WG / 64); ++k) total += wcnt[k];
        s.mom[0] = (double)total;
        // unweighted: one_over_n = 1/(float)n (fold of 1.0f == n exactly); Huber: 1/Σw
        const float one_over_n = 1.0f / res[6];
        s.one_over_n = one_over_n;
        for (int k = 0; k < 6; ++k) s.mean[k] = res[k] * one_over_n;
    }
    __syncthreads();
    if (mse && s.mse_sum < 0.0) {  // (uniform) the MSE terms span more than 53 bits: PCL's sequential
        dacc = 0.0;                 // double chain, over the chunks staged again (wave 0 idles)
        if (wv == 0) {
            for (int c = 0; c < nch; ++c) __syncthreads();
        } else if (wv * 64 < fill0) {
            for (int c = 0; c < nch; ++c) {
                __syncthreads();
                if (lane == 0) dacc = fold_seq_d(reinterpret_cast<const double*>(buf[c & 1][7]), min(CH, n - c * CH), dacc);
            }
        } else {
            if (nch > 0) {
                float4 r[kPerA][2];
                load_a(0, r);
                store_a(0, r);
            }
            for (int c = 0; c < nch; ++c) {
                __syncthreads();
                if (c + 1 < nch) {
                    float4 r[kPerA][2];
                    load_a(c + 1, r);
                    store_a(c + 1, r);
                }
            }
        }
        __syncthreads();  // (the last chunk folded before s.mse_sum is rewritten)
        if (wave == 1 && lane == 0) s.mse_sum = dacc;
        __syncthreads();
    }
}

// Pass B: sigma = one_over_n * Σ d'_a·s'_b over the float-demeaned correspondences, in Eigen 3.3's
// GEMM order (icp4r_math.hpp sigma_kc; oracle/icp_oracle.c umeyama_f32): the |C| correspondences are
// cut into S panels of kc, each panel's 9 coefficients are sequential float chains from +0, and the
// panels are added into sigma (from +0) as one_over_n * chain, in panel order.  The fillers form the
// products (Huber: (w·d'_a)·s'_b) and the fold lanes sum them (IEEE addition is commutative:
// p + acc == a·b + acc bit for bit).  Rejected correspondences (d² > max_d2) are not in PCL's list:
// they add the chain's identity (+0) where they fall, and panel boundaries are counted in accepted
// correspondences only (fold_bounds).
//  * one panel (|C| <= 680 at the default host facts): wave 0 lanes 0..8 fold the 9 chains over
//    chunks of CH points, as before;
//  * S panels: up to kSliceGroup panels at once — 9·G chains, one fold lane each (waves 0..1), over
//    LDS chunks that hold T steps of every panel of the group (row (panel, ab) of T floats, rows
//    strided ≡ 4 mod 8 floats so the fold lanes' ds_read_b128 hit distinct banks): the chain per
//    panel is kc long instead of |C|.
// Leaves the finished sigma in s.sigmaf.

// Panel starts of panels [s0, s0 + G] (point indices) when some correspondences are rejected: the
// panel of rank r starts at the point holding the (s·kc)-th accepted correspondence.  A scan over
// the points from the group's first start, WG at a time (ranks by ballot + wave prefix), until the
// group's last boundary is found.  bnd[0] must hold the group's first start; bnd[G] = n when s0 + G
// reaches S.
template <int WG, typename Acc>
__device__ __forceinline__ void fold_bounds(int n, int kc, int S, int s0, int G, Acc accepted, int32_t* bnd,
                                            int32_t* wsum) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int NW = WG / 64;
    const int last = min(s0 + G, S);  // boundaries s0 + 1 .. last
    if (tid == 0 && last == S) bnd[last - s0] = n;
    int base = bnd[0];
    int running = s0 * kc;  // the rank of the first accepted correspondence at or after bnd[0]
    const int stop_rank = (last == S) ? INT_MAX : last * kc;
    while (base < n && running <= stop_rank) {
        const int i = base + tid;
        const bool acc = i < n && accepted(i);
        const uint64_t bal = __ballot(acc);
        const int pre = __builtin_popcountll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wave] = __builtin_popcountll(bal);
        __syncthreads();
        int off = running, tot = running;
#pragma unroll
        for (int v = 0; v < NW; ++v) {
            off += v < wave ? wsum[v] : 0;
            tot += wsum[v];
        }
        const int r = off + pre;
        if (acc && r > s0 * kc && r % kc == 0) {
            const int sl = r / kc;
            if (sl <= last && sl < S) bnd[sl - s0] = i;
        }
        running = tot;
        base += WG;
        __syncthreads();  // (wsum reused)
    }
    __syncthreads();
}

template <int WG, int CH, int ROW, bool PAR>
__device__ __forceinline__ void fold_pass_b(const KParams& kp, const FoldIn& f, float (*buf)[9][ROW], SolveShared& s) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool weighted = kp.huber_delta < INFINITY;
    auto rec = [&](int i, float4& r0, float4& r1) {
        if (f.C) {
            r0 = f.C[2 * i];
            r1 = f.C[2 * i + 1];
        } else {
            r0 = f.X[i];
            r1 = f.NT[i];
        }
    };
    auto rec_fix = [&](float4& r0, float4& r1) {
        if (!f.C) {
            const float d2 = l2_simple(r0.x, r0.y, r0.z, r1.x, r1.y, r1.z);
            r0.w = weighted ? (float)huber_w(d2, kp.huber_delta) : 1.0f;
            r1.w = d2;
        }
    };
    const int n = f.n;
    if (f.tk) f.tk[19] = __builtin_amdgcn_s_memrealtime();
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const float ms[3] = {s.mean[0], s.mean[1], s.mean[2]};
    const float md[3] = {s.mean[3], s.mean[4], s.mean[5]};
    const float oon = s.one_over_n;
    const int cnt = (int)s.mom[0];
    const int kc = sigma_kc(cnt, kp.sigma_max_kc);
    const int S = (cnt > 0 && kc > 0) ? (cnt + kc - 1) / kc : 1;
    // the 9 products of one correspondence (0 when it is rejected)
    auto products = [&](float4 r0, float4 r1, float (&pr)[9]) __attribute__((always_inline)) {
        rec_fix(r0, r1);
        float sv[3] = {0.f, 0.f, 0.f}, dv[3] = {0.f, 0.f, 0.f}, wt = 0.f;
        if (!(r1.w > kp.max_d2)) {
            sv[0] = r0.x - ms[0];
            sv[1] = r0.y - ms[1];
            sv[2] = r0.z - ms[2];
            dv[0] = r1.x - md[0];
            dv[1] = r1.y - md[1];
            dv[2] = r1.z - md[2];
            wt = r0.w;
        }
#pragma unroll
        for (int ra = 0; ra < 3; ++ra)
#pragma unroll
            for (int rb = 0; rb < 3; ++rb) pr[ra * 3 + rb] = weighted ? (wt * dv[ra]) * sv[rb] : dv[ra] * sv[rb];
    };
    // every correspondence kept and unweighted (PCL's defaults): the products need no distance
    const bool plain = !weighted && cnt >= n;  // (nothing rejected in this iteration)
    auto products_plain = [&](const float4& r0, const float4& r1, float (&pr)[9]) __attribute__((always_inline)) {
        const float sv[3] = {r0.x - ms[0], r0.y - ms[1], r0.z - ms[2]};
        const float dv[3] = {r1.x - md[0], r1.y - md[1], r1.z - md[2]};
#pragma unroll
        for (int ra = 0; ra < 3; ++ra)
#pragma unroll
            for (int rb = 0; rb < 3; ++rb) pr[ra * 3 + rb] = dv[ra] * sv[rb];
    };
    if (!PAR || S <= 1) {
        // SEQ: wave 0 lanes 0..8 fold the 9 chains over the points of panels [0, npe) of the range
        // (panel k: [pb(k), pb(k + 1))) in point order, in chunks of up to CB; at each panel end
        // sigma += one_over_n * chain and the chain restarts from +0 — Eigen's panel order with one
        // lane per coefficient, the chain as long as the old single chain.  Chunks are not cut at
        // panel ends (a chunk's staging costs a round trip).  A panel end inside a chunk: the fillers
        // pad the ending panel's rows with +0 up to the next multiple of 32 and shift the new panel's
        // products behind it, so one fold_seq_switch rotation runs the row in whole groups (a
        // remainder would wait out an LDS round trip per few elements); such a chunk holds up to
        // CB - pad points.  Two panel ends in one chunk (only when kc < CB) take the unpadded slow
        // path (fold_span).  The chunk sequence is computed identically by the fold lanes and the
        // fillers (uniform arithmetic), so both run the same number of barriers.
        constexpr int CB = ROW - kFoldPad;  // row capacity (points + pad)
        constexpr int kFillB = WG - 64, kPerB = (CB + kFillB - 1) / kFillB;
        float sig = 0.0f, sacc = 0.0f;  // lane a*3+b of wave 0: sigma(a, b) and the open panel's chain
        struct Chunk {
            int c0, len, xs, k, nb;  // start, points, inner panel end (relative; INT_MAX: none), cursor
            bool multi;
        };
        auto seq = [&](auto pb, int npe) __attribute__((always_inline)) {
            const int p0 = pb(0), p1 = pb(npe);
            // chunk at c0 with the cursor (k, nb: the next panel end > c0)
            auto make = [&](int c0, int k, int nb) -> Chunk {
                Chunk ch;
                ch.c0 = c0;
                ch.k = k;
                ch.nb = nb;
                ch.len = min(CB, p1 - c0);
                ch.xs = INT_MAX;
                ch.multi = false;
                if (nb < c0 + ch.len) {
                    const int xs = nb - c0, xa = (xs + 31) & ~31;
                    ch.multi = k + 1 <= npe && pb(k + 1) < c0 + ch.len;
                    if (!ch.multi) {
                        if (xa >= CB) {
                            ch.len = xs;  // no room for the pad: the chunk ends with the panel
                        } else {
                            ch.xs = xs;
                            ch.len = min(ch.len, CB - (xa - xs));
                        }
                    }
                }
                return ch;
            };
            auto next = [&](const Chunk& ch) -> Chunk {  // the chunk after ch (past its panel ends)
                const int c1 = ch.c0 + ch.len;
                int k = ch.k, nb = ch.nb;
                while (nb <= c1) {
                    ++k;
                    nb = k <= npe ? pb(k) : INT_MAX;
                }
                return make(c1, k, nb);
            };
            auto load_b = [&](const Chunk& ch, float4 (&r)[kPerB][2]) __attribute__((always_inline)) {
#pragma unroll
                for (int e = 0; e < kPerB; ++e) {
                    const int i = ch.c0 + min(tid - 64 + e * kFillB, ch.len - 1);
#ifdef ICP4R_DIAG_REVB  // (timing diagnostic only: pass B reads the points last to first — wrong results)
                    rec(n - 1 - i, r[e][0], r[e][1]);
#else
                    rec(i, r[e][0], r[e][1]);
#endif
                }
            };
            auto store_b = [&](int c, const Chunk& ch, float4 (&r)[kPerB][2]) __attribute__((always_inline)) {
                float(*b)[ROW] = buf[c & 1];
                const int xs = ch.multi ? INT_MAX : ch.xs;
                const int padx = xs != INT_MAX ? ((xs + 31) & ~31) - xs : 0;
                if (plain) {
#pragma unroll
                    for (int e = 0; e < kPerB; ++e) {
                        const int o = tid - 64 + e * kFillB;
                        if (o >= ch.len) break;
                        float pr[9];
                        products_plain(r[e][0], r[e][1], pr);
                        const int at = o < xs ? o : o + padx;
#pragma unroll
                        for (int k = 0; k < 9; ++k) b[k][at] = pr[k];
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < kPerB; ++e) {
                        const int o = tid - 64 + e * kFillB;
                        if (o >= ch.len) break;
                        float pr[9];
                        products(r[e][0], r[e][1], pr);
                        const int at = o < xs ? o : o + padx;
#pragma unroll
                        for (int k = 0; k < 9; ++k) b[k][at] = pr[k];
                    }
                }
                if (tid - 64 < padx)
#pragma unroll
                    for (int k = 0; k < 9; ++k) b[k][xs + tid - 64] = 0.0f;
            };
            Chunk ch = make(p0, 1, npe >= 1 ? pb(1) : INT_MAX);
            if (wv == 0) {
                int k = 1, nb = ch.nb;  // the next panel end
                fold_prio(true);
                for (int c = 0; ch.c0 < p1; ++c) {
                    __syncthreads();
                    const int c0 = ch.c0, c1 = c0 + ch.len;
                    const float* row = buf[c & 1][lane < 9 ? lane : 0];
                    if (!ch.multi) {
                        if (ch.xs == INT_MAX) {
                            if (lane < 9) sacc = fold_seq<float>(row, ch.len, sacc);
                        } else {
                            const int xa = (ch.xs + 31) & ~31;
                            if (lane < 9) {
                                // [0, xs) and the +0 pad into the ending chain, the rest into a new one
                                float acc2 = 0.0f;
                                fold_seq_switch<float>(row, xa + (ch.len - ch.xs), xa, sacc, acc2);
                                sig = sig + oon * sacc;  // res(i, j) += alpha * C0 into the zeroed sigma
                                sacc = acc2;
                            }
                            ++k;
                            nb = k <= npe ? pb(k) : INT_MAX;
                        }
                        if (nb == c1) {  // a panel ends with the chunk
                            if (lane < 9) sig = sig + oon * sacc;
                            sacc = 0.0f;
                            ++k;
                            nb = k <= npe ? pb(k) : INT_MAX;
                        }
                    } else {
                        int q = c0;
                        while (nb <= c1) {
                            if (lane < 9) {
                                sacc = fold_span<float>(row, q - c0, nb - c0, sacc);
                                sig = sig + oon * sacc;
                            }
                            sacc = 0.0f;
                            q = nb;
                            ++k;
                            nb = k <= npe ? pb(k) : INT_MAX;
                        }
                        if (q < c1 && lane < 9) sacc = fold_span<float>(row, q - c0, c1 - c0, sacc);
                    }
                    ch = next(ch);
                }
                fold_prio(false);
            } else {
                if (ch.c0 < p1) {
                    float4 r[kPerB][2];
                    load_b(ch, r);
                    store_b(0, ch, r);
                }
                for (int c = 0; ch.c0 < p1; ++c) {
                    __syncthreads();
                    ch = next(ch);  // the chunk to stage: c + 1
                    if (ch.c0 < p1) {
                        float4 r[kPerB][2];
                        load_b(ch, r);
                        store_b(c + 1, ch, r);
                    }
                }
            }
            __syncthreads();  // (the buffers are reused by the next range)
        };
        // the panels kSliceGroup at a time: their starts in s.bnd — (s0 + k) kc when every
        // correspondence is kept, else counted in accepted correspondences (fold_bounds)
        const bool rejected = cnt < n && S > 1;
        if (tid == 0) s.bnd[0] = 0;
        __syncthreads();
        for (int s0 = 0; s0 < S; s0 += kSliceGroup) {
            const int G = min(kSliceGroup, S - s0);
            if (rejected) {
                auto accepted = [&](int i) {
                    float4 r0, r1;
                    rec(i, r0, r1);
                    rec_fix(r0, r1);
                    return !(r1.w > kp.max_d2);
                };
                fold_bounds<WG>(n, kc, S, s0, G, accepted, s.bnd, s.wsum);
            } else {
                if (tid >= 1 && tid <= G) s.bnd[tid] = (s0 + tid >= S) ? n : (s0 + tid) * kc;
                __syncthreads();
            }
            seq([&](int k) { return s.bnd[k]; }, G);
            if (tid == 0) s.bnd[0] = s.bnd[G];
            __syncthreads();
        }
        if (wave == 0 && lane < 9) s.sigmaf[lane] = sig;
        __syncthreads();
        return;
    }

    // S panels, in groups of up to kSliceGroup
    constexpr int CAP = 9 * ROW;  // floats per chunk buffer
    auto bufs = [&](int k) -> float* { return &buf[k & 1][0][0]; };  // (no local array: it went to scratch)
    const bool rejected = cnt < n;  // some correspondence left PCL's list: panel starts by rank
    float sig = 0.0f;               // wave 0 lanes 0..8: sigma(a, b), the panels added in order
    if (tid == 0) s.bnd[0] = 0;
    __syncthreads();
    if (f.tk) f.tk[18] = __builtin_amdgcn_s_memrealtime();
    for (int s0 = 0; s0 < S; s0 += kSliceGroup) {
        const int G = min(kSliceGroup, S - s0);
        const int R = 9 * G;                                      // fold chains of the group
        const int FW = (R + 63) / 64;                             // fold waves (1 or 2)
        const int nF = WG - 64 * FW;                              // fillers
        if (rejected) {
            auto accepted = [&](int i) {
                float4 r0, r1;
                rec(i, r0, r1);
                rec_fix(r0, r1);
                return !(r1.w > kp.max_d2);
            };
            fold_bounds<WG>(n, kc, S, s0, G, accepted, s.bnd, s.wsum);
        }
        // panel sl of the group covers points [start(sl), start(sl + 1))
        auto start = [&](int sl) -> int {
            return rejected ? s.bnd[sl] : min((s0 + sl) * kc, n);
        };
        int maxlen = 0;
        for (int sl = 0; sl < G; ++sl) maxlen = max(maxlen, (s0 + sl + 1 >= S ? n : start(sl + 1)) - start(sl));
        // chunks of T steps per panel row, double-buffered (one chunk over both buffers, for the
        // 2k clouds' 4 panels, measured slower: its staging takes two round trips and hides nothing)
        const int stride = (((CAP / R) - 4) & ~7) + 4;           // row stride, ≡ 4 mod 8 floats
        const int T = stride - 4;                                 // steps per chunk (a multiple of 8)
        const float invT = 1.0f / (float)T;
        const int nch = (maxlen + T - 1) / T;
        // the fillers' slots of chunk c: slot q = (panel sl, step t), q = sl * T + t
        const int per = (G * T + nF - 1) / nF;
        auto fill = [&](int c) __attribute__((always_inline)) {
            float* b = bufs(c);
            const int me = tid - 64 * FW;
            for (int e0 = 0; e0 < per; e0 += kFillBatch) {
                float4 r[kFillBatch][2];
                int at[kFillBatch];
#pragma unroll
                for (int e = 0; e < kFillBatch; ++e) {
                    const int q = me + (e0 + e) * nF;
                    // q / T by a float reciprocal, corrected (exact for these small q)
                    int sl = (int)((float)q * invT), t = q - sl * T;
                    if (t >= T) { ++sl; t -= T; }
                    if (t < 0) { --sl; t += T; }
                    const int i0 = sl < G ? start(sl) : n;
                    const int i1 = sl < G ? (s0 + sl + 1 >= S ? n : start(sl + 1)) : n;
                    const int i = i0 + c * T + t;
                    at[e] = (e0 + e < per && sl < G && i < i1) ? sl * 9 * stride + t : -1;
                    rec(at[e] >= 0 ? i : 0, r[e][0], r[e][1]);
                }
#pragma unroll
                for (int e = 0; e < kFillBatch; ++e) {
                    if (at[e] < 0) continue;
                    float pr[9];
                    products(r[e][0], r[e][1], pr);
#pragma unroll
                    for (int k = 0; k < 9; ++k) b[at[e] + k * stride] = pr[k];
                }
            }
        };
        float acc = 0.0f;  // fold lane L = sl * 9 + ab: the chain of panel s0 + sl, coefficient ab
        const int L = tid;
        const int my_sl = L / 9;
        const int my_len = (wv < FW && L < R) ? ((s0 + my_sl + 1 >= S ? n : start(my_sl + 1)) - start(my_sl)) : 0;
        if (f.tk && s0 == 0) f.tk[0] = __builtin_amdgcn_s_memrealtime();
        if (wv >= FW && nch > 0) fill(0);
        for (int c = 0; c < nch; ++c) {
            __syncthreads();
            if (f.tk && s0 == 0 && c < 2) f.tk[c == 0 ? 1 : 16] = __builtin_amdgcn_s_memrealtime();
            if (wv < FW) {
                const int len = min(T, my_len - c * T);
                if (L < R && len > 0) acc = fold_row(bufs(c) + L * stride, len, acc);
                if (f.tk && s0 == 0 && c < 2) f.tk[15 + 2 * c] = __builtin_amdgcn_s_memrealtime();
            } else if (c + 1 < nch) {
                fill(c + 1);
            }
        }
        __syncthreads();  // every chunk folded: the buffer of chunk nch (unused) takes the chains
        if (f.tk && s0 == 0) f.tk[2] = __builtin_amdgcn_s_memrealtime();
        float* cs = bufs(nch);
        if (wv < FW && L < R) cs[L] = acc;
        __syncthreads();
        if (wave == 0 && lane < 9)
            for (int sl = 0; sl < G; ++sl) sig = sig + oon * cs[sl * 9 + lane];  // res += alpha * C0
        if (rejected && tid == 0) s.bnd[0] = s.bnd[G];  // the next group's first start
        __syncthreads();
    }
    if (wave == 0 && lane < 9) s.sigmaf[lane] = sig;
    __syncthreads();
    if (f.tk) f.tk[3] = __builtin_amdgcn_s_memrealtime();
}

// The update of pair p; returns the pair's work in the next pass (its misses in the fused test; 0
// when it is not searched again).
__device__ __forceinline__ int fold_update_pair(const PairArgs& a, const WorkArgs& w, int tail_test, int p,
                                                FoldShared& sh) {
    PairState& st = w.state[p];
    if (st.phase != kPhaseActive) return 0;
    const int tid = threadIdx.x;
    const int n = a.src_n[p];
    clear_need(w, p, n, tid, kFoldWG);
    const int64_t xs = w.x_stride;
    const KParams& kp = a.kp;
    const float4* C = w.corr ? w.corr + (int64_t)p * xs * 2 : nullptr;
    const float4* Xp = w.X + (int64_t)p * xs;
    const float4* NT = w.nn_t ? w.nn_t + (int64_t)p * xs : nullptr;

    const bool ticks = w.ticks != nullptr && p == 0 && tid == 0;
    if (ticks) w.ticks[0] = __builtin_amdgcn_s_memrealtime();
#if ICP4R_WG_TICKS  // diagnostic build: every pair's phase stamps in its 10th update (tools/experiments/wg_ticks.py)
    uint64_t* wt = (w.ticks && tid == 0 && st.iterations == 9) ? w.ticks + 32 + 4 * (int64_t)gridDim.x + 8 * (int64_t)p
                                                              : nullptr;
    if (wt) {
        wt[0] = __builtin_amdgcn_s_memrealtime();
        // where the fold wave (wave 0) runs: HW_ID (SIMD [5:4], CU [11:8], SH [12], SE [15:13]) and XCC_ID
        wt[5] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                ((uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
    }
#define WG_TICK(k) \
    if (wt) wt[k] = __builtin_amdgcn_s_memrealtime()
#else
#define WG_TICK(k)
#endif
    const FoldIn fin{C, Xp, NT, n};
    // the previous tail folded this pass A's Σs (w.sums_tail: eligible registrations; the flag is the
    // pair's, set only by a tail that ran)
    const bool sums_tail = w.sums_tail && tail_test && w.nn_u && !C;  // (launch-uniform)
    const bool use_sums = sums_tail && uload(&st.sums_ok) == 1;
    fold_pass_a<kFoldWG, kFoldChunkP, kFoldRow>(kp, fin, sh.buf, sh.res, sh.cnt, sh.s, use_sums ? st.sum_s : nullptr);
    if (use_sums && tid == 0) st.sums_ok = 0;
    if (ticks) w.ticks[1] = __builtin_amdgcn_s_memrealtime();
    WG_TICK(1);
    fold_pass_b<kFoldWG, kFoldChunkP, kFoldRow, false>(kp, fin, sh.buf, sh.s);
    if (ticks) w.ticks[2] = __builtin_amdgcn_s_memrealtime();
    WG_TICK(2);
    // the fused test's first point group is loaded, and its LDS bitmap cleared, while thread 0 solves
    const bool tail = tail_test && w.nn_u;
    int nwork = 0;
    TailFirst<ICP4R_TAIL_PER> tf;
    uint32_t* need = reinterpret_cast<uint32_t*>(&sh.buf[0][0][0]);  // the fold buffers are free now
    if (tail) {
        // (the Σs-folding tail loads its first group itself: a second prefetch layout held across the
        // solve spilled to scratch)
        if (!sums_tail) tail_prefetch<kFoldWG, ICP4R_TAIL_PER>(w, p, n, tf);
        for (int k = tid; k < ((n + 31) >> 5); k += kFoldWG) need[k] = 0u;
        if (tid == 0) sh.mcount = 0;
    }
    if (tid == 0) solve_pair<kNumericsPCL>(sh.s, st, kp);
    __syncthreads();
    if (ticks) w.ticks[3] = __builtin_amdgcn_s_memrealtime();
    WG_TICK(3);
    if (sh.s.flag == 1) return 0;  // error: PCL breaks before transforming
    if (!w.defer_xform) transform_pair<kFoldWG>(w, p, n, sh.s.T_inc, w.seed_next && w.corr);
    // The next pass's cached-neighbour test, fused (tail_test: another iteration follows and the pair
    // is still active): the same work as nn_cache_test_kernel for this pair — the deferred
    // transformCloud(T_inc), the bounds moved, the test, hit keys, the miss bitmap — done here, where
    // its HBM stream overlaps the other workgroups' latency-bound fold chains instead of taking a
    // launch of its own.  The workgroup owns the pair, so the bitmap is built in LDS and stored whole.
    if (tail && sh.s.flag == 0) {
        // the fold buffers: the bitmap (cleared above), its word prefixes and the LDS miss records
        int32_t* pre = reinterpret_cast<int32_t*>(need + kNeedWords);
        float4* lv = reinterpret_cast<float4*>(pre + kNeedWords);
        uint2* lm = reinterpret_cast<uint2*>(lv + (sums_tail ? kFoldRecsSums : kFoldRecs));
        float T[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) T[q] = sh.s.T_inc[q];
#if ICP4R_WG_TICKS
        uint64_t* stamp = wt ? wt + 6 : nullptr;
#else
        uint64_t* stamp = nullptr;
#endif
        if (sums_tail) {
            // the staging rows of the Σs fold at the end of the fold buffers, the miss records before
            float* stg = reinterpret_cast<float*>(&sh.buf[0][0][0]) + (2 * 9 * kFoldRow - 2 * kSumBuf);
            nwork = pair_cache_test<kFoldWG, kSumPer, false, true>(
                a, w, p, n, T, need, pre, lv, lm, kFoldRecsSums, &sh.mcount, sh.cnt, false, stamp, nullptr, stg,
                st.sum_s, &st.sums_ok);
        } else {
            nwork = pair_cache_test<kFoldWG, ICP4R_TAIL_PER, false>(a, w, p, n, T, need, pre, lv, lm, kFoldRecs,
                                                                    &sh.mcount, sh.cnt, false, stamp, &tf);
        }
    }
    if (ticks) w.ticks[4] = __builtin_amdgcn_s_memrealtime();
    WG_TICK(4);
    return nwork;
}

// order_ncu > 0: the next pass's work list is built here, by the launch's last workgroup (the
// nn_order_kernel launch and its kernel boundary removed from every iteration pass).  Every
// workgroup publishes its pair's work word (an agent-scope store: write-through, past every cache),
// waits for it, then counts itself in with an agent-scope add; the workgroup whose add completes
// the launch's count reads the words back with agent-scope (L1-bypassing) loads.  The counter only
// grows (plist_n[3], zeroed per registration): a launch's last add is the one that makes it a
// multiple of the grid size.
// Ordering: this is the measured-valid hand-off of MI355X_MICROARCH.md §Workgroup dispatch (the
// first row of its sc1 table): ONE lane per workgroup, its payload (owork[p]) stored sc1
// (write-through) and drained with s_waitcnt vmcnt(0) before the agent-scope add; the consumer is the
// workgroup whose add came last, told by the add's return value, and every load of the payload is an
// sc1 load issued after that add returned (the other waves: after the barrier below).  The asm
// statement's "memory" clobber keeps the compiler from moving the store past the add.  An acq_rel add
// would instead put an L2 write-back (buffer_wbl2) in every workgroup — 1.7-6.5 us each by the same
// section's price list — for an ordering the sc1 accesses already give.
#ifndef ICP4R_UPD_OCC
#define ICP4R_UPD_OCC 4  // (experiment) workgroups per CU of fold_update_kernel: 4, 3 or 2
#endif
__global__ __launch_bounds__(kFoldWG, ICP4R_UPD_OCC) void fold_update_kernel(PairArgs a, WorkArgs w, int tail_test, int order_ncu) {
    __shared__ FoldShared sh;
    __shared__ OrderShared osh;
    __shared__ int32_t last;
    const int p = xcd_remap(blockIdx.x, gridDim.x);
    const int nwork = fold_update_pair(a, w, tail_test, p, sh);
    if (order_ncu <= 0) return;
    if (threadIdx.x == 0) {
        __hip_atomic_store(w.owork + p, nwork, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = __hip_atomic_fetch_add(w.plist_n + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (old + 1) % (int)gridDim.x == 0 ? 1 : 0;
    }
    __syncthreads();
    if (!last) return;
    order_items<kFoldWG, true>(a, w, (int)gridDim.x, 0, 0, order_ncu, osh);
}

// ---------------------------------------------------------------------------------------------
// fold_update_res_kernel (round 6): the batched update with the pair's points read from HBM once and
// held on chip across pass A, pass B and the fused test.  fold_update_kernel streams X and nn_t three
// times per launch (pass A, pass B, the tail: 1.01 GB for 268 MB of clouds at C3); here a 256-thread
// workgroup holds its pair's <= 8192 points — thread t, column j: point t + 256 j — two workgroups per
// CU: X_i.xyz and the NN's x, y in registers (160 VGPRs), the NN's z and L_i = X_i.w in LDS (L rounded
// down to half precision: a lower bound stays a lower bound, so the cached-neighbour test stays exact —
// a miss is searched — and every result is unchanged).
//  loads:  8 columns' X and nn_t in flight at a time, one batch ahead of pass A's folds;
//  pass A: two columns at a time staged from registers into LDS rows, wave 0 lanes 0..6 fold the seven
//          sequential float chains (Σs, Σd, Σw) over them; |C| is a reduction, and the MSE sum (when a
//          criterion is live) its exact integer form per thread (fold_update_kernel's argument), with
//          PCL's sequential double chain over re-read points as the fallback;
//  pass B: Eigen's panels side by side (fold_pass_b<PAR>'s arithmetic): every thread writes the
//          products of its points whose step (index mod kc) falls into the chunk into the panel rows,
//          117 fold lanes sum them (a correspondence rejected for an overflowing d²: fold_pass_b over
//          re-read points);
//  tail:   the next pass's cached-neighbour test from the held points, U read once; a miss's tag
//          (nn_t.w: positions) read for the misses only.
// Per point and iteration: X and nn_t read (32 B), U read (4 B), X and U written (20 B) — the
// one-read bytes.  Results are bit-identical to fold_update_kernel (the parity tests run both).
constexpr int kResWG = 256;
constexpr int kResCols = kResMaxN / kResWG;  // points per thread: column j = points [256 j, 256 j + 256)
constexpr int kResRowA = kResWG + kFoldPad;  // pass A: one column per chunk
constexpr int kResStage = 7680;              // staging floats (30 KB): pass A rows, pass B panel rows, the
                                             // fallbacks' buffers, the tail's bitmap, prefixes and records
constexpr int kResRecs = ((kResStage - 2 * kNeedWords) * 4 / 24) & ~15;  // the tail's LDS miss records
static_assert(kResMaxN == kResWG * kResCols && kResCols % 8 == 0 && kResCols <= 32, "columns");
static_assert(2 * 7 * kResRowA <= kResStage, "pass A rows");
struct ResShared {
    float qz[kResMaxN];     // the NN's z
    _Float16 L[kResMaxN];   // X_i.w rounded down: the test's lower bounds
    alignas(16) float stage[kResStage];
    float res[8];
    int32_t cnt[kResWG / 64];
    uint64_t mse_s[kResWG / 64];
    int32_t mse_e[kResWG / 64];
    int32_t mcount;
    SolveShared s;
};

#ifndef ICP4R_RES_LB
#define ICP4R_RES_LB 4  // columns' loads in flight at a time
#endif
#ifndef ICP4R_RES_FOLD
#define ICP4R_RES_FOLD fold_row  // pass A's fold (fold_row8 / fold_row3: fewer / more registers)
#endif
typedef float fcols __attribute__((ext_vector_type(kResCols)));  // one coordinate of a thread's columns
typedef uint32_t ucols __attribute__((ext_vector_type(kResCols)));
__device__ __forceinline__ int uni(int j) { return __builtin_amdgcn_readfirstlane(j); }

// x rounded toward -inf to half precision (a lower bound stays one)
__device__ __forceinline__ _Float16 half_down(float x) {
    _Float16 h = (_Float16)x;
    if ((float)h > x) {
        uint16_t b = __builtin_bit_cast(uint16_t, h);
        b = (b & 0x8000u) ? (uint16_t)(b + 1) : (b == 0 ? (uint16_t)0x8001u : (uint16_t)(b - 1));
        h = __builtin_bit_cast(_Float16, b);
    }
    return h;
}

// fold_row with three register sets of 16 in rotation (two groups' loads in flight while one is summed)
__device__ __forceinline__ float fold_row3(const float* f, int len, float acc) {
    int k = 0;
    if (len >= 48) {
        float4 a[4], b[4], c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = *reinterpret_cast<const float4*>(f + 4 * u);
#pragma unroll
        for (int u = 0; u < 4; ++u) b[u] = *reinterpret_cast<const float4*>(f + 16 + 4 * u);
        for (; k + 48 <= len; k += 48) {
            // the loads past this round re-read group 0 harmlessly when nothing follows
            const int n1 = (k + 64 <= len) ? k + 48 : 0, n2 = (k + 80 <= len) ? k + 64 : 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = *reinterpret_cast<const float4*>(f + k + 32 + 4 * u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc = chain_add4(acc, a[u]);
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] = *reinterpret_cast<const float4*>(f + n1 + 4 * u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc = chain_add4(acc, b[u]);
#pragma unroll
            for (int u = 0; u < 4; ++u) b[u] = *reinterpret_cast<const float4*>(f + n2 + 4 * u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc = chain_add4(acc, c[u]);
        }
        // a, b hold [k, k + 16) and [k + 16, k + 32) when they exist
        if (k + 16 <= len) {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc = chain_add4(acc, a[u]);
            k += 16;
            if (k + 16 <= len) {
#pragma unroll
                for (int u = 0; u < 4; ++u) acc = chain_add4(acc, b[u]);
                k += 16;
            }
        }
    }
    return k < len ? fold_row(f + k, len - k, acc) : acc;
}

// A chain's step over an LDS row (16-B aligned) with three register sets of 8 in rotation (two groups'
// loads in flight while one is summed): 24 registers — the on-chip update's fold lane shares its wave's
// allocation with the held points
__device__ __forceinline__ float fold_row8(const float* f, int len, float acc) {
    int k = 0;
    if (len >= 24) {
        float4 a[2], b[2], c[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) a[u] = *reinterpret_cast<const float4*>(f + 4 * u);
#pragma unroll
        for (int u = 0; u < 2; ++u) b[u] = *reinterpret_cast<const float4*>(f + 8 + 4 * u);
        for (; k + 24 <= len; k += 24) {
            const int n1 = (k + 32 <= len) ? k + 24 : 0, n2 = (k + 40 <= len) ? k + 32 : 0;
#pragma unroll
            for (int u = 0; u < 2; ++u) c[u] = *reinterpret_cast<const float4*>(f + k + 16 + 4 * u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 2; ++u) acc = chain_add4(acc, a[u]);
#pragma unroll
            for (int u = 0; u < 2; ++u) a[u] = *reinterpret_cast<const float4*>(f + n1 + 4 * u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 2; ++u) acc = chain_add4(acc, b[u]);
#pragma unroll
            for (int u = 0; u < 2; ++u) b[u] = *reinterpret_cast<const float4*>(f + n2 + 4 * u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 2; ++u) acc = chain_add4(acc, c[u]);
        }
        if (k + 8 <= len) {  // a holds [k, k + 8)
#pragma unroll
            for (int u = 0; u < 2; ++u) acc = chain_add4(acc, a[u]);
            k += 8;
            if (k + 8 <= len) {
#pragma unroll
                for (int u = 0; u < 2; ++u) acc = chain_add4(acc, b[u]);
                k += 8;
            }
        }
    }
    return k < len ? fold_tail<float>(f + k, len - k, acc) : acc;
}

__device__ __forceinline__ int res_update_pair(const PairArgs& a, const WorkArgs& w, int tail_test, int p,
                                               ResShared& sh) {
    PairState& st = w.state[p];
    if (st.phase != kPhaseActive) return 0;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = a.src_n[p];  // <= kResMaxN (launch_update)
    clear_need(w, p, n, tid, kResWG);
    const int64_t xs = (int64_t)p * w.x_stride;
    const float4* Xp = w.X + xs;
    const float4* NT = w.nn_t + xs;
    const KParams& kp = a.kp;
    const bool mse = kp.need_mse != 0;
    const int ncol = (n + kResWG - 1) / kResWG;
    float* const buf = sh.stage;
#if ICP4R_WG_TICKS  // diagnostic build: every pair's phase stamps in its 10th update (tools/experiments/wg_ticks.py)
    uint64_t* wt = (w.ticks && tid == 0 && st.iterations == 9) ? w.ticks + 32 + 4 * (int64_t)gridDim.x + 8 * (int64_t)p
                                                              : nullptr;
#define RES_TICK(k) \
    if (wt) wt[k] = __builtin_amdgcn_s_memrealtime()
    // pair 0's finer stamps (pass A per column, pass B per chunk) after every pair's 8 slots
    uint64_t* wx = (wt && p == 0) ? w.ticks + 32 + 12 * (int64_t)gridDim.x : nullptr;
#define RES_TICKX(k) \
    if (wx) wx[k] = __builtin_amdgcn_s_memrealtime()
#else
#define RES_TICK(k)
#define RES_TICKX(k)
#endif
    RES_TICK(0);

    // ---- the pair, read once, in batches of 8 columns one batch ahead of pass A's folds.  The columns
    // are register vectors indexed by a wave-uniform column number (s_set_gpr_idx: one instruction per
    // access), so every loop over them is a loop, not 32 unrolled copies — an unrolled kernel's code
    // (~0.5 MB) had been fetched from L2 instruction by instruction
    fcols px, py, pz, qx, qy;
    constexpr int kLB = ICP4R_RES_LB;
    float4 lv_[kLB], lt_[kLB];  // a batch in flight
    auto issue = [&](int b) __attribute__((always_inline)) {
#pragma unroll
        for (int e = 0; e < kLB; ++e) {
            const int j = uni(b * kLB + e), i = min(tid + kResWG * j, n - 1);
            if (j < ncol) {
                lv_[e] = Xp[i];
                lt_[e] = NT[i];
            }
        }
    };
    auto extract = [&](int b) __attribute__((always_inline)) {
#pragma unroll
        for (int e = 0; e < kLB; ++e) {
            const int j = uni(b * kLB + e), i = tid + kResWG * j;
            if (j < ncol) {
                px[j] = lv_[e].x;
                py[j] = lv_[e].y;
                pz[j] = lv_[e].z;
                qx[j] = lt_[e].x;
                qy[j] = lt_[e].y;
                sh.qz[i] = lt_[e].z;  // (past n: point n - 1's, never read)
                sh.L[i] = half_down(lv_[e].w);
            }
        }
    };
    issue(0);
    extract(0);
    if (ncol > kLB) issue(1);
    RES_TICK(7);

    // ---- pass A: chunk K = columns 2K, 2K + 1 staged into buffer K & 1 (rows Σs.xyz, Σd.xyz, Σw)
    int cnt = 0;
    uint32_t amask = 0;  // bit j: point t + 256 j is a correspondence (d² <= max_d2)
    uint64_t ms_s = 0;
    int ms_e = INT_MAX;
    auto stage_col = [&](int j) __attribute__((always_inline)) {
        j = uni(j);
        const int i = tid + kResWG * j;
        if (i >= n) return;
        float* b = buf + (j & 1) * 7 * kResRowA + tid;
        const float z = sh.qz[i];
        const float d2 = l2_simple(px[j], py[j], pz[j], qx[j], qy[j], z);
        const bool ok = !(d2 > kp.max_d2);  // (max_d2 = FLT_MAX: only an overflowing d² is rejected)
        b[0] = ok ? px[j] : -0.0f;
        b[kResRowA] = ok ? py[j] : -0.0f;
        b[2 * kResRowA] = ok ? pz[j] : -0.0f;
        b[3 * kResRowA] = ok ? qx[j] : -0.0f;
        b[4 * kResRowA] = ok ? qy[j] : -0.0f;
        b[5 * kResRowA] = ok ? z : -0.0f;
        b[6 * kResRowA] = ok ? 1.0f : 0.0f;
        cnt += ok ? 1 : 0;
        amask |= ok ? 1u << j : 0u;
        if (mse) lane_exact_add(ok ? (double)d2 : 0.0, ms_s, ms_e);
    };
    float acc = (lane < 6) ? -0.0f : 0.0f;  // Eigen's rowwise().sum() from the first element; Σw from 0
    if (ncol > 0) stage_col(0);
    for (int K = 0; K < ncol; ++K) {
        __syncthreads();  // column K staged; buffer (K + 1) & 1 folded (column K - 1)
        if (wave == 0 && lane < 7) {
            fold_prio(true);
            acc = ICP4R_RES_FOLD(buf + ((K & 1) * 7 + lane) * kResRowA, min(kResWG, n - K * kResWG), acc);
            fold_prio(false);
        }
        RES_TICKX(K);
        // the next batch of columns arrives before column K + 1 needs it; the one after goes in flight
        if ((K + 1) % kLB == 0 && K + 1 < ncol) {
            extract((K + 1) / kLB);
            if (K + 1 + kLB < ncol) issue((K + 1) / kLB + 1);
        }
        if (K + 1 < ncol) stage_col(K + 1);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if (mse) wave_exact_total(ms_s, ms_e);
    if (lane == 0) {
        sh.cnt[wave] = cnt;
        sh.mse_s[wave] = ms_s;
        sh.mse_e[wave] = ms_e;
    }
    if (wave == 0 && lane < 7) sh.res[lane] = acc;
    __syncthreads();
    if (tid == 0) {
        int total = 0;
        for (int k = 0; k < kResWG / 64; ++k) total += sh.cnt[k];
        sh.s.mom[0] = (double)total;
        // unweighted: one_over_n = 1/(float)n (fold of 1.0f == n exactly)
        const float one_over_n = 1.0f / sh.res[6];
        sh.s.one_over_n = one_over_n;
        for (int k = 0; k < 6; ++k) sh.s.mean[k] = sh.res[k] * one_over_n;
        double msum = 0.0;  // (0 without an MSE criterion: not used then)
        if (mse) {  // the waves' exact sums combined (-1: the terms span more than 53 bits)
            int e = INT_MAX;
            for (int k = 0; k < kResWG / 64; ++k) e = min(e, sh.mse_e[k]);
            uint64_t t = 0;
            for (int k = 0; k < kResWG / 64; ++k)
                t = min(t + (sh.mse_e[k] == INT_MAX ? 0 : exact_rescale(sh.mse_s[k], sh.mse_e[k] - e)), kExactSat);
            msum = t >= kExactSat ? -1.0 : (e == INT_MAX ? 0.0 : ldexp((double)t, e));
        }
        sh.s.mse_sum = msum;
    }
    __syncthreads();
    if (mse && sh.s.mse_sum < 0.0) {
        // (rare) the terms span more than 53 bits: PCL's sequential double chain (calculateMSE) over the
        // points' d² (rejected: +0, which changes no partial sum), re-read from HBM a column at a time so
        // that no register of the held pair is needed; thread 0 adds them in order
        double* db = reinterpret_cast<double*>(buf);
        double dacc = 0.0;
        for (int c = 0; c < ncol; ++c) {
            const int i = c * kResWG + tid;
            if (i < n) {
                const float4 v = Xp[i], t = NT[i];
                const float d2 = l2_simple(v.x, v.y, v.z, t.x, t.y, t.z);
                db[tid] = (double)(!(d2 > kp.max_d2) ? d2 : 0.0f);
            }
            __syncthreads();
            if (tid == 0)
                for (int k = 0, len = min(kResWG, n - c * kResWG); k < len; ++k) dacc = dacc + db[k];
            __syncthreads();
        }
        if (tid == 0) sh.s.mse_sum = dacc;
        __syncthreads();
    }
    RES_TICK(1);

    // ---- pass B: sigma in Eigen's panel order, the panels side by side (fold_pass_b<PAR>'s arithmetic).
    // A point's step is its rank among the correspondences (its index when every point is one) mod kc.
    {
        const int cntA = (int)sh.s.mom[0];
        const bool plain = cntA >= n;
        int32_t* base = reinterpret_cast<int32_t*>(buf);  // (rejections: rank of (column, wave)'s first point)
        if (!plain) {
            for (int j = 0; j < ncol; ++j) {
                const uint64_t bal = __ballot((amask >> j) & 1u);
                if (lane == 0) base[j * 4 + wave] = __builtin_popcountll(bal);
            }
            __syncthreads();
            if (wave == 0) {  // exclusive scan in point order (column-major, then wave)
                const int c0 = lane < 2 * ncol ? base[2 * lane] : 0, c1 = lane < 2 * ncol ? base[2 * lane + 1] : 0;
                int incl = c0 + c1;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const int o = __shfl_up(incl, off, 64);
                    if (lane >= off) incl += o;
                }
                if (lane < 2 * ncol) {
                    base[2 * lane] = incl - c0 - c1;
                    base[2 * lane + 1] = incl - c1;
                }
            }
            __syncthreads();
        }
        // rank of point t + 256 j among the correspondences (-1: rejected); every lane calls it
        auto rank = [&](int j) __attribute__((always_inline)) -> int {
            if (plain) return tid + kResWG * j < n ? tid + kResWG * j : -1;
            const uint32_t on = (amask >> j) & 1u;
            const uint64_t bal = __ballot(on);
            const int r = base[j * 4 + wave] +
                          (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            return on ? r : -1;
        };
        const float oon = sh.s.one_over_n;
        const int kc = sigma_kc(cntA, kp.sigma_max_kc);
        const int S = (cntA > 0 && kc > 0) ? (cntA + kc - 1) / kc : 1;
        const float invkc = 1.0f / (float)kc;
        float sig = 0.0f;  // wave 0 lanes 0..8: sigma(a, b), the panels added in order
        for (int s0 = 0; s0 < S; s0 += kSliceGroup) {
            const int G = min(kSliceGroup, S - s0);
            const int R = 9 * G;                                   // fold chains of the group
            const int stride = (((kResStage / R) - 4) & ~7) + 4;  // one buffer: rows of T steps, ≡ 4 mod 8
            const int T = stride - 4;
            const int r0 = s0 * kc;                                // the group's first rank
            const int r1 = min((s0 + G) * kc, cntA);
            const int nch = (min(kc, r1 - r0) + T - 1) / T;
            // fold lane L = sl * 9 + ab: the chain of panel s0 + sl, coefficient ab
            const int my_len = tid < R ? min(kc, cntA - (s0 + tid / 9) * kc) : 0;
            const float invT = 1.0f / (float)T;
            // (rejections) each column's point in this group: chunk | panel << 8 | step in the chunk << 16
            // (chunk 255: none) — one register per column, read by the chunk scan with the column index
            ucols info;
            if (!plain) {
#pragma unroll
            for (int j = 0; j < kResCols; ++j) {
                uint32_t v = 255u;
                if (j < ncol) {
                    const int r = rank(j) - r0;
                    if (r >= 0 && r < r1 - r0) {
                        int sl = (int)((float)r * invkc);  // r / kc, corrected (exact for these r)
                        int sp = r - sl * kc;
                        if (sp >= kc) { ++sl; sp -= kc; }
                        if (sp < 0) { --sl; sp += kc; }
                        int c = (int)((float)sp * invT);
                        if (c * T > sp) --c;
                        if ((c + 1) * T <= sp) ++c;
                        v = (uint32_t)min(c, 254) | ((uint32_t)sl << 8) | ((uint32_t)(sp - c * T) << 16);
                    }
                }
                info[j] = v;
            }
            }
            if (s0 == 0) RES_TICK(5);
            float accp = 0.0f;
            for (int c = 0; c < nch; ++c) {
                const int w0 = c * T;  // the chunk's first step
                // the means, re-read per chunk as wave-uniform (SGPR) values: hoisted out of the chunk
                // loop, the demeaned coordinates had gone to scratch
                float mv[6];
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    mv[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sh.s.mean[k])));
                    asm volatile("" : "+s"(mv[k]));
                }
                const float ms0 = mv[0], ms1 = mv[1], ms2 = mv[2], md0 = mv[3], md1 = mv[4], md2 = mv[5];
                // every thread writes the products of its points whose step lies in [w0, w0 + T)
                auto put = [&](int j, uint32_t sl, uint32_t tt) __attribute__((always_inline)) {
                    const int i = tid + kResWG * j;
                    const float sv0 = px[j] - ms0, sv1 = py[j] - ms1, sv2 = pz[j] - ms2;
                    const float dv0 = qx[j] - md0, dv1 = qy[j] - md1, dv2 = sh.qz[i] - md2;
                    float* o = buf + sl * 9 * stride + tt;
                    o[0] = dv0 * sv0;
                    o[stride] = dv0 * sv1;
                    o[2 * stride] = dv0 * sv2;
                    o[3 * stride] = dv1 * sv0;
                    o[4 * stride] = dv1 * sv1;
                    o[5 * stride] = dv1 * sv2;
                    o[6 * stride] = dv2 * sv0;
                    o[7 * stride] = dv2 * sv1;
                    o[8 * stride] = dv2 * sv2;
                };
                if (plain) {
                    // a point's rank is its index: panel sl's steps [w0, w0 + T) are the points [a, b), in
                    // one or two columns (wave-uniform bounds)
                    for (int sl = 0; sl < G; ++sl) {
                        const int a = r0 + sl * kc + w0;
                        const int b = min(a + T, min(r0 + (sl + 1) * kc, r1));
                        for (int j0 = a / kResWG; a < b && j0 <= (b - 1) / kResWG; ++j0) {
                            const int j = uni(j0);
                            const int i = tid + kResWG * j;
                            if (i >= a && i < b) put(j, (uint32_t)sl, (uint32_t)(i - a));
                        }
                    }
                } else {
                    for (int j0 = 0; j0 < ncol; ++j0) {
                        const int j = uni(j0);
                        const uint32_t v = info[j];
                        if ((v & 255u) == (uint32_t)c) put(j, (v >> 8) & 255u, v >> 16);
                    }
                }
                __syncthreads();  // the chunk staged
                if (s0 == 0) RES_TICKX(32 + 2 * c);
                if (tid < R) {
                    const int len = min(T, my_len - w0);
                    if (len > 0) accp = fold_row(buf + tid * stride, len, accp);
                }
                __syncthreads();  // the chunk folded: the buffer is free
                if (s0 == 0) RES_TICKX(33 + 2 * c);
            }
            if (tid < R) buf[tid] = accp;
            __syncthreads();
            if (wave == 0 && lane < 9)
                for (int k = 0; k < G; ++k) sig = sig + oon * buf[k * 9 + lane];  // res += alpha * C0
            __syncthreads();
        }
        if (wave == 0 && lane < 9) sh.s.sigmaf[lane] = sig;
    }
    RES_TICK(2);

    // ---- the solve (thread 0), the tail's bitmap cleared meanwhile
    uint32_t* need = reinterpret_cast<uint32_t*>(buf);  // (pass B's buffers are free)
    int32_t* pre = reinterpret_cast<int32_t*>(need + kNeedWords);
    float4* lv = reinterpret_cast<float4*>(pre + kNeedWords);
    uint2* lm = reinterpret_cast<uint2*>(lv + kResRecs);
    static_assert(2 * kNeedWords * 4 + kResRecs * 24 <= kResStage * 4, "tail records");
    // the tail's U, every column in flight across the solve (one register per column)
    const bool tail = tail_test && w.nn_u;
    float* uu = w.nn_u + xs;
    fcols uv;
    if (tail) {
#pragma unroll
        for (int j = 0; j < kResCols; ++j)
            if (j < ncol) uv[j] = uu[min(tid + kResWG * j, n - 1)];
        for (int k = tid; k < ((n + 31) >> 5); k += kResWG) need[k] = 0u;
        if (tid == 0) sh.mcount = 0;
    }
    __syncthreads();  // (sigmaf, and pass B's last reads of the buffer)
    if (tid == 0) solve_pair_body<kNumericsPCL>(sh.s, st, kp);
    __syncthreads();
    RES_TICK(3);
    if (sh.s.flag != 0 || !tail) return 0;  // error, converged, or no further pass

    // ---- tail: the next pass's cached-neighbour test (pair_cache_test's arithmetic)
    float T[16];  // (wave-uniform: SGPR operands of the transform)
#pragma unroll
    for (int q = 0; q < 16; ++q) T[q] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sh.s.T_inc[q])));
    float4* X = w.X + xs;
    float4* sqg = w.sq + xs;
    uint2* smg = w.sm + xs;
    int hits = 0, misses = 0;
    for (int j0 = 0; j0 < ncol; ++j0) {
        const int j = uni(j0);
        const int i = tid + kResWG * j;
        const bool valid = i < n;
        float ox, oy, oz;
        xform_pt(T, px[j], py[j], pz[j], ox, oy, oz);  // PCL transformCloud, in place
        const float2 Lm = move_lu(make_float2((float)sh.L[i], uv[j]), px[j], py[j], pz[j], ox, oy, oz);
        const float d2 = l2_simple(ox, oy, oz, qx[j], qy[j], sh.qz[i]);
        const bool hit = valid & cache_hit(Lm.x, d2);
        if (valid) {
            st_v4<1>(&X[i], make_float4(ox, oy, oz, Lm.x));
            st_sc<1>(&uu[i], Lm.y);
        }
        const bool miss = valid && !hit;
        const int k = wave_append(miss, &sh.mcount);
        if (hit) {
            ++hits;
        } else if (miss) {  // the record without its positions (nn_t.w: read below, for the misses only)
            if (k < kResRecs) {
                lv[k] = make_float4(ox, oy, oz, Lm.y);
                lm[k] = make_uint2((uint32_t)i, 0u);
            } else {
                sqg[k] = make_float4(ox, oy, oz, Lm.y);
                smg[k] = make_uint2((uint32_t)i, 0u);
            }
            ++misses;
        }
    }
    RES_TICK(6);
    // every record appended: the overflow records' stores drained before the barrier (another wave
    // reads them back below, with L1-bypassing loads)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // the misses' positions: nn_t.w (the NN's sorted target position | the query's sorted position)
    const int tot = sh.mcount;
    for (int k0 = tid; k0 < tot; k0 += 4 * kResWG) {
        uint32_t ii[4];
        float tg[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int k = min(k0 + e * kResWG, tot - 1);
            ii[e] = k < kResRecs ? lm[k].x
                                 : __hip_atomic_load(reinterpret_cast<uint32_t*>(smg + k), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
            ii[e] = min(ii[e], (uint32_t)(n - 1));  // (a record's index is below n)
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) tg[e] = NT[ii[e]].w;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int k = k0 + e * kResWG;
            if (k >= tot) break;
            const uint32_t sp = nt_pos(tg[e]);
            atomicOr(&need[sp >> 5], 1u << (sp & 31));
            const uint2 m = make_uint2(ii[e] | (nt_tpos(tg[e]) << kNtPosShift), sp);
            if (k < kResRecs)
                lm[k] = m;
            else
                smg[k] = m;
        }
    }
    const int tp = test_place<kResWG>(w, p, n, hits, misses, need, pre, lv, lm, kResRecs, sh.cnt, false, nullptr);
    RES_TICK(4);
#undef RES_TICK
#undef RES_TICKX
    return tp;
}

__global__ __launch_bounds__(kResWG, 2) void fold_update_res_kernel(PairArgs a, WorkArgs w, int tail_test,
                                                                     int order_ncu) {
    __shared__ ResShared sh;
    __shared__ OrderShared osh;
    __shared__ int32_t last;
    const int p = xcd_remap(blockIdx.x, gridDim.x);
    const int nwork = res_update_pair(a, w, tail_test, p, sh);
    if (order_ncu <= 0) return;
    // the next pass's work list by the launch's last workgroup (fold_update_kernel's hand-off)
    if (threadIdx.x == 0) {
        __hip_atomic_store(w.owork + p, nwork, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = __hip_atomic_fetch_add(w.plist_n + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (old + 1) % (int)gridDim.x == 0 ? 1 : 0;
    }
    __syncthreads();
    if (!last) return;
    order_items_body<kResWG, true>(a, w, (int)gridDim.x, 0, 0, order_ncu, osh);
}

// ---------------------------------------------------------------------------------------------
// fold_update_wide_kernel: the update of plans with at most one pair per CU (single pairs — the node's
// per-frame call, C1 / C2 / C5 — and small batches; no fused cache test, no fused work list): one
// 1024-thread workgroup and most of the CU's LDS per pair.  Pass A is the same sequential centroid
// chains over larger chunks; pass B runs the sigma panels side by side (fold_pass_b<PAR>: up to 14
// panels, 9 chains each, over chunks of 128 steps per panel), so its chain is one panel (kc) long
// instead of |C|, and the 14 filler waves stage a chunk in one round trip.  Same results bit for bit
// as fold_update_kernel (the parity tests run both; plan option wide_update = 0 selects the narrow one).
constexpr int kWideWG = 1024;
constexpr int kWideChunkP = 1792;  // points per pass-A chunk; pass B: 9 x 14 panel rows of 128 steps
constexpr int kWideRow = kWideChunkP + kFoldPad;
struct WideShared {
    alignas(16) float buf[2][9][kWideRow];
    float res[8];
    int32_t cnt[kWideWG / 64];
    int32_t lay[5];  // fold_update_held_kernel: pass B's layout (kc, S, stride, T, chunks), by thread 0
    SolveShared s;
};

__global__ __launch_bounds__(kWideWG) void fold_update_wide_kernel(PairArgs a, WorkArgs w) {
    __shared__ WideShared sh;
    const int p = xcd_remap(blockIdx.x, gridDim.x);
    PairState& st = w.state[p];
    if (st.phase != kPhaseActive) return;
    const int tid = threadIdx.x;
    const int n = a.src_n[p];
    clear_need(w, p, n, tid, kWideWG);
    const int64_t xs = w.x_stride;
    const KParams& kp = a.kp;
    const float4* C = w.corr ? w.corr + (int64_t)p * xs * 2 : nullptr;
    const float4* Xp = w.X + (int64_t)p * xs;
    const float4* NT = w.nn_t ? w.nn_t + (int64_t)p * xs : nullptr;
    const bool ticks = w.ticks != nullptr && p == 0 && tid == 0;
    if (ticks) w.ticks[0] = __builtin_amdgcn_s_memrealtime();
    const FoldIn fin{C, Xp, NT, n, ticks ? w.ticks + 12 : nullptr};
    // fold_keys: pass A reads X and the merged keys' targets and writes the records pass B reads
    // (corr_kernel's work, without its launch)
    FoldIn fa = fin;
    if (w.fold_keys && C) {
        fa.C = nullptr;
        fa.K = w.nn_key + (int64_t)p * xs;
        fa.TG = a.tgt + a.tgt_off[p];
        fa.Cw = const_cast<float4*>(C);
    }
    fold_pass_a<kWideWG, kWideChunkP, kWideRow>(kp, fa, sh.buf, sh.res, sh.cnt, sh.s);
    if (ticks) w.ticks[1] = __builtin_amdgcn_s_memrealtime();
    fold_pass_b<kWideWG, kWideChunkP, kWideRow, true>(kp, fin, sh.buf, sh.s);
    if (ticks) w.ticks[2] = __builtin_amdgcn_s_memrealtime();
#ifdef ICP4R_SOLVE_PROBE
    // debug: the rotation of this sigma twice, back to back (ticks[5], [6]: durations) — a cold
    // instruction cache shows as a first run much slower than the second
    if (ticks) {
        for (int rep = 0; rep < 2; ++rep) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            float z;
            asm volatile("v_mov_b32 %0, 0" : "=v"(z));
            float sg[9], R[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) sg[k] = sh.s.sigmaf[k] + z;
            umeyama_rotation_f32_reg(sg, R);
#pragma unroll
            for (int k = 0; k < 9; ++k) asm volatile("" ::"v"(R[k]));
            w.ticks[5 + rep] = __builtin_amdgcn_s_memrealtime() - t0;
        }
    }
#endif
    if (tid == 0) solve_pair<kNumericsPCL>(sh.s, st, kp);
    __syncthreads();
    if (ticks) w.ticks[3] = __builtin_amdgcn_s_memrealtime();
    if (sh.s.flag == 1) return;  // error: PCL breaks before transforming
    if (!w.defer_xform) transform_pair<kWideWG>(w, p, n, sh.s.T_inc, w.seed_next && w.corr);
    if (ticks) w.ticks[4] = __builtin_amdgcn_s_memrealtime();
}

// ---------------------------------------------------------------------------------------------
// fold_update_held_kernel<HOLD, S0> (round 6): fold_update_wide_kernel for sources of at most
// HOLD x F points (F filler threads: <3, true> up to 2,112 — the node's 2k C1 scan, F = 704; <10, false>
// up to 8,960 — the 8k scans of C2 / C5, F = 896), with the pair's correspondence records read from
// HBM once per update.  The filler threads (waves 2..15; S0: but 4, 8, 12) load their records (record
// i is filler i mod F's slot i / F) — chunk 0's two slots first, the rest after the first barrier —
// and keep each as six floats in registers (s and d; d² and the weight are
// recomputed — the search formed the record's d² as l2_simple(s, d) and its weight from that, with
// contraction off, so the same bits): pass A's chunk c is slots 2c and 2c + 1 of every filler (LDS
// stores only, no round trip per chunk), and pass B's panel chunks take each record's nine products
// from the filler that holds it — the wide kernel's fill of every pass-B chunk was a global round trip
// (C1: pass B 7.7 -> 5.2 us; 2.3 us of it had been the first fill).  Waves 0 and 1 (the fold lanes,
// the MSE wave) hold nothing: the roles run as separate wave-uniform loops, so the held records are
// never live beside fold_seq's 96 registers.  The chains, their orders and the panel adds are
// fold_pass_a / fold_pass_b<PAR>'s, so the results are the wide kernel's bit for bit; pass B takes that
// kernel's global path when a correspondence was rejected or weighted (the panels then start by rank),
// for one panel, or for more panels than one group.
constexpr int kHeldFill0 = 128;                       // first filler thread
// S0 (the small form): waves 4, 8 and 12 — the fold wave's SIMD partners (wave w runs on SIMD w mod 4)
// — hold and stage nothing, so that wave 0's add chains run alone on their SIMD: 11 filler waves
template <bool S0>
constexpr int held_fillers() { return S0 ? 11 * 64 : kWideWG - kHeldFill0; }  // 704 / 896
static_assert(2 * held_fillers<false>() <= kWideChunkP, "pass A's chunk fits the wide buffers");
#ifndef ICP4R_PACKED_FILL
#define ICP4R_PACKED_FILL 0  // (experiment) the held pass B's products with packed float math
#endif
// pass B's first chunk in the small form (steps; 0: every chunk T steps).  Measured (two A/B rounds):
// C1 0.384 (0) / 0.381 (128) / 0.385 (64) / 0.388 ms (32); at 8k any ramp lost (C2 1.162 -> 1.175
// with 128, 1.197 with 32), so the 8k form keeps uniform chunks.
#ifndef ICP4R_PASSB_RAMP
#define ICP4R_PASSB_RAMP 128
#endif
static_assert(kHeldMaxN == 10 * held_fillers<false>() && kHeldSmallN == 3 * held_fillers<true>(), "held sizes");

// PCL's sequential double chain over LDS, few registers (the MSE fallback beside the held records)
__device__ __forceinline__ double fold_seq_d_lite(const double* f, int len, double acc) {
    int k = 0;
    for (; k + 8 <= len; k += 8) {
        const double2 g0 = *reinterpret_cast<const double2*>(f + k), g1 = *reinterpret_cast<const double2*>(f + k + 2);
        const double2 g2 = *reinterpret_cast<const double2*>(f + k + 4), g3 = *reinterpret_cast<const double2*>(f + k + 6);
        acc = acc + g0.x;
        acc = acc + g0.y;
        acc = acc + g1.x;
        acc = acc + g1.y;
        acc = acc + g2.x;
        acc = acc + g2.y;
        acc = acc + g3.x;
        acc = acc + g3.y;
    }
    for (; k < len; ++k) acc = acc + f[k];
    return acc;
}

template <int HOLD, bool S0>
__global__ __launch_bounds__(kWideWG) void fold_update_held_kernel(PairArgs a, WorkArgs w) {
    constexpr int kHeldFillers = held_fillers<S0>();
    constexpr int kPassBRamp = S0 ? ICP4R_PASSB_RAMP : 0;
    constexpr int kHeldCH = 2 * kHeldFillers;  // pass A chunk: two slots of every filler
    __shared__ WideShared sh;
    const int p = xcd_remap(blockIdx.x, gridDim.x);
    if (w.ticks != nullptr && p == 0 && threadIdx.x == 0) w.ticks[9] = __builtin_amdgcn_s_memrealtime();
    PairState& st = w.state[p];
    if (st.phase != kPhaseActive) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int n = a.src_n[p];
    const int64_t xs = w.x_stride;
    const KParams& kp = a.kp;
    const float4* C = w.corr ? w.corr + (int64_t)p * xs * 2 : nullptr;
    const float4* Xp = w.X + (int64_t)p * xs;
    const float4* NT = w.nn_t ? w.nn_t + (int64_t)p * xs : nullptr;
    const bool ticks = w.ticks != nullptr && p == 0 && tid == 0;
    // key mode (w.fold_keys): X and the merged keys' targets; the records are written for pass B's
    // global path (corr_kernel's work, as in the wide kernel)
    const bool keys = w.fold_keys && C;
    const NNKey* K = keys ? w.nn_key + (int64_t)p * xs : nullptr;
    const float4* TG = keys ? a.tgt + a.tgt_off[p] : nullptr;
    const bool weighted = kp.huber_delta < INFINITY;
    const bool mse = kp.need_mse != 0;
    const float ident = weighted ? 0.0f : -0.0f;
    const int nch = (n + kHeldCH - 1) / kHeldCH;
    // filler slot column: waves 2..15 (S0: but 4, 8, 12 — the idle waves, `idle`)
    const bool idle = S0 && wv >= 2 && (wv & 3) == 0;
    const int f = S0 ? (wv - 2 - (wv >> 2)) * 64 + lane : tid - kHeldFill0;

    // the records (fillers only: loaded inside pass A's filler branch, so that they are never live in
    // the fold wave's branch — a load ahead of the role branches had kept them live there)
    float sx[HOLD], sy[HOLD], sz[HOLD], dx[HOLD], dy[HOLD], dz[HOLD];
    // pass B's layout (fold_pass_b<PAR>: S panels of kc, rows of T steps strided stride) and each held
    // record's place in it, packed: offset << 4 | chunk + 1 (0: none)
    constexpr int CAP = 9 * kWideRow;
    auto layout = [&](int cnt_, int& kc, int& S, int& stride, int& T, int& nchb) __attribute__((always_inline)) {
        kc = sigma_kc(cnt_, kp.sigma_max_kc);
        S = (cnt_ > 0 && kc > 0) ? (cnt_ + kc - 1) / kc : 1;
        stride = (((CAP / max(9 * S, 18)) - 4) & ~7) + 4;
        T = stride - 4;
        // chunks of a ramp: kPassBRamp steps first, doubling up to T (the first chunk's fill is on the
        // critical path; the later fills overlap the folds before them).  More panels than one group
        // (rows too short, down to T = 0 for hundreds of panels) take pass B's global path: 15 chunks
        // stands for "not held" there, and no loop runs on such a layout.
        nchb = 15;
        if (S <= kSliceGroup && T >= 8) {
            nchb = 0;
            for (int b = 0, len = kPassBRamp > 0 ? min(T, kPassBRamp) : T; b < kc; b += len, len = min(T, 2 * len)) ++nchb;
        }
    };
    int pk[HOLD];
    auto held_offsets = [&](int cnt_) __attribute__((always_inline)) {
        int kc, S, stride, T, nchb;
        layout(cnt_, kc, S, stride, T, nchb);
        if (nchb > 14) return;  // (pass B's global path: no offsets needed, and no loop on T = 0)
        // (the panel by a float reciprocal, corrected: exact for these small operands; the chunk by
        // walking the ramp)
        const float invkc = 1.0f / (float)kc;
#pragma unroll
        for (int k = 0; k < HOLD; ++k) {
            const int i = f + k * kHeldFillers;
            int q = (int)((float)i * invkc);
            int t = i - q * kc;
            if (t >= kc) { ++q; t -= kc; }
            if (t < 0) { --q; t += kc; }
            int c = 0, len = kPassBRamp > 0 ? min(T, kPassBRamp) : T;
            while (t >= len) {
                t -= len;
                len = min(T, 2 * len);
                ++c;
            }
            pk[k] = i < n ? ((q * 9 * stride + t) << 4) | (c + 1) : 0;
        }
    };
    clear_need(w, p, n, tid, kWideWG);
    if (ticks) w.ticks[0] = __builtin_amdgcn_s_memrealtime();

    // ---- pass A (fold_pass_a's chains over chunks of kHeldCH points)
    int cnt = 0;
    // slots 2c, 2c + 1 of this filler -> chunk c (first staging, key mode: and corr_kernel's record pair
    // {s.xyz, w}, {d.xyz, d²} for pass B's global path — per chunk, so that chunk 0 waits for its own
    // slots' gathers only)
    auto store_a = [&](int c, bool first) __attribute__((always_inline)) {
        float(*b)[kWideRow] = sh.buf[c & 1];
#pragma unroll
        for (int k = 0; k < HOLD; ++k) {
            if ((k >> 1) != c) continue;
            const int i = k * kHeldFillers + f;
            if (i >= n) continue;
            const int o = i - c * kHeldCH;
            const float d2 = l2_simple(sx[k], sy[k], sz[k], dx[k], dy[k], dz[k]);
            const float sv[6] = {sx[k], sy[k], sz[k], dx[k], dy[k], dz[k]};
            if (keys && first) {
                const float w0 = weighted ? (float)huber_w(d2, kp.huber_delta) : 1.0f;
                w.corr[(int64_t)p * xs * 2 + 2 * i] = make_float4(sx[k], sy[k], sz[k], w0);
                w.corr[(int64_t)p * xs * 2 + 2 * i + 1] = make_float4(dx[k], dy[k], dz[k], d2);
            }
            float v[6], wt = 0.0f, dd = 0.0f;
#pragma unroll
            for (int q = 0; q < 6; ++q) v[q] = ident;
            if (!(d2 > kp.max_d2)) {
                wt = weighted ? (float)huber_w(d2, kp.huber_delta) : 1.0f;
#pragma unroll
                for (int q = 0; q < 6; ++q) v[q] = weighted ? wt * sv[q] : sv[q];
                dd = d2;
                ++cnt;
            }
#pragma unroll
            for (int q = 0; q < 6; ++q) b[q][o] = v[q];
            b[6][o] = wt;
            reinterpret_cast<double*>(b[7])[o] = (double)dd;
        }
    };
    float acc = (lane < 6) ? ident : 0.0f;
    double dacc = 0.0;
    if (wv == 0) {
        fold_prio(true);
        for (int c = 0; c < nch; ++c) {
            __syncthreads();
            if (ticks && c < 6) w.ticks[20 + c] = __builtin_amdgcn_s_memrealtime();
            if (lane < 7) acc = fold_seq<float>(sh.buf[c & 1][lane], min(kHeldCH, n - c * kHeldCH), acc);
        }
        fold_prio(false);
        if (ticks) w.ticks[26] = __builtin_amdgcn_s_memrealtime();
    } else if (wv == 1) {
        if (mse) {  // the MSE sum's exact form (fold_pass_a), the whole wave per chunk
            uint64_t xsum = 0;
            int xe = INT_MAX;
            for (int c = 0; c < nch; ++c) {
                __syncthreads();
                const double* dv = reinterpret_cast<const double*>(sh.buf[c & 1][7]);
                const int len = min(kHeldCH, n - c * kHeldCH);
                for (int o = lane; o < len; o += 64) lane_exact_add(dv[o], xsum, xe);
            }
            wave_exact_total(xsum, xe);
            dacc = xsum >= kExactSat ? -1.0 : (xe == INT_MAX ? 0.0 : ldexp((double)xsum, xe));
        } else {
            for (int c = 0; c < nch; ++c) __syncthreads();
        }
    } else if (idle) {
        for (int c = 0; c < nch; ++c) __syncthreads();
    } else {
        // the held records, every load in flight together (16-B loads: with the two modes' loads
        // merged, a pointer that lost its alignment was split into four dword loads — 2.4 us more)
        // (chunk 0's two slots first, staged, then the other slots' loads, which land during chunk 0's
        // fold: issued all together, every wave's later slots queued ahead of the other waves' first
        // ones and chunk 0 waited for nearly all of them — the fold started 3.6 us in at 8k)
        auto load = [&](int k0, int k1) __attribute__((always_inline)) {
            if (keys) {
                uint32_t ti[HOLD];
#pragma unroll
                for (int k = 0; k < HOLD; ++k) {
                    if (k < k0 || k >= k1) continue;
                    const int i = min(f + k * kHeldFillers, n - 1);
                    const float4 x = Xp[i];
                    sx[k] = x.x;
                    sy[k] = x.y;
                    sz[k] = x.z;
                    ti[k] = (uint32_t)key_idx(K[i]);
                }
#pragma unroll
                for (int k = 0; k < HOLD; ++k) {
                    if (k < k0 || k >= k1) continue;
                    const float4 t = TG[ti[k]];
                    dx[k] = t.x;
                    dy[k] = t.y;
                    dz[k] = t.z;
                }
            } else {
#pragma unroll
                for (int k = 0; k < HOLD; ++k) {
                    if (k < k0 || k >= k1) continue;
                    const int i = min(f + k * kHeldFillers, n - 1);
                    const float4* q0 = static_cast<const float4*>(__builtin_assume_aligned(C ? C + 2 * i : Xp + i, 16));
                    const float4* q1 = static_cast<const float4*>(__builtin_assume_aligned(C ? C + 2 * i + 1 : NT + i, 16));
                    const float4 r0 = *q0, r1 = *q1;
                    sx[k] = r0.x;
                    sy[k] = r0.y;
                    sz[k] = r0.z;
                    dx[k] = r1.x;
                    dy[k] = r1.y;
                    dz[k] = r1.z;
                }
            }
        };
        load(0, 2);
        store_a(0, true);
        for (int c = 0; c < nch; ++c) {
            __syncthreads();
            if (c == 0) load(2, HOLD);  // (after the barrier: the fold of chunk 0 starts meanwhile)
            if (c + 1 < nch) store_a(c + 1, true);
        }
        // pass B's chunk offsets for the plain case (every correspondence kept: kc = sigma_kc(n)),
        // while the fold wave finishes (14 filler waves on 4 SIMDs: ~1.3 us of VALU at 8k if left to
        // pass B's critical path)
        held_offsets(n);
    }
    // |C|: exact integer reduction of the fillers' counts (DPP: wave 0 runs it after its chain)
    cnt = wave_sumi(cnt);
    if (lane == 0) sh.cnt[wave] = cnt;
    if (wave == 0 && lane < 7) sh.res[lane] = acc;
    if (wave == 1 && lane == 0) sh.s.mse_sum = dacc;
    __syncthreads();
    if (tid == 0) {
        int total = 0;
        for (int k = 0; k < kWideWG / 64; ++k) total += sh.cnt[k];
        sh.s.mom[0] = (double)total;
        const float one_over_n = 1.0f / sh.res[6];
        sh.s.one_over_n = one_over_n;
        for (int k = 0; k < 6; ++k) sh.s.mean[k] = sh.res[k] * one_over_n;
        // pass B's layout, once (its integer divisions in every lane of 16 waves had cost ~1 us of
        // VALU on pass B's critical path)
        layout(total, sh.lay[0], sh.lay[1], sh.lay[2], sh.lay[3], sh.lay[4]);
    }
    __syncthreads();
    if (mse && sh.s.mse_sum < 0.0) {  // (uniform) PCL's sequential double chain over the chunks again
        dacc = 0.0;
        if (wv == 0 || idle) {
            for (int c = 0; c < nch; ++c) __syncthreads();
        } else if (wv == 1) {
            for (int c = 0; c < nch; ++c) {
                __syncthreads();
                if (lane == 0)
                    dacc = fold_seq_d_lite(reinterpret_cast<const double*>(sh.buf[c & 1][7]), min(kHeldCH, n - c * kHeldCH),
                                           dacc);
            }
        } else {
            store_a(0, false);
            for (int c = 0; c < nch; ++c) {
                __syncthreads();
                if (c + 1 < nch) store_a(c + 1, false);
            }
        }
        __syncthreads();
        if (wave == 1 && lane == 0) sh.s.mse_sum = dacc;
        __syncthreads();
    }
    if (ticks) w.ticks[1] = __builtin_amdgcn_s_memrealtime();

    // ---- pass B
    SolveShared& s = sh.s;
    const int cntC = (int)s.mom[0];
    const int kc = sh.lay[0], S = sh.lay[1], stride = sh.lay[2], T = sh.lay[3], nchb = sh.lay[4];
    const int G = S, R = 9 * G, FW = (R + 63) / 64;
    if (weighted || cntC < n || S <= 1 || S > kSliceGroup || nchb > 14) {
        const FoldIn fin{C, Xp, NT, n};
        fold_pass_b<kWideWG, kWideChunkP, kWideRow, true>(kp, fin, sh.buf, s);
    } else {
        // every correspondence kept, unweighted: panel sl = [sl kc, min((sl + 1) kc, n)), one group of
        // S panels (fold_pass_b<PAR>'s layout: row (panel, ab) of T steps, rows strided = 4 mod 8)
        const float ms[3] = {s.mean[0], s.mean[1], s.mean[2]};
        const float md[3] = {s.mean[3], s.mean[4], s.mean[5]};
        const float oon = s.one_over_n;
        auto bufs = [&](int k) -> float* { return &sh.buf[k & 1][0][0]; };
        float sig = 0.0f, pacc = 0.0f;
        if (wv < 2) {
            const int L = tid;
            const int my_sl = L / 9;
            const int my_len = (wv < FW && L < R) ? min(kc, n - my_sl * kc) : 0;
            for (int c = 0, cb = 0, cl = kPassBRamp > 0 ? min(T, kPassBRamp) : T; c < nchb; ++c, cb += cl, cl = min(T, 2 * cl)) {
                __syncthreads();
                if (ticks && c < 2) w.ticks[28 + c] = __builtin_amdgcn_s_memrealtime();
                const int len = min(cl, my_len - cb);
                if (wv < FW && L < R && len > 0) pacc = fold_row(bufs(c) + L * stride, len, pacc);
            }
            if (ticks) w.ticks[30] = __builtin_amdgcn_s_memrealtime();
        } else if (idle) {
            for (int c = 0; c < nchb; ++c) __syncthreads();
        } else {
            // each held record's LDS offset in its chunk's buffer and the chunk (-1: none), by a
            // float reciprocal of kc, corrected
            // (pk: from pass A — cntC == n here, the layout it assumed)
            auto fill = [&](int c) __attribute__((always_inline)) {
                float* b = bufs(c);
#pragma unroll
                for (int k = 0; k < HOLD; ++k) {
                    if ((pk[k] & 15) != c + 1) continue;
                    const int off = pk[k] >> 4;
#if ICP4R_PACKED_FILL
                    // packed (v_pk_add / v_pk_mul: two IEEE float operations per instruction, the same
                    // roundings — contraction is off): the fill is VALU work of 14 waves on 4 SIMDs
                    typedef float f2 __attribute__((ext_vector_type(2)));
                    const f2 s01 = f2{sx[k], sy[k]} - f2{ms[0], ms[1]};
                    const f2 d01 = f2{dx[k], dy[k]} - f2{md[0], md[1]};
                    const float s2 = sz[k] - ms[2], d2 = dz[k] - md[2];
                    const float dvs[3] = {d01.x, d01.y, d2};
                    float* o = b + off;
#pragma unroll
                    for (int ra = 0; ra < 3; ++ra) {
                        const f2 pr = f2{dvs[ra], dvs[ra]} * s01;
                        o[(ra * 3 + 0) * stride] = pr.x;
                        o[(ra * 3 + 1) * stride] = pr.y;
                        o[(ra * 3 + 2) * stride] = dvs[ra] * s2;
                    }
#else
                    const float sv[3] = {sx[k] - ms[0], sy[k] - ms[1], sz[k] - ms[2]};
                    const float dv[3] = {dx[k] - md[0], dy[k] - md[1], dz[k] - md[2]};
                    float* o = b + off;
#pragma unroll
                    for (int ra = 0; ra < 3; ++ra)
#pragma unroll
                        for (int rb = 0; rb < 3; ++rb) o[(ra * 3 + rb) * stride] = dv[ra] * sv[rb];
#endif
                }
            };
            fill(0);
            if (w.ticks != nullptr && p == 0 && lane == 0) w.ticks[32 + wave - 2] = __builtin_amdgcn_s_memrealtime();
            for (int c = 0; c < nchb; ++c) {
                __syncthreads();
                if (c + 1 < nchb) fill(c + 1);
            }
        }
        __syncthreads();  // every chunk folded: the buffer of chunk nchb (unused) takes the chains
        float* cs = bufs(nchb);
        if (wv < FW && tid < R) cs[tid] = pacc;
        __syncthreads();
        if (wave == 0 && lane < 9)
            for (int sl = 0; sl < G; ++sl) sig = sig + oon * cs[sl * 9 + lane];  // res += alpha * C0
        if (wave == 0 && lane < 9) s.sigmaf[lane] = sig;
        __syncthreads();
    }
    if (ticks) w.ticks[2] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) solve_pair_body<kNumericsPCL>(sh.s, st, kp);  // (inline: no call's register saves)
    __syncthreads();
    if (ticks) w.ticks[3] = __builtin_amdgcn_s_memrealtime();
    if (sh.s.flag == 1) return;  // error: PCL breaks before transforming
    if (!w.defer_xform) transform_pair<kWideWG>(w, p, n, sh.s.T_inc, w.seed_next && w.corr);
    if (ticks) w.ticks[4] = __builtin_amdgcn_s_memrealtime();
}

// ---------------------------------------------------------------------------------------------
// update_kernel (F64 numerics): one workgroup per active pair: correspondences -> double moments
// (fixed-order block reduction) -> solve -> convergence -> X := T_inc * X.
constexpr int kUpdWG = 512;
constexpr int kUpdWaves = kUpdWG / 64;

__global__ __launch_bounds__(kUpdWG) void update_f64_kernel(PairArgs a, WorkArgs w) {
    constexpr int NM = MomLayout<kNumericsF64>::N;
    constexpr int I_CNT = MomLayout<kNumericsF64>::CNT;
    __shared__ SolveShared sh;
    __shared__ double red[kUpdWaves * NM];
    const int p = xcd_remap(blockIdx.x, gridDim.x);
    PairState& st = w.state[p];
    if (st.phase != kPhaseActive) return;
    const int tid = threadIdx.x;
    const int n = a.src_n[p];
    clear_need(w, p, n, tid, kUpdWG);
    const float4* tgt = a.tgt + a.tgt_off[p];
    float4* X = w.X + (int64_t)p * w.x_stride;
    const int64_t slot0 = (int64_t)p * w.x_stride;
    const KParams& kp = a.kp;
    const bool weighted = kp.huber_delta < INFINITY;
    double mom[NM];
#pragma unroll
    for (int k = 0; k < NM; ++k) mom[k] = 0.0;
    for (int i = tid; i < n; i += kUpdWG) {
        float d2;
        int j;
        load_nn(w, slot0 + i, d2, j);
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
    block_sum<NM, kUpdWaves>(mom, red, sh.mom);
    if (tid == 0) solve_pair<kNumericsF64>(sh, st, kp);
    __syncthreads();
    if (sh.flag == 1) return;
    if (!w.defer_xform) transform_pair<kUpdWG>(w, p, n, sh.T_inc, false);
}

// ---------------------------------------------------------------------------------------------
// fitness_prep_kernel: X := final * input (Registration::getFitnessScore / align's output).
// test (cached-neighbour plan): the fitness pass' cached-neighbour test runs here too, by the pair's
// workgroup (pair_cache_test), instead of as nn_cache_test_kernel after it — one read of X, U, nn_t
// and the input per point, no launch of its own.
constexpr int kPrepWG = 256;
constexpr int kPrepRecs = 1024;  // the fitness test's LDS miss records (the fitness pass misses ~1 %)
__global__ __launch_bounds__(kPrepWG) void fitness_prep_kernel(PairArgs a, WorkArgs w, int test) {
    const int p = xcd_remap(blockIdx.x, gridDim.x);
    const PairState& st = w.state[p];
    if (st.phase == kPhaseInvalid) return;
    __shared__ float Tf[16];
    __shared__ uint32_t need[kNeedWords];
    __shared__ int32_t pre[kNeedWords];
    __shared__ float4 lv[kPrepRecs];
    __shared__ uint2 lm[kPrepRecs];
    __shared__ int32_t mcount, wcnt[kPrepWG / 64];
    const int n = a.src_n[p];
    if (threadIdx.x < 16) Tf[threadIdx.x] = st.final_T[threadIdx.x];
    if (test && w.nn_u) {
        for (int k = threadIdx.x; k < (n + 31) >> 5; k += kPrepWG) need[k] = 0u;
        if (threadIdx.x == 0) mcount = 0;
        __syncthreads();
        float T[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) T[q] = Tf[q];
        pair_cache_test<kPrepWG, 4, true>(a, w, p, n, T, need, pre, lv, lm, kPrepRecs, &mcount, wcnt, true);
        return;
    }
    __syncthreads();
    const float4* src = a.src + a.src_off[p];
    float4* X = w.X + (int64_t)p * w.x_stride;
    float* uu = w.nn_u ? w.nn_u + (int64_t)p * w.x_stride : nullptr;
    // (w.seed_next: the fitness pass's seed keys too — see transform_pair)
    const bool seed = w.seed_next && w.corr && a.kp.compute_fitness;
    NNKey* key = w.nn_key + (int64_t)p * w.x_stride;
    const float4* C = w.corr ? w.corr + (int64_t)p * w.x_stride * 2 : nullptr;
    for (int i = threadIdx.x; i < n; i += kPrepWG) {
        const float4 s = src[i];
        float4 o = s;
        xform_pt(Tf, s.x, s.y, s.z, o.x, o.y, o.z);
        if (seed) {
            const float4 t = C[2 * i + 1];
            key[i] = make_key(l2_simple(o.x, o.y, o.z, t.x, t.y, t.z), (uint32_t)key_idx(key[i]));
        }
        if (uu) {  // X still holds the last NN pass's points (a deferred transform never ran), .w = L
            const float4 old = X[i];
            const float2 Lm = move_lu(make_float2(old.w, uu[i]), old.x, old.y, old.z, o.x, o.y, o.z);
            o.w = Lm.x;
            uu[i] = Lm.y;
        }
        X[i] = o;
    }
}

// finish_kernel: fitness = mean of d² over d² <= max_range (double), results, aligned output.
constexpr int kFinWG = 256;
__global__ __launch_bounds__(kFinWG) void finish_kernel(PairArgs a, WorkArgs w) {
    const int p = xcd_remap(blockIdx.x, gridDim.x);
    const PairState& st = w.state[p];
    const int n = a.src_n[p];
    const int64_t slot0 = (int64_t)p * w.x_stride;
    const bool have = st.phase != kPhaseInvalid && a.kp.compute_fitness && n > 0;
    // Registration::getFitnessScore: sequential double sum over points with d² <= max_range, in
    // index order, by wave 0 lane 0 over LDS chunks that waves 1..3 stage (double buffer); points
    // beyond max_range contribute +0 (a no-op on the non-negative running sum); the count is an
    // exact integer reduction.  Bit-identical to the reference loop.
    __shared__ double chunk[2][kFoldChunkP];  // (doubles: the fold lane only adds, fold_seq_d)
    __shared__ int32_t fcnt_w[kFinWG / 64];
    __shared__ uint64_t fsum_w[kFinWG / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double fsum = 0.0;
    int fcnt = 0;
    // Exact parallel form of the same sum.  Every term is a float widened to double, so every term is
    // an integer multiple of 2^e, e = the lowest set bit's exponent over the nonzero terms.  When the
    // exact total S is below 2^(e + 53), every partial sum of the non-negative terms is a multiple of
    // 2^e below 2^(e + 53), i.e. a double: the sequential loop never rounds and returns S itself.  S is
    // then an integer sum in units of 2^e (associative), saturated at 2^53; otherwise (a span of more
    // than 53 bits between the smallest term's last bit and the total) the sequential fold below runs.
    // Batches of at least kFinExactMaxPairs pairs keep the sequential fold only: their chains overlap
    // across the pairs, and the exact attempt measured slower there (C3: 43 -> 63 us per batch; a
    // pair whose span test fails pays both forms).
    constexpr int kFinExactMaxPairs = 256;
    bool exact = false;
    if (have && (int)gridDim.x < kFinExactMaxPairs) {
        constexpr uint64_t kSat = 1ull << 53;
        // the values: in registers for clouds of at most kFinWG * kFinPer points (every load in flight
        // at once, one read of the keys), else re-read per pass; NaN = no point (never in range)
        constexpr int kFinPer = 32;
        const bool reg = n <= kFinWG * kFinPer;
        float v[kFinPer];
        if (reg) {
#pragma unroll
            for (int k = 0; k < kFinPer; ++k) {
                const int i = threadIdx.x + k * kFinWG;
                v[k] = i < n ? key_d2(w.nn_key[slot0 + i]) : __int_as_float(0x7fc00000);
            }
        }
        auto each = [&](auto&& f) {
            if (reg) {
#pragma unroll
                for (int k = 0; k < kFinPer; ++k) f(v[k]);
            } else {
                for (int i = threadIdx.x; i < n; i += kFinWG) f(key_d2(w.nn_key[slot0 + i]));
            }
        };
        int emin = INT_MAX;
        each([&](float d2) {
            const double x = (double)d2;
            if (x <= a.kp.fit_max_range) {
                ++fcnt;
                if (x > 0.0) {
                    const uint64_t b = (uint64_t)__double_as_longlong(x);
                    const int ex = (int)((b >> 52) & 0x7ff);
                    const uint64_t mant = (b & ((1ull << 52) - 1)) | (1ull << 52);
                    emin = min(emin, ex - 1075 + (int)__builtin_ctzll(mant));
                }
            }
        });
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            emin = min(emin, __shfl_xor(emin, off, 64));
            fcnt += __shfl_xor(fcnt, off, 64);
        }
        if (lane == 0) {
            fcnt_w[wave] = fcnt;
            fsum_w[wave] = (uint64_t)(uint32_t)emin;
        }
        __syncthreads();
        fcnt = 0;
        emin = INT_MAX;
        for (int k = 0; k < kFinWG / 64; ++k) {
            fcnt += fcnt_w[k];
            emin = min(emin, (int)(uint32_t)fsum_w[k]);
        }
        __syncthreads();  // (fsum_w reused below)
        uint64_t S = 0;
        if (emin != INT_MAX) {
            each([&](float d2) {
                const double x = (double)d2;
                if (x <= a.kp.fit_max_range && x > 0.0) {
                    const uint64_t b = (uint64_t)__double_as_longlong(x);
                    const int ex = (int)((b >> 52) & 0x7ff);
                    const uint64_t mant = (b & ((1ull << 52) - 1)) | (1ull << 52);
                    // x = mant * 2^(ex - 1075); below 2^(emin + 53) iff ex - 1023 - emin <= 52, and then
                    // x / 2^emin = mant >> (emin + 1075 - ex), a shift by at most ctz(mant): exact
                    const uint64_t t = (ex - 1023 - emin <= 52) ? (mant >> (emin + 1075 - ex)) : kSat;
                    S = (S + t < kSat) ? S + t : kSat;
                }
            });
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) S = min(S + __shfl_xor(S, off, 64), kSat);
            if (lane == 0) fsum_w[wave] = S;
            __syncthreads();
            S = 0;
            for (int k = 0; k < kFinWG / 64; ++k) S = min(S + fsum_w[k], kSat);
        }
        if (S < kSat) {
            exact = true;
            fsum = emin == INT_MAX ? 0.0 : ldexp((double)S, emin);
        }
    }
    if (have && !exact) {
        fcnt = 0;
        __syncthreads();  // (fcnt_w reused)
        const int nch = (n + kFoldChunkP - 1) / kFoldChunkP;
        auto fill = [&](int c) {
            const int base = c * kFoldChunkP, len = min(kFoldChunkP, n - base);
            for (int o = threadIdx.x - 64; o < len; o += kFinWG - 64) {
                const float d2 = key_d2(w.nn_key[slot0 + base + o]);  // (d² only: see WorkArgs::nn_key)
                const bool in = (double)d2 <= a.kp.fit_max_range;
                chunk[c & 1][o] = in ? (double)d2 : 0.0;
                fcnt += in ? 1 : 0;
            }
        };
        if (wave >= 1) fill(0);
        for (int c = 0; c < nch; ++c) {
            __syncthreads();
            if (wave == 0) {
                if (lane == 0) fsum = fold_seq_d(chunk[c & 1], min(kFoldChunkP, n - c * kFoldChunkP), fsum);
            } else if (c + 1 < nch) {
                fill(c + 1);
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) fcnt += __shfl_xor(fcnt, off, 64);
        if (lane == 0) fcnt_w[wave] = fcnt;
        __syncthreads();
        fcnt = 0;
        for (int k = 0; k < kFinWG / 64; ++k) fcnt += fcnt_w[k];
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
// solo_kernel: one pair's whole registration by one 1024-thread workgroup — the unbatched plan for
// targets of at most kLdsTargets points (C1, C2: the node's per-frame call,
// iterative_closest_point.cpp:510-521), after init_kernel and index_kernel.  The pair's targets and
// boxes are staged into LDS once, and every ICP iteration runs inside the launch, separated by
// workgroup barriers only:
//   test    the cached-neighbour test of every source in sorted-position order (the deferred
//           transformCloud(T_inc), the bounds moved, hit or miss), the misses' search records
//           compacted in that order into the pair's query list — first pass: every source;
//   search  lds_runs<true> over the list (the batched search's run machinery and arithmetic);
//   update  fold passes A and B over (X, nn_t) in index order, the Umeyama solve, hasConverged;
// then the fitness pass (final * input, the test, the misses searched with keys, the sequential
// double sum of Registration::getFitnessScore) and the result row.  Per iteration this removes the
// launches, their boundaries and the target staging of the multi-launch plan; every result is
// bit-identical to it (the same per-query and per-chain arithmetic in the same order).
constexpr int kSoloWG = kLdsWG;
constexpr int kSoloFitChunk = 960;  // fitness chunk: 15 waves fill, wave 0 lane 0 folds
constexpr int kSoloGrp = 4;         // the first pass' sorted positions in flight per thread
// LDS.  (compile-time) ICP4R_SOLO_RESIDENT=1: the pair's target tile stays resident for the whole registration,
// and the search's per-wave state, the update's fold buffers (192-point chunks), the test's bitmap
// and records and the fitness chunks take turns in the 18 KB beside it.  0: the tile and the
// update's 512-point fold buffers (fold_update_kernel's) take turns in one region, the tile
// restaged from the L2 for each search.
#ifndef ICP4R_SOLO_RESIDENT
#define ICP4R_SOLO_RESIDENT 1
#endif
constexpr bool kSoloResident = ICP4R_SOLO_RESIDENT != 0;
struct SoloTile {
    v4f tl[kLdsTargets];
    alignas(16) float bx[kLdsTargets / kLdsLeaf][6];
    float sbx[kLdsTargets / kLdsLeaf / kSuper][6];
};
struct SoloSearch {  // the search's per-wave state
    unsigned long long best[kLdsWaves][64];
    uint32_t sec[kLdsWaves][64];
    uint16_t items[kLdsWaves][kRing + 64];
};
constexpr int kSoloChunk = kSoloResident ? 192 : kFoldChunkP;  // fold chunk (points)
constexpr int kSoloRow = kSoloChunk + kFoldPad;
struct SoloFold {  // the update
    alignas(16) float buf[2][9][kSoloRow];
    float res[8];
    int32_t cnt[kLdsWaves];
    SolveShared sv;
};
// the test's LDS miss records (24 B each), after the bitmap and its prefixes, in the region they share
constexpr int kSoloRecs = ((int)(kSoloResident ? sizeof(SoloSearch) : sizeof(SoloTile)) - 8 * kNeedWords) / 24 & ~15;
struct SoloTest {  // the cached-neighbour test: the miss bitmap, its word prefixes, the miss records
    uint32_t need[kNeedWords];
    int32_t pre[kNeedWords];
    float4 lv[kSoloRecs];
    uint2 lm[kSoloRecs];
};
#if ICP4R_SOLO_RESIDENT
struct SoloShared {
    SoloTile t;
    union {
        SoloSearch s;
        SoloFold f;
        SoloTest c;
        alignas(16) double fit[2][kSoloFitChunk];  // the fitness sum's chunks (doubles: fold_seq_d)
    } u;
    int32_t wtot[kLdsWaves];  // per-wave counts (the test's misses, the fitness count)
    int32_t mcount;           // the test's LDS record count
};
#define SOLO_T(sh) (sh).t
#define SOLO_S(sh) (sh).u.s
#else
struct SoloShared {
    union {
        SoloTile t;
        SoloFold f;
        SoloTest c;
        alignas(16) double fit[2][kSoloFitChunk];
    } u;
    SoloSearch s;
    int32_t wtot[kLdsWaves];
    int32_t mcount;
};
#define SOLO_T(sh) (sh).u.t
#define SOLO_S(sh) (sh).s
#endif
#define SOLO_F(sh) (sh).u.f
#define SOLO_C(sh) (sh).u.c
#define SOLO_FIT(sh) (sh).u.fit
static_assert(sizeof(SoloShared) <= 160 * 1024, "solo LDS");

// The first pass' query list of the solo plan: every source in sorted-position order (thread t takes
// positions [t * per, (t + 1) * per), kSoloGrp at a time with every load in flight): qv = {X_i as
// init_kernel wrote it, U = +inf}, qm = {source index | sorted position << 14, the target at the same
// relative sorted position — the seed}.  Returns n.
__device__ int solo_first_list(const PairArgs& a, const WorkArgs& w, int p, int n, int m) {
    const int tid = threadIdx.x;
    const int64_t xs0 = (int64_t)p * w.x_stride;
    const float4* X = w.X + xs0;
    const int32_t* sperm = w.sperm + xs0;
    float4* qv = w.qv + xs0;
    uint2* qm = w.qm + xs0;
    const int per = (n + kSoloWG - 1) / kSoloWG;
    const int k0 = min(tid * per, n), k1 = min(k0 + per, n);
    for (int g = k0; g < k1; g += kSoloGrp) {
        int ii[kSoloGrp];
        float4 v[kSoloGrp];
#pragma unroll
        for (int e = 0; e < kSoloGrp; ++e) ii[e] = sperm[min(g + e, k1 - 1)];
#pragma unroll
        for (int e = 0; e < kSoloGrp; ++e) v[e] = X[ii[e]];
#pragma unroll
        for (int e = 0; e < kSoloGrp; ++e) {
            const int k = g + e;
            if (k >= k1) break;
            qv[k] = make_float4(v[e].x, v[e].y, v[e].z, INFINITY);
            qm[k] = make_uint2((uint32_t)ii[e] | ((uint32_t)k << kNtPosShift), (uint32_t)(((int64_t)k * m) / n));
        }
    }
    return n;
}

// The cached-neighbour test of an iteration pass (FROM_SRC = false: X := T_inc X, deferred) or of
// the fitness pass (FROM_SRC: T = final applied to the input): pair_cache_test by the whole
// workgroup, its records in the tile's LDS region; when they overflow it (a pair far from
// converged), the records left in sq / sm are placed at their ranks here.  Returns the list length.
template <bool FROM_SRC>
__device__ int solo_cache_test(const PairArgs& a, const WorkArgs& w, int p, int n, const float (&T)[16],
                               SoloShared& sh, unsigned long long* tk = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nwords = (n + 31) >> 5;
    const uint64_t t0 = tk ? __builtin_amdgcn_s_memrealtime() : 0;
    for (int k = tid; k < nwords; k += kSoloWG) SOLO_C(sh).need[k] = 0u;
    if (tid == 0) sh.mcount = 0;
    __syncthreads();
    const int tot = pair_cache_test<kSoloWG, 2, FROM_SRC>(a, w, p, n, T, SOLO_C(sh).need, SOLO_C(sh).pre, SOLO_C(sh).lv,
                                                         SOLO_C(sh).lm, kSoloRecs, &sh.mcount, sh.wtot, FROM_SRC);
    if (tk) {  // debug: the test's own wall, and how many passes overflowed the LDS records
        tk[27] += __builtin_amdgcn_s_memrealtime() - t0;
        tk[28] += tot > kSoloRecs ? 1 : 0;
        tk[29] += tot;
    }
    if (tot <= kSoloRecs) return tot;
    // overflow: every record is in sq / sm (test order), the bitmap still in LDS — word prefixes
    // (wave 0), then each record to its rank
    __syncthreads();
    if (wave == 0) {
        constexpr int kW = kNeedWords / 64;
        int c[kW], sum = 0;
#pragma unroll
        for (int j = 0; j < kW; ++j) {
            const int wd = lane * kW + j;
            c[j] = wd < nwords ? __builtin_popcount(SOLO_C(sh).need[wd]) : 0;
            sum += c[j];
        }
        int incl = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_up(incl, off, 64);
            if (lane >= off) incl += o;
        }
        int run = incl - sum;
#pragma unroll
        for (int j = 0; j < kW; ++j) {
            SOLO_C(sh).pre[lane * kW + j] = run;
            run += c[j];
        }
    }
    __syncthreads();
    const int64_t xs0 = (int64_t)p * w.x_stride;
    for (int k = tid; k < tot; k += kSoloWG) {
        const float4 r = w.sq[xs0 + k];
        const uint2 m = w.sm[xs0 + k];
        const uint32_t sp = min(m.y, (uint32_t)(n - 1));
        const int rk = SOLO_C(sh).pre[sp >> 5] + __builtin_popcount(SOLO_C(sh).need[sp >> 5] & ((1u << (sp & 31)) - 1u));
        w.qv[xs0 + rk] = r;
        w.qm[xs0 + rk] = make_uint2((m.x & kNtIdxMask) | (sp << kNtPosShift), m.x >> kNtPosShift);
    }
    return tot;
}

__global__ __launch_bounds__(kSoloWG) void solo_kernel(PairArgs a, WorkArgs w, int iters) {
    __shared__ SoloShared sh;
    const int p = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    PairState& st = w.state[p];
    const KParams& kp = a.kp;
    const int n = uload(a.src_n + p), m = uload(a.tgt_n + p);
    const int64_t xs0 = (int64_t)p * w.x_stride;
    const bool valid = uload(&st.phase) != kPhaseInvalid;
    const int nsb = (((m + kLdsLeaf - 1) / kLdsLeaf) + kSuper - 1) / kSuper;
    const LdsTile tile{SOLO_T(sh).tl, SOLO_T(sh).bx, SOLO_T(sh).sbx};
    RunStats rs;
    auto search = [&](int nlist, bool keys) {
        __syncthreads();  // the list (global, this workgroup's) and the region's previous use
        v4f isl, ish;
        if (kSoloResident) {
            const v4f* sbg = reinterpret_cast<const v4f*>(w.sbox + (int64_t)p * 2 * w.sb_stride);
            const int sbl = min(lane, nsb - 1);
            isl = sbg[2 * sbl];
            ish = sbg[2 * sbl + 1];
        } else {
            stage_tile<kSoloWG>(tile, w, p, nsb, isl, ish);
            __syncthreads();
        }
        lds_runs<true>(tile, SOLO_S(sh).best[wave], SOLO_S(sh).sec[wave], SOLO_S(sh).items[wave], w.qv + xs0, w.qm + xs0, nlist, m, nsb,
                       isl, ish, a, w, p, xs0, w.X + xs0, w.nn_key + xs0, keys, false, rs);
        __syncthreads();
    };
    // debug (plan option phase_ticks = 1): pair 0's phase walls summed over the registration (s_memrealtime,
    // 100 MHz) into ticks[0..9]: staging, test, search, pass A, pass B, solve, fitness test, fitness
    // search, fitness sum, iterations (tools/experiments/solo_phases.py)
    unsigned long long* tk = (w.ticks && p == 0 && tid == 0) ? reinterpret_cast<unsigned long long*>(w.ticks) : nullptr;
    uint64_t tk_last = tk ? __builtin_amdgcn_s_memrealtime() : 0;
    auto tick = [&](int slot) {
        if (!tk) return;
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        tk[slot] += now - tk_last;
        tk_last = now;
    };
    if (valid) {
        if (kSoloResident) {
            v4f isl, ish;
            stage_tile<kSoloWG>(tile, w, p, nsb, isl, ish);  // (the search reloads its boxes)
        }
        float T[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) T[q] = 0.0f;
        int flag = 0;
        __syncthreads();
        tick(0);
        for (int it = 0; it < iters && flag == 0; ++it) {
            // (first pass: src_order_kernel wrote the records, seeded at the source's kd leaf in the
            // target's tree, when the sources are ordered by it — plan option src_order = 1)
            const int nlist = it > 0 ? solo_cache_test<false>(a, w, p, n, T, sh, tk)
                              : (w.stage_first && src_by_tgt_tree(a, w, p)) ? n : solo_first_list(a, w, p, n, m);
            tick(1);
            search(nlist, false);
            tick(2);
            const FoldIn fin{nullptr, w.X + xs0, w.nn_t + xs0, n};
            fold_pass_a<kSoloWG, kSoloChunk, kSoloRow>(kp, fin, SOLO_F(sh).buf, SOLO_F(sh).res, SOLO_F(sh).cnt, SOLO_F(sh).sv);
            tick(3);
            fold_pass_b<kSoloWG, kSoloChunk, kSoloRow, false>(kp, fin, SOLO_F(sh).buf, SOLO_F(sh).sv);
            tick(4);
            if (tid == 0) solve_pair<kNumericsPCL>(SOLO_F(sh).sv, st, kp);
            __syncthreads();
            tick(5);
            if (tk) tk[9] += 1;
            flag = SOLO_F(sh).sv.flag;
#pragma unroll
            for (int q = 0; q < 16; ++q) T[q] = SOLO_F(sh).sv.T_inc[q];  // the next pass's deferred transform
        }
        // the fitness pass (getFitnessScore after align) and align's output: final * input
        if (kp.compute_fitness || a.aligned) {
            __syncthreads();  // thread 0's final_T
#pragma unroll
            for (int q = 0; q < 16; ++q) T[q] = st.final_T[q];
            if (kp.compute_fitness) {
                const int nlist = solo_cache_test<true>(a, w, p, n, T, sh);
                tick(6);
                search(nlist, true);
                tick(7);
                if (a.aligned) {  // X = final * input (the test wrote it, the search rewrote its misses)
                    __syncthreads();
                    const float4* src = a.src + a.src_off[p];
                    const float4* X = w.X + xs0;
                    for (int i = tid; i < n; i += kSoloWG) {
                        float4 v = X[i];
                        v.w = src[i].w;  // intensity copied through
                        a.aligned[a.src_off[p] + i] = v;
                    }
                }
            } else {
                const float4* src = a.src + a.src_off[p];
                for (int i = tid; i < n; i += kSoloWG) {
                    const float4 s = src[i];
                    float4 o = s;
                    xform_pt(T, s.x, s.y, s.z, o.x, o.y, o.z);
                    a.aligned[a.src_off[p] + i] = o;  // (.w: the input's intensity)
                }
            }
        }
    }
    // Registration::getFitnessScore: the sequential double sum over points with d² <= max_range in
    // index order (wave 0 lane 0 over LDS chunks the other waves fill; points beyond contribute +0)
    // and the exact count (finish_kernel's fold, bit for bit)
    const bool have = valid && kp.compute_fitness && n > 0;
    double fsum = 0.0;
    int fcnt = 0;
    if (have) {
        const NNKey* key = w.nn_key + xs0;
        const int nch = (n + kSoloFitChunk - 1) / kSoloFitChunk;
        auto fill = [&](int c) {
            const int base = c * kSoloFitChunk, len = min(kSoloFitChunk, n - base);
            for (int o = tid - 64; o < len; o += kSoloWG - 64) {
                const float d2 = key_d2(key[base + o]);
                const bool in = (double)d2 <= kp.fit_max_range;
                SOLO_FIT(sh)[c & 1][o] = in ? (double)d2 : 0.0;
                fcnt += in ? 1 : 0;
            }
        };
        if (wave >= 1) fill(0);
        for (int c = 0; c < nch; ++c) {
            __syncthreads();
            if (wave == 0) {
                if (lane == 0) fsum = fold_seq_d(SOLO_FIT(sh)[c & 1], min(kSoloFitChunk, n - c * kSoloFitChunk), fsum);
            } else if (c + 1 < nch) {
                fill(c + 1);
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) fcnt += __shfl_xor(fcnt, off, 64);
        if (lane == 0) sh.wtot[wave] = fcnt;
        __syncthreads();
        fcnt = 0;
        for (int k = 0; k < kLdsWaves; ++k) fcnt += sh.wtot[k];
    }
    tick(8);
    if (tid == 0) {
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
    if (lane == 0) {
        count_add(w.evals, 0, rs.evals);
        count_add(w.evals, 1, rs.tests);
    }
}

// Test hook: the device float Umeyama rotation for k sigma matrices (one thread each).
__global__ void rot_f32_kernel(const float* sigma, float* R, int k) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= k) return;
    float sg[9], Ri[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) sg[e] = sigma[9 * i + e];
    umeyama_rotation_f32_reg(sg, Ri);
#pragma unroll
    for (int e = 0; e < 9; ++e) R[9 * i + e] = Ri[e];
}

hipError_t launch_rot_f32(const float* sigma, float* R, int k, hipStream_t st) {
    hipLaunchKernelGGL(rot_f32_kernel, dim3((k + 63) / 64), dim3(64), 0, st, sigma, R, k);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
hipError_t launch_init(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st) {
    if (npairs < 64)
        hipLaunchKernelGGL(init_kernel<1024>, dim3(npairs), dim3(1024), 0, st, a, w);
    else
        hipLaunchKernelGGL(init_kernel<256>, dim3(npairs), dim3(256), 0, st, a, w);
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

hipError_t launch_index(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st) {
    // every source by the target's tree: launch the target builds alone (a grid with idle source
    // workgroups left half the CUs without a build)
    const bool tgt_only = w.src_by_tgt && w.kdn && (w.kd_index & 1) && w.t_stride <= kKdMaxN && w.x_stride <= kKdMaxN;
    const unsigned nch = (unsigned)((w.t_stride + kKdMaxN - 1) / kKdMaxN);
    if (w.mo_hist) {  // (setup_work sets it only for plans that refine: see index_mo_hist_kernel)
        if (!(w.tbb && (w.kd_index & 1) && w.t_stride > kKdMaxN && (w.leaf == 16 || w.leaf == 32) &&
              (int64_t)w.mo_groups * kMoChunk >= w.t_stride))
            return hipErrorInvalidValue;
        hipLaunchKernelGGL(index_mo_hist_kernel, dim3(w.mo_groups, npairs), dim3(kIdxWG), 0, st, a, w);
        hipLaunchKernelGGL(index_mo_scatter_kernel, dim3(w.mo_groups, npairs), dim3(kIdxWG), 0, st, a, w);
        // (no src_order_kernel: a target past kKdMaxN has no kd tree for its source to descend)
        hipLaunchKernelGGL(index_refine_kernel, dim3(nch + 1, npairs), dim3(kIdxWG), 0, st, a, w);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(index_kernel, dim3(npairs, tgt_only ? 1 : 2), dim3(kIdxWG), 0, st, a, w);
    if (w.src_by_tgt && w.kdn && !(ICP4R_FUSE_SRC_ORDER && tgt_only))
        hipLaunchKernelGGL(src_order_kernel, dim3(npairs), dim3(kSoWG), 0, st, a, w);
    if ((w.kd_index & 1) && w.t_stride > kKdMaxN && (w.leaf == 16 || w.leaf == 32))
        hipLaunchKernelGGL(index_refine_kernel, dim3(nch, npairs), dim3(kIdxWG), 0, st, a, w);
    return hipGetLastError();
}

hipError_t launch_index_cloud(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st) {
    if (w.mo_hist || (w.src_by_tgt && w.kdn)) return hipErrorInvalidValue;  // (the target chain's forms)
    hipLaunchKernelGGL(index_cloud_kernel, dim3(npairs), dim3(kIdxWG), 0, st, a, w);
    if ((w.kd_index & 1) && w.t_stride > kKdMaxN && (w.leaf == 16 || w.leaf == 32)) {
        const unsigned nch = (unsigned)((w.t_stride + kKdMaxN - 1) / kKdMaxN);
        hipLaunchKernelGGL(index_refine_kernel, dim3(nch, npairs), dim3(kIdxWG), 0, st, a, w);
    }
    return hipGetLastError();
}

hipError_t launch_nn_lds(const PairArgs& a, const WorkArgs& w, int npairs, int max_n, int fitness_pass, int first,
                         int ncu, hipStream_t st, const NNLdsEvents& ev, int test_fused, int ordered) {
    // (query records: source index and sorted position in kNtPosShift bits each, every mode)
    if (w.leaf != kLdsLeaf || w.t_stride > kLdsTargets || npairs <= 0 || max_n > (1 << kNtPosShift))
        return hipErrorInvalidValue;
    const bool cache = w.nn_u != nullptr;
    if (cache && (max_n > kCacheMaxN || !w.sq || !w.qv || !w.need || !w.miss_cnt || !w.nn_t || !w.defer_xform))
        return hipErrorInvalidValue;
    if (!w.plist || !w.plist_n || !w.queue || !w.qv || !w.qm) return hipErrorInvalidValue;
    hipError_t e;
    if (cache && !first && !test_fused) {  // (test_fused: the previous fold_update_kernel ran it)
        const int chunks = (max_n + kTestWG * kTestPer - 1) / (kTestWG * kTestPer);
        if (ev.test_start && (e = hipEventRecord(ev.test_start, st)) != hipSuccess) return e;
        hipLaunchKernelGGL(nn_cache_test_kernel, dim3(chunks, npairs), dim3(kTestWG), 0, st, a, w, fitness_pass);
        if (ev.test_stop && (e = hipEventRecord(ev.test_stop, st)) != hipSuccess) return e;
    }
    if (ordered && (first || !cache || fitness_pass || !test_fused)) return hipErrorInvalidValue;
    if (!ordered)
        hipLaunchKernelGGL(nn_order_kernel, dim3(1), dim3(kOrderWG), 0, st, a, w, npairs, fitness_pass,
                           (first || !cache) ? 1 : 0, ncu);
    const int grid = npairs < ncu ? npairs : ncu;  // persistent: one workgroup per CU (LDS-bound)
    if (ev.search_start && (e = hipEventRecord(ev.search_start, st)) != hipSuccess) return e;
    if (cache)
        hipLaunchKernelGGL((nn_lds_kernel<true>), dim3(grid), dim3(kLdsWG), 0, st, a, w, fitness_pass, first,
                           test_fused && !first ? 1 : 0);
    else
        hipLaunchKernelGGL((nn_lds_kernel<false>), dim3(grid), dim3(kLdsWG), 0, st, a, w, fitness_pass, first, 0);
    if (ev.search_stop && (e = hipEventRecord(ev.search_stop, st)) != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t launch_nn_tile(const PairArgs& a, const WorkArgs& w, int npairs, int max_n, int max_m, int fitness_pass,
                          int first, int qrun, hipStream_t st, hipEvent_t tile_start, hipEvent_t tile_stop) {
    if (w.leaf != kLdsLeaf || !w.tsort || !w.sperm || max_m >= kTileMaxM || npairs <= 0 || max_n <= 0 ||
        (qrun != 64 && qrun != 32 && qrun != 16 && qrun != 8))
        return hipErrorInvalidValue;
    hipError_t e;
    const int qpart = kLdsWaves * qrun;  // queries per workgroup
    const dim3 grid((max_m + kLdsTargets - 1) / kLdsTargets, (max_n + qpart - 1) / qpart, npairs);
    // one tile: the search kernel seeds, stores and writes the records itself (w.tile_own = 0: the
    // three-launch form, for A/B)
    const bool own = grid.x == 1 && w.tile_own != 0;
    // (w.seed_next: the previous update / fitness_prep_kernel wrote the seeds, except for the first pass)
    if (!own && (first || !w.seed_next))
        hipLaunchKernelGGL(nn_seed_kernel, dim3((max_n + 255) / 256, npairs), dim3(256), 0, st, a, w, fitness_pass,
                           first);
    if (tile_start && (e = hipEventRecord(tile_start, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(nn_tile_kernel, grid, dim3(kLdsWG), 0, st, a, w, fitness_pass, own ? first : -1, qrun);
    if (tile_stop && (e = hipEventRecord(tile_stop, st)) != hipSuccess) return e;
    if (!own && w.corr != nullptr && !fitness_pass && !w.fold_keys)  // records from the merged keys
        hipLaunchKernelGGL(corr_kernel, dim3((max_n + 255) / 256, npairs), dim3(256), 0, st, a, w);
    return hipGetLastError();
}

hipError_t launch_nn_pruned(int q, int chunk_sb, int chunks, const PairArgs& a, const WorkArgs& w, int npairs,
                            int max_n, int fitness_pass, int first, hipStream_t st) {
    const int per_block = kNNWG * q;
    const dim3 grid((max_n + per_block - 1) / per_block, npairs, chunks), block(kNNWG);
    if (chunk_sb < 1 || chunk_sb > 64 || chunks < 1) return hipErrorInvalidValue;
    if (chunks > 1)
        hipLaunchKernelGGL(nn_seed_kernel, dim3((max_n + 255) / 256, npairs), dim3(256), 0, st, a, w, fitness_pass, first);
#define ICP4R_PR_CASE(QQ, BB) \
    hipLaunchKernelGGL((nn_pruned_kernel<QQ, BB>), grid, block, 0, st, a, w, fitness_pass, first, chunk_sb)
    if (w.leaf == 16) {
        switch (q) {
            case 1: ICP4R_PR_CASE(1, 16); break;
            case 2: ICP4R_PR_CASE(2, 16); break;
            case 4: ICP4R_PR_CASE(4, 16); break;
            default: return hipErrorInvalidValue;
        }
    } else if (w.leaf == 32) {
        switch (q) {
            case 1: ICP4R_PR_CASE(1, 32); break;
            case 2: ICP4R_PR_CASE(2, 32); break;
            case 4: ICP4R_PR_CASE(4, 32); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        return hipErrorInvalidValue;
    }
#undef ICP4R_PR_CASE
    if (chunks > 1 && w.corr != nullptr && !fitness_pass)  // records from the merged keys
        hipLaunchKernelGGL(corr_kernel, dim3((max_n + 255) / 256, npairs), dim3(256), 0, st, a, w);
    return hipGetLastError();
}

hipError_t launch_update(const PairArgs& a, const WorkArgs& w, int npairs, int max_n, bool need_corr, hipStream_t st,
                         int tail_test, int order_ncu, bool wide) {
    if (order_ncu > 0 && (!tail_test || !w.owork || !w.plist || !w.plist_n || !w.nn_u || a.kp.numerics != kNumericsPCL))
        return hipErrorInvalidValue;
    if (a.kp.numerics == kNumericsPCL) {
        if (need_corr)
            hipLaunchKernelGGL(corr_kernel, dim3((max_n + 255) / 256, npairs), dim3(256), 0, st, a, w);
        if (wide && !tail_test && order_ncu <= 0 && w.held_update && max_n <= kHeldSmallN)
            hipLaunchKernelGGL((fold_update_held_kernel<3, true>), dim3(npairs), dim3(kWideWG), 0, st, a, w);
        else if (wide && !tail_test && order_ncu <= 0 && w.held_update && max_n <= kHeldMaxN)
            hipLaunchKernelGGL((fold_update_held_kernel<10, false>), dim3(npairs), dim3(kWideWG), 0, st, a, w);
        else if (wide && !tail_test && order_ncu <= 0)
            hipLaunchKernelGGL(fold_update_wide_kernel, dim3(npairs), dim3(kWideWG), 0, st, a, w);
        else if (w.res_update && !need_corr && !w.corr && max_n <= kResMaxN && w.nn_t && w.nn_u && w.defer_xform &&
                 a.kp.huber_delta == INFINITY && a.kp.max_d2 >= FLT_MAX &&
                 !w.sums_tail && (!tail_test || (w.sq && w.sm && w.need && w.miss_cnt)))
            hipLaunchKernelGGL(fold_update_res_kernel, dim3(npairs), dim3(kResWG), 0, st, a, w, tail_test, order_ncu);
        else
            hipLaunchKernelGGL(fold_update_kernel, dim3(npairs), dim3(kFoldWG),
                               ICP4R_UPD_OCC >= 4 ? 0 : (ICP4R_UPD_OCC == 3 ? 12000 : 20000), st, a, w, tail_test,
                               order_ncu);
    } else {
        hipLaunchKernelGGL(update_f64_kernel, dim3(npairs), dim3(kUpdWG), 0, st, a, w);
    }
    return hipGetLastError();
}

hipError_t launch_solo(const PairArgs& a, const WorkArgs& w, int npairs, int max_n, int iters, hipStream_t st) {
    if (a.kp.numerics != kNumericsPCL || w.leaf != kLdsLeaf || w.t_stride > kLdsTargets || max_n > kCacheMaxN ||
        w.x_stride > kCacheMaxN || !w.tsort || !w.tbox || !w.sbox || !w.sperm || !w.nn_u || !w.nn_t || !w.qv ||
        !w.qm || !w.sq || !w.sm || !w.need || !w.miss_cnt || npairs <= 0 || iters <= 0)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(solo_kernel, dim3(npairs), dim3(kSoloWG), 0, st, a, w, iters);
    return hipGetLastError();
}

hipError_t launch_fitness_prep(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st, int test) {
    if (test && (!w.nn_u || !w.need || !w.miss_cnt || !w.nn_t || !w.sq || !w.tsort || w.x_stride > kCacheMaxN))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(fitness_prep_kernel, dim3(npairs), dim3(kPrepWG), 0, st, a, w, test);
    return hipGetLastError();
}

hipError_t launch_finish(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st) {
    hipLaunchKernelGGL(finish_kernel, dim3(npairs), dim3(kFinWG), 0, st, a, w);
    return hipGetLastError();
}

}  // namespace icp4r
