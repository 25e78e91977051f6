// icp4r_internal.hpp — types shared by the C-ABI host code and the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "icp4r/icp4r.h"
#include "icp4r/icp4r_ego.h"
#include "icp4r/icp4r_gicp.h"
#include "icp4r_math.hpp"

namespace icp4r {

constexpr int kNNWG = 256;        // threads per NN workgroup (4 waves)
constexpr int kMaxQ = 16;         // register-resident queries per lane in nn_kernel (instantiated)
constexpr int kDefaultQ = 4;      // brute force: default cap (tools/tune_sweep.py)
constexpr int kDefaultPrunedQ = 2;  // pruned: default cap
constexpr int kDefaultLeaf = 16;    // pruned: targets per block
constexpr int kMaxGroups = 3;        // batched plans: pair groups on their own streams (run_pairs)
constexpr int kDefaultGroups = 2;
constexpr int kDefaultStageSel = 32;    // batched search: plan option stage_sel's default
constexpr int kDefaultPartSize = 2048;  // batched search: misses per work item of a heavy pair (round 6: 1024 -> 2048, C3 +0.6 %)
constexpr int kFoldChunk = 1024;  // points per LDS chunk of the sequential fitness fold
constexpr int kSuper = 8;         // target blocks per superblock (pruned NN)
constexpr int kPrunedMinM = 512;  // ICP4R_NN_AUTO prunes when the largest target has >= this many points
constexpr int kCacheMaxN = 16384; // cached-neighbour test (nn_lds_kernel<true>): max source points per pair
// Work counters: one 128-B slot per wave (mod kCountSlots).  A single counter word hit by every wave
// of a launch serialises the atomics at one L2 channel (~10 ns each: 30k waves = 0.3 ms per launch).
constexpr int kKdNodes = 2048;                 // kd tree nodes kept per target (heap ids < this)
constexpr int kKdnStride = 8 + kKdNodes;
constexpr int kCountSlots = 2048;
constexpr int kCountStride = 16;

constexpr int kNumericsPCL = ICP4R_NUMERICS_PCL;
constexpr int kNumericsF64 = ICP4R_NUMERICS_F64;
constexpr int kStatusEmpty = ICP4R_E_EMPTY;
constexpr int kStatusTooFewCorr = ICP4R_E_TOO_FEW_CORR;
constexpr int kStatusNonFinite = ICP4R_E_NONFINITE;
constexpr int kStatusInvalid = ICP4R_E_INVALID;

// per-pair loop phase
constexpr int kPhaseActive = 0;     // iterating
constexpr int kPhaseConverged = 1;  // hasConverged() fired
constexpr int kPhaseFailed = 2;     // |C| < min_correspondences (PCL: converged_ = false, break)
constexpr int kPhaseInvalid = 3;    // empty target / non-finite input: nothing computed

using Result = icp4r_result;

struct KParams {
    ConvParams conv;
    int32_t min_corr;
    int32_t numerics;
    int32_t compute_fitness;
    float max_d2;          // reject a correspondence iff d2 > max_d2 (float image of max_dist^2)
    double huber_delta;    // +inf: unweighted (PCL)
    double fit_max_range;  // getFitnessScore(max_range): keep d2 <= max_range
    int32_t need_mse;      // 0 when no MSE criterion can fire (both thresholds <= 0): the MSE only
                           // feeds those two '<' tests, so its sequential sum is skipped
    int32_t sigma_max_kc;  // Eigen's largest GEMM panel depth for sigma (sigma_max_kc(); INT32_MAX:
                           // no panels) — the panel depth of |C| correspondences is sigma_kc()
};

struct PairArgs {
    const float4* src;
    const float4* tgt;
    const int64_t* src_off;
    const int32_t* src_n;
    const int64_t* tgt_off;
    const int32_t* tgt_n;
    const float* guess;  // npairs*16 column-major or nullptr
    float4* aligned;     // optional
    Result* results;
    KParams kp;
};

// Device-resident per-pair loop state (ICP members of PCL: transformation_, final_transformation_,
// nr_iterations_, converged_, and DefaultConvergenceCriteria's prev MSE / similar counter).
struct PairState {
    float T_inc[16];
    float final_T[16];
    double prev_mse;
    int32_t similar;
    int32_t conv_state;
    int32_t iterations;
    int32_t phase;
    int32_t status;
    int32_t ncorr;
    // Σs of the next update's pass A (Eigen's rowwise().sum() of the moved source, in index order),
    // folded by the previous update's fused tail over the X it wrote (fold_update_kernel: eligible
    // registrations only — every correspondence kept, unweighted, no MSE criterion); sums_ok = 1 while
    // they are valid for the next pass A, which then reads nn_t only
    float sum_s[3];
    int32_t sums_ok;
};

// NN result of one query: (float bits of d² << 32) | target index.  d² >= 0, so the unsigned order
// of the keys is the lexicographic (d², index) order; the minimum key is PCL's answer (nearest
// target, lowest index among equal distances) whatever order the targets are visited in.
using NNKey = uint64_t;
__host__ __device__ inline float key_d2(NNKey k) {
    union {
        uint32_t u;
        float f;
    } c;
    c.u = (uint32_t)(k >> 32);
    return c.f;
}
__host__ __device__ inline int32_t key_idx(NNKey k) { return (int32_t)(uint32_t)k; }

// Workspace, pair p at [p * stride, ...) of each array.
struct WorkArgs {
    float4* X;          // input_transformed [npairs * x_stride]
    NNKey* nn_key;      // per-query NN key   [npairs * x_stride]; splits > 1 merge by atomicMin.  After
                        // a fused fitness pass (pair_cache_test, fitness) a HIT's index bits hold its NN's
                        // SORTED target position, not the original index: only key_d2 is meaningful
                        // there (finish_kernel reads d² only; nothing may read key_idx after that pass)
    PairState* state;   // [npairs]
    int64_t x_stride;   // >= max source points per pair
    int32_t splits;     // brute force: target splits per pair (1 for batches; >1 for single-pair latency)
    int32_t leaf;       // pruned: targets per block (16 or 32); 0 = brute force
    int32_t kd_index;   // clouds of <= 8192 points get the balanced kd order (index_kernel), else Morton;
                        // bit 0: targets, bit 1: sources
    int32_t src_by_tgt; // 1: a source whose target gets the kd order is ordered by descending the target's
                        // kd tree (src_order_kernel) instead of by its own tree: queries sorted by the
                        // target leaf they fall in, and that leaf seeds their first search
    int32_t stage_first;  // 1 (batched plan): src_order_kernel writes the first pass' query records
    int32_t seed_next;    // 1 (multi-tile plan, PCL numerics): the update's transform and fitness_prep_kernel
                          // write the next NN pass's seed keys (the previous NN at the moved point) from the
                          // correspondence records, so no nn_seed_kernel launch
                          // (qv / qm, sorted order) itself; 0: the first pass' nn_key seeds
    float* tbb;         // [npairs * 8] the target's bounding box (lo xyz, hi xyz), from init_kernel's
                        // validation pass (the Morton index skips its own pass over the cloud); or nullptr
    uint16_t* mo_hist;  // [npairs * mo_groups * 2^14] per-workgroup Morton cell counts (u16) of a large target
                        // (multi-workgroup sort, index_mo_hist_kernel); nullptr: one workgroup per target
    int32_t mo_groups;  // workgroups per target of that sort (>= t_stride / 8192)
    int32_t* mo_rep;    // [npairs * 2^14] per Morton cell: the original index of one of its targets, -1: empty
                        // (written by that sort; nn_seed_kernel's first-pass seed: a target in the query's cell)
    uint32_t* kdn;      // [npairs * kKdnStride] the target kd tree: [0, 6) quantisation lo / scale bits,
                        // [8 + node] internal node (heap order) = 1 << 31 | mid << 13 | axis << 11 | key
    // Pruned-search index, built once per registration by index_kernel (SURVEY.md §8f "sorted map"):
    float4* tsort;      // [npairs * t_stride] targets in index order (kd / Morton), .w = original index bits;
                        // positions [m, t_stride): +inf coordinates (never a match)
    int32_t* tinv;      // [npairs * t_stride] original target index -> sorted position
    float4* tbox;       // [npairs * 2 * b_stride] per block: lo, hi (empty blocks: +inf, -inf)
    float4* sbox;       // [npairs * 2 * sb_stride] per superblock of kSuper blocks: lo, hi
    int32_t* sperm;     // [npairs * x_stride] source indices in index order (kd / Morton)
    int64_t t_stride, b_stride, sb_stride;
    float4* corr;       // PCL numerics: [npairs * x_stride * 2] per source point {s.xyz, w}, {d.xyz, d²}
    // Cached-neighbour test (nn_lds_kernel<true>; nullptr = off):
    // L_i (X_i.w): a lower bound on |X_i - t_k| for every target k other than the NN; U_i (nn_u[i]):
    // an upper bound of the second-nearest distance.  Set by a search, widened by every kernel that
    // moves X_i.
    float* nn_u;        // [npairs * x_stride] U_i
    int32_t tile_own;     // 1 (one-tile plan): nn_tile_kernel seeds, searches and writes the records itself
                          // (plan option tile_own = 0: the three-launch form, for A/B)
    int32_t defer_xform;  // 1: the update leaves X_i := T_inc X_i to the next pass's test kernel
    int32_t sums_tail;    // 1: the fused tail also folds the next pass A's Σs (eligible pairs: PairState)
    int32_t fold_keys;    // 1 (multi-tile single pairs, wide update): no corr_kernel after the search — the
                          // update's pass A forms the correspondence records from X and the merged keys'
                          // targets and writes them for pass B
    int32_t res_update;   // 1 (batched plan, sources <= kResMaxN): fold_update_res_kernel, the pair held on
                          // chip across the update (plan option res_update = 0: fold_update_kernel)
    int32_t held_update;  // 1 (wide update, sources <= kHeldMaxN): fold_update_held_kernel, the records held
                          // in the fillers' registers from pass A to pass B (plan option held_update)
    int32_t fit_xform;    // 1 (one-tile plan, no cache, no seeds): the fitness pass' nn_tile_kernel forms
                          // X := final * input itself (fitness_prep_kernel's work; plan option fit_xform)
    float4* nn_t;       // [npairs * x_stride] the NN target of X_i: xyz, .w = its sorted target position |
                        // the query's sorted position << 14 (nt_pack)
    float4* sq;         // [npairs * x_stride] the pass's miss list in the order the test found them: a
                        // missed query's {X.xyz, U} (the test appends, the search stages by rank) ...
    uint2* sm;          // ... {its source index | its NN's sorted target position << 14, its sorted position}
    float4* qv;         // [npairs * x_stride] a search item's queries in list order {x, y, z, U} ...
    uint2* qm;          // ... {source index | sorted position << 14, seed's sorted target position}
    uint32_t* need;     // [npairs * need_stride] per pair: bit s = the query at Morton position s missed
    int64_t need_stride;
    int32_t* miss_cnt;  // [npairs] misses of the current pass (cleared by the update); | kMissUnranked when
                        // the fused test left them unplaced (sq / sm + bitmap) for the search to place
    // Batched search (nn_lds_kernel): the pass's pair work list, heaviest first, and its queue
    int32_t* plist;     // [npairs * ceil(x_stride / 64)] items (pair << 10 | part)
    int32_t* plist_n;   // [4]: items, (queue), the pass's part size (nn_order_kernel)
    int32_t* queue;     // [1] next work-list index (reset by nn_order_kernel)
    int32_t* owork;     // [npairs] the next pass' work per pair, published by fold_update_kernel when it
                        // builds the work list itself (plist_n[3]: its arrival counter)
    int32_t part_size;  // nn_lds_kernel: misses per work item of a heavy pair (0: one item per pair);
                        // plist holds items (pair << 10 | part)
    int32_t stage_sel;  // nn_lds_kernel: a ranked item of at most this many misses stages only the
                        // superblocks its queries can reach (stage_tile_sel; plan option stage_sel, 0: off)
    unsigned long long* evals;  // [kCountSlots][kCountStride]: per slot distance evaluations, box tests,
                                // cached-neighbour hits (count_add; the host sums the slots)
    uint64_t* ticks;    // debug (plan option phase_ticks = 1): s_memrealtime (100 MHz) at fold_update phase
                        // boundaries of pair 0 — start, pass A, pass B, solve, transform
    uint64_t* pass_ticks;  // debug (plan option phase_ticks = 1): this NN pass' own slots [kPassTickSlots] of the
                           // batched search's event counts / clocks (tools/experiments/nn_events.py), or nullptr
};
constexpr int kPassTickSlots = 16;  // per NN pass: 11 event counters / clocks + 4 per-item walls
constexpr int kMaxTickPasses = 64;  // passes with their own slots (later passes: none)
// first per-pass slot of a batch of npairs (after the pair-0 stamps and the per-pair debug slots)
inline int64_t pass_tick_base(int npairs) { return 32 + 20 * (int64_t)npairs; }

hipError_t launch_init(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st);
hipError_t launch_nn(int q, bool packed, const PairArgs& a, const WorkArgs& w, int npairs, int max_n,
                     int fitness_pass, hipStream_t st);
hipError_t launch_index(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st);
// one cloud's index alone (as pair p's target; w's index buffers), no source column or order
hipError_t launch_index_cloud(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st);
// chunk_sb: superblocks per target chunk (<= 64); chunks: grid.z (1: one wave searches every superblock)
hipError_t launch_nn_pruned(int q, int chunk_sb, int chunks, const PairArgs& a, const WorkArgs& w, int npairs,
                            int max_n, int fitness_pass, int first, hipStream_t st);
// the pruned plan's LDS-tiled search: nn_seed_kernel, nn_tile_kernel (target tiles x query parts),
// corr_kernel (records, when the update reads them)
hipError_t launch_nn_tile(const PairArgs& a, const WorkArgs& w, int npairs, int max_n, int max_m, int fitness_pass,
                          int first, int qrun, hipStream_t st, hipEvent_t tile_start = nullptr, hipEvent_t tile_stop = nullptr);
// events recorded around the batched NN's stages (any may be null)
struct NNLdsEvents {
    hipEvent_t test_start = nullptr, test_stop = nullptr, search_start = nullptr, search_stop = nullptr;
};
// ordered: the previous fold_update_kernel built the work list (no nn_order_kernel launch)
hipError_t launch_nn_lds(const PairArgs& a, const WorkArgs& w, int npairs, int max_n, int fitness_pass, int first,
                         int ncu, hipStream_t st, const NNLdsEvents& ev, int test_fused = 0, int ordered = 0);
constexpr int kLdsMaxTargets = 8192;  // nn_lds_kernel: whole target set in LDS
constexpr int kLdsMinPairs = 256;     // ... used for batches of at least this many pairs
constexpr int kLdsMaxSources = 1 << 14;  // ... with at most this many sources (14-bit index / position fields)
constexpr int kResMaxN = 8192;            // fold_update_res_kernel: sources of at most this many points
constexpr int kDefaultResUpdate = 0;      // ... plan option res_update's default
constexpr int kHeldMaxN = 10 * 896;       // fold_update_held_kernel: sources of at most this many points
constexpr int kHeldSmallN = 3 * 704;      // ... its 3-record form (the 2k scans; 11 filler waves) up to this many
constexpr int kDefaultHeldUpdate = 1;     // ... plan option held_update's default
constexpr int kSoloMaxN = 1024;           // solo_kernel by default for single pairs of at most this many sources
// wide: one 1024-thread workgroup per pair (fold_update_wide_kernel) — plans with at most one pair
// per CU and neither the fused test nor the fused work list
hipError_t launch_update(const PairArgs& a, const WorkArgs& w, int npairs, int max_n, bool need_corr,
                         hipStream_t st, int tail_test = 0,
                         int order_ncu = 0,  // > 0: the launch also builds the next pass's work list
                         bool wide = false);
// solo_kernel: every iteration and the fitness pass of each pair in one workgroup (PCL numerics,
// targets <= kLdsMaxTargets, sources <= kCacheMaxN; after launch_init and launch_index)
hipError_t launch_solo(const PairArgs& a, const WorkArgs& w, int npairs, int max_n, int iters, hipStream_t st);
hipError_t launch_fitness_prep(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st, int test = 0);
hipError_t launch_finish(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st);
hipError_t launch_rot_f32(const float* sigma, float* R, int k, hipStream_t st);

// ---- scan-to-map store (icp4r_map.hip)
struct SectorArgs {
    float cx, cy, cz;  // query point (the vehicle position p_now)
    float radius;      // RADAR_RADIUS
    float heading;     // degrees (float, as Sector_Search receives it)
};
struct Mat3x4d {
    double R[9];  // row-major
    double t[3];
};
hipError_t launch_associate(const float4* in, int64_t n, const Mat3x4d& M, float4* out, hipStream_t st);
int64_t sector_blocks(int64_t n);
hipError_t launch_sector(const float4* map, int64_t n, const SectorArgs& a, int32_t* counts, int32_t* offsets,
                         int32_t* total, float4* out, hipStream_t st);

// ---- radar ego velocity (icp4r_ego.hip)
struct EgoArgs {
    const float* rec;      // device records, 5 floats each
    const int64_t* off;    // [nscans] first record of scan s
    const int32_t* cnt;    // [nscans]
    int64_t stride;        // workspace points per scan (>= max cnt)
    float4* feat;          // [nscans * stride] distance, arfa, beta, v_r
    double4* pd;           // [nscans * stride] cos(DEG2RAD(beta)) v_r, cos / sin / DEG2RAD of arfa
    int32_t* scores;       // [nscans * max_h] inlier counts
    int32_t max_h;         // hypotheses of the largest scan
    int32_t iterations;    // icp4r_ego_params.iterations (<= 0: (int)(0.2 n) per scan)
    double sigma, dyn;
    uint64_t seed;
    uint8_t* mask;         // optional: static flag per record
    icp4r_ego_result* results;
};
hipError_t launch_ego(const EgoArgs& e, int nscans, int max_n, float4* xyzi, hipStream_t st);
hipError_t launch_ego_features(const EgoArgs& e, int nscans, int max_n, float4* xyzi, hipStream_t st);

// ---- generalized ICP (icp4r_gicp.hip): fast_gicp's LsqRegistration state per pair
struct GicpState {
    double R[9], t[3];  // x0 (row-major rotation, translation)
    double lambda;      // lm_lambda_ (< 0: not yet initialised)
};
// One iteration runs as three kernels over slices of each pair's source points (gicp_slices(n), a
// function of n only, so a pair's sums do not depend on the batch around it): the linearisation (its
// last slice solves the first kGicpSpec Levenberg-Marquardt trials), the trials' errors (its last
// slice decides), and the move of X.
constexpr int kGicpSys = 21 + 6 + 1 + 1;  // H (upper triangle), g, y, |valid|
constexpr int kGicpSpec = 2;             // LM trials evaluated per pass (the rest, rarely needed, one by one)
constexpr int kGicpMaxSlices = 64;
constexpr int kGicpGrid = 2048;
constexpr int kGicpKnnWaves = 16384;     // k-NN covariance walk: lanes per query up to 8 while the
                                         // grid stays within this many waves (0 lanes: this rule)          // workgroups per iteration kernel, about (a pair: at most its slices)
struct GicpTrial {
    double R[9], t[3];    // the trial transform delta * x0
    double dR[9], dt[3];  // delta
    double d[6];          // the LDLT step
    double lambda;
};
struct GicpCand {  // written by the linearisation's last slice, read by the trial kernel
    GicpTrial c[kGicpSpec];
    double lambda0;        // the iteration's first damping (lm_init * max|diag H| on the first iteration)
    double sys[kGicpSys];  // H, g, y0, |valid| at x0
    double R0[9], t0[3];   // x0
};
struct GicpArgs {
    GicpState* gs;        // [npairs]
    GicpCand* cand;       // [npairs]
    double* part_lin;     // [npairs][kGicpMaxSlices][kGicpSys] per-slice linearisation sums
    double* part_err;     // [npairs][kGicpMaxSlices][kGicpSpec] per-slice trial errors
    int32_t* cnt;         // [npairs] slices arrived (zero between launches)
    const double* cov_src;  // [npairs * x_stride * 6] regularised source covariances (upper triangle)
    const double* cov_tgt;  // [npairs * t_stride * 6]
    double* mah;          // [npairs * x_stride * 6] Mahalanobis of the current correspondences
    int64_t t_stride;
    double max_d2;        // corr_dist_threshold_² (float) as double
    double rot_eps, trans_eps, lm_init;
    int32_t lm_max_iterations, max_iterations;
    int32_t spec;         // LM trials evaluated speculatively, 0..kGicpSpec (plan option gicp_spec)
    int32_t grid;         // workgroups per iteration kernel, about (plan option gicp_grid)
};
hipError_t launch_gicp_init(const float* guess, GicpState* gs, int npairs, hipStream_t st);
hipError_t launch_gicp_cov(const float4* cloud, const int64_t* off, const int32_t* cnt, int npairs, int max_n,
                           int64_t stride, int k, int reg, double* cov, int lanes, hipStream_t st);
// k-NN covariances over a Morton index of the cloud itself (w.tsort / tbox / sbox, leaf 16)
hipError_t launch_gicp_knn_cov(const float4* cloud, const int64_t* off, const int32_t* cnt, const WorkArgs& w,
                               int npairs, int max_n, int64_t stride, int k, int reg, double* cov, int lanes,
                               hipStream_t st);
// the number of pairs still iterating into *out and, if host_out, into pinned host memory
// host_out (pinned): (seq << 32) | the active count, one 64-bit store — a check's value is told apart from a
// stale one of an earlier call still in flight by its sequence number
hipError_t launch_gicp_active(const PairState* st, int npairs, int32_t* out, int64_t* host_out, uint32_t seq,
                              hipStream_t s);
hipError_t launch_gicp_iter(const PairArgs& a, const WorkArgs& w, const GicpArgs& g, int npairs, int max_n, int it,
                            hipStream_t st);

}  // namespace icp4r
