// icp4r_capi.cpp — the C ABI (include/icp4r/icp4r.h) over the HIP kernels.
//
// Host-side mirror of the PCL boundary the reference calls (src/iterative_closest_point.cpp:510-521):
// a context owns one device's stream and grow-only device buffers; every entry validates its
// arguments, launches, and reports a status plus a thread-local message (icp4r_last_error).  There
// is no CPU fallback: if the device path cannot run, the call fails with ICP4R_E_HIP.
#include <dlfcn.h>
#include <float.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <utility>
#include <vector>

#include "icp4r/icp4r.h"
#include "icp4r_batch.hpp"
#include "icp4r_host.hpp"
#include "icp4r_internal.hpp"

using namespace icp4r;

namespace icp4r_host {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

int check_cloud(const float* c, int64_t n, int32_t stride, const char* what) {
    if (n < 0) return fail(ICP4R_E_INVALID, "%s: negative point count", what);
    if (n > 0 && !c) return fail(ICP4R_E_INVALID, "%s: NULL cloud with %lld points", what, (long long)n);
    if (stride < 12 || stride % 4) return fail(ICP4R_E_INVALID, "%s: stride %d bytes (need >= 12, multiple of 4)", what, stride);
    return ICP4R_OK;
}

void pack_host(const float* c, int64_t n, int32_t stride_bytes, std::vector<float>& out) {
    out.resize((size_t)(n > 0 ? n : 1) * 4);
    const unsigned char* b = reinterpret_cast<const unsigned char*>(c);
    for (int64_t i = 0; i < n; ++i) {
        const float* p = reinterpret_cast<const float*>(b + (size_t)i * stride_bytes);
        out[4 * (size_t)i + 0] = p[0];
        out[4 * (size_t)i + 1] = p[1];
        out[4 * (size_t)i + 2] = p[2];
        out[4 * (size_t)i + 3] = stride_bytes >= 16 ? p[3] : 0.0f;
    }
}

const RoctxApi& roctx() {
    static const RoctxApi api = [] {
        RoctxApi a;
        void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
        if (!h) h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            a.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
            a.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
            if (!a.push || !a.pop) a.push = nullptr, a.pop = nullptr;
        }
        return a;
    }();
    return api;
}

}  // namespace icp4r_host

using icp4r_host::DevBuf;
using icp4r_host::EventPair;
using icp4r_host::check_cloud;
using icp4r_host::fail;
using icp4r_host::pack_host;

// Batch-pipeline helpers shared with the other entry points (icp4r_gicp.cpp): icp4r_batch.hpp.
namespace icp4r_pipe {

constexpr size_t kCountBytes = (size_t)kCountSlots * kCountStride * sizeof(uint64_t);

// Sum the per-slot work counters (evaluations, box tests, cache hits) since the last reset.
constexpr int kNumCounters = 8;
int read_counters(icp4r_ctx* ctx, uint64_t (&out)[kNumCounters]) {
    for (int k = 0; k < kNumCounters; ++k) out[k] = 0;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipDeviceSynchronize());
    if (!ctx->evals.p) return ICP4R_OK;
    std::vector<uint64_t> v((size_t)kCountSlots * kCountStride);
    HIP_TRY(hipMemcpy(v.data(), ctx->evals.p, kCountBytes, hipMemcpyDeviceToHost));
    for (int s = 0; s < kCountSlots; ++s)
        for (int k = 0; k < kNumCounters; ++k) out[k] += v[(size_t)s * kCountStride + k];
    return ICP4R_OK;
}

const char* const kPlanOptNames[kNumPlanOpts] = {
    "nn_q", "leaf", "chunk_sb", "nn_lds", "nn_cache", "nn_tile", "tile_run", "solo", "xpad",
    "phase_ticks", "kd", "morton_mwg", "part", "src_order", "fuse_seed", "tile_own", "tile_defer",
    "groups", "search_cu_div", "fuse_test", "fuse_order", "sums_tail", "wide_update", "gather_padded",
    "gicp_cov_brute", "fold_keys", "gicp_spec", "gicp_grid", "gicp_knn_lanes", "res_update",
    "held_update", "fit_xform", "counters", "stage_sel"};

int opt(const icp4r_ctx* ctx, PlanOpt k, int dflt) {
    return (ctx && (ctx->plan_set >> k & 1ull)) ? ctx->plan_val[k] : dflt;
}

// Geometry of the NN pass.
//  * pruned (ICP4R_NN_AUTO when the target has >= kPrunedMinM points, or ICP4R_NN_PRUNED): Q queries
//    per lane, 64*Q Morton-contiguous queries per wave; Q shrinks while the grid has < 8192 waves
//    (a single 8k pair runs at Q = 1: 128 waves), leaf = 16 targets per block.
//  * brute force: Q queries per lane (fewer when pairs are few, so the grid still fills 256 CUs),
//    then split the target range until there are >= 2048 workgroups (8 per CU) while each split
//    keeps >= 256 targets.  Q = 4 scalar measured fastest (tools/experiments/tune_sweep.py, profiles/tune_r01.jsonl).
// Tuning overrides (tools/experiments/tune_sweep.py): ICP4R_NN_Q caps Q, ICP4R_LEAF = 16 | 32.
Plan make_plan(const icp4r_ctx* ctx, int npairs, int max_n, int max_m, int nn_mode, bool allow_lds,
               bool registration) {
    Plan pl;
    pl.pruned = nn_mode == ICP4R_NN_PRUNED || (nn_mode == ICP4R_NN_AUTO && max_m >= kPrunedMinM);
    pl.packed = false;
    pl.lds = false;
    pl.cache = false;
    pl.splits = 1;
    pl.leaf = 0;
    pl.chunk_sb = 64;
    pl.chunks = 1;
    pl.tile = false;
    pl.tile_run = 64;
    pl.solo = false;
    pl.max_m = max_m;
    const int qcap = opt(ctx, kOptNnQ, pl.pruned ? kDefaultPrunedQ : kDefaultQ);
    pl.q = (qcap == 1 || qcap == 2 || qcap == 4 || qcap == 8 || qcap == 16) ? qcap
                                                                             : (pl.pruned ? kDefaultPrunedQ : kDefaultQ);
    auto qblocks = [&](int q) { return (int64_t)((max_n + kNNWG * q - 1) / (kNNWG * q)); };
    if (pl.pruned) {
        if (pl.q > 4) pl.q = 4;
        const int leaf = opt(ctx, kOptLeaf, kDefaultLeaf);
        pl.leaf = (leaf == 16 || leaf == 32) ? leaf : kDefaultLeaf;
        while (pl.q > 1 && (int64_t)npairs * qblocks(pl.q) * (kNNWG / 64) < 8192) pl.q /= 2;
        pl.blocks = (int64_t)npairs * qblocks(pl.q);
        // target chunks for the streamed kernel: at most 64 superblocks each (one lane per superblock
        // of the candidate ballot); small grids (single pairs) cut the target further, down to 16
        // superblocks per chunk, until the launch has about 1024 waves (ICP4R_CHUNK_SB overrides)
        const int nsb = (((max_m + pl.leaf - 1) / pl.leaf) + kSuper - 1) / kSuper;
        const int64_t waves = pl.blocks * (kNNWG / 64);
        int cs = 64;
        while (cs > 16 && waves * ((nsb + cs - 1) / cs) < 1024) cs /= 2;
        const int cs_env = opt(ctx, kOptChunkSb, 0);
        if (cs_env == 16 || cs_env == 32 || cs_env == 64) cs = cs_env;
        pl.chunk_sb = cs;
        pl.chunks = nsb > 0 ? (nsb + cs - 1) / cs : 1;
        pl.blocks *= pl.chunks;
        // batches whose targets fit in LDS: one workgroup per pair (plan option nn_lds = 0|1 overrides).  Its
        // query records pack the source index and sorted position in 14 bits each (kLdsMaxSources),
        // so larger sources take the tiled search instead.
        const int lds = opt(ctx, kOptNnLds, -1);
        const bool fits = allow_lds && pl.leaf == 16 && max_m <= kLdsMaxTargets && max_n <= kLdsMaxSources;
        pl.lds = fits && (lds == 1 || (lds < 0 && npairs >= kLdsMinPairs));
        if (pl.lds) {
            pl.q = 2;
            pl.blocks = npairs;
            pl.chunks = 1;
            pl.cache = opt(ctx, kOptNnCache, 1) != 0;
        } else {
            // single pairs / small batches: the LDS-tiled search (target tiles of 8192 x query parts)
            pl.tile = pl.leaf == 16 && max_m < (1 << 19) && opt(ctx, kOptNnTile, 1) != 0;
            if (pl.tile) {
                pl.chunks = (max_m + 8191) / 8192;
                // queries per wave run: shorter runs (more workgroups, each staging its tile) until the
                // grid covers the CUs — a single pair's search is latency-bound per run (C2 1.85 ->
                // 1.75 ms, C5 2.35 -> 2.20 ms at 16; C1 0.457 -> 0.449 ms at 8; plan option tile_run = 64 / 32 /
                // 16 / 8 forces one)
                const int tr = opt(ctx, kOptTileRun, 0);
                auto parts = [&](int run) { return (int64_t)npairs * ((max_n + 16 * run - 1) / (16 * run)) * pl.chunks; };
                pl.tile_run = 64;
                if (tr == 64 || tr == 32 || tr == 16 || tr == 8)
                    pl.tile_run = tr;
                else
                    while (pl.tile_run > 8 && parts(pl.tile_run) < 256) pl.tile_run /= 2;
                pl.blocks = parts(pl.tile_run);
            }
            // a PCL-numerics registration whose targets fit one LDS tile: the whole registration of
            // each pair in one workgroup (solo_kernel; plan option solo = 0: the multi-launch plan)
            // (up to kSoloMaxN sources: beyond, the one CU's search of the first pass' queries and the
            // misses costs more than the multi-launch plan's boundaries since its search spreads over
            // the CUs in runs of 16 — C1's 2k pair 0.55 ms solo vs 0.50 multi at PCL's 10 iterations;
            // solo stays ahead on long fixed runs up to 3k sources, 0.78 vs 0.81 ms at 20 — see
            // tools/experiments/solo_sweep.py, profiles/round3/s4/solo_sweep_r16.jsonl; plan option solo = 1 forces it up to
            // kCacheMaxN, 0 disables it)
            const int solo_env = opt(ctx, kOptSolo, -1);
            pl.solo = registration && pl.tile && pl.chunks == 1 && solo_env != 0 &&
                      max_n <= (solo_env == 1 ? kCacheMaxN : kSoloMaxN);
            if (pl.solo) pl.blocks = npairs;
        }
        return pl;
    }
    const int64_t want = 2048;
    while (pl.q > 1 && (int64_t)npairs * qblocks(pl.q) < want) pl.q /= 2;
    while ((int64_t)npairs * qblocks(pl.q) * pl.splits < want && max_m / (pl.splits * 2) >= 256 && pl.splits < 64)
        pl.splits *= 2;
    pl.blocks = (int64_t)npairs * qblocks(pl.q) * pl.splits;
    pl.packed = nn_mode == ICP4R_NN_BRUTE_PACKED && pl.q >= 2;
    return pl;
}

float max_d2_threshold(double max_dist) {
    const double md2 = max_dist * max_dist;
    if (!(md2 < (double)FLT_MAX)) return FLT_MAX;  // also +inf / NaN: keep every finite d2
    float f = (float)md2;
    if ((double)f > md2) f = nextafterf(f, 0.0f);
    return f;
}

int make_kparams(const icp4r_params* p, KParams* kp) {
    icp4r_params d;
    if (!p) {
        icp4r_params_default(&d);
        p = &d;
    }
    if (p->max_iterations < 0) return fail(ICP4R_E_INVALID, "max_iterations must be >= 0");
    if (p->numerics != ICP4R_NUMERICS_PCL && p->numerics != ICP4R_NUMERICS_F64)
        return fail(ICP4R_E_INVALID, "unknown numerics mode %d", p->numerics);
    if (p->nn_mode != ICP4R_NN_AUTO && p->nn_mode != ICP4R_NN_BRUTE && p->nn_mode != ICP4R_NN_BRUTE_PACKED &&
        p->nn_mode != ICP4R_NN_PRUNED)
        return fail(ICP4R_E_INVALID, "unknown nn_mode %d", p->nn_mode);
    if (!(p->huber_delta > 0)) return fail(ICP4R_E_INVALID, "huber_delta must be > 0 (+inf disables)");
    memset(kp, 0, sizeof(*kp));
    kp->conv.max_iterations = p->max_iterations;
    kp->conv.max_similar = p->max_iterations_similar_transforms;
    kp->conv.rot_thr = p->transformation_rotation_epsilon > 0 ? p->transformation_rotation_epsilon
                                                              : 1.0 - p->transformation_epsilon;
    kp->conv.trans_thr = p->transformation_epsilon;
    kp->conv.abs_mse = p->mse_threshold_absolute;
    kp->conv.rel_mse = p->euclidean_fitness_epsilon;
    kp->min_corr = p->min_correspondences;
    kp->numerics = p->numerics;
    kp->compute_fitness = p->compute_fitness;
    kp->max_d2 = max_d2_threshold(p->max_correspondence_distance);
    kp->huber_delta = p->huber_delta;
    kp->fit_max_range = p->fitness_max_range;
    kp->need_mse = (p->mse_threshold_absolute > 0 || p->euclidean_fitness_epsilon > 0) ? 1 : 0;
    if (p->eigen_gebp_mr < 0 || p->eigen_gebp_mr > 64)
        return fail(ICP4R_E_INVALID, "eigen_gebp_mr %d out of range (0: the default 8)", p->eigen_gebp_mr);
    kp->sigma_max_kc = sigma_max_kc(p->eigen_l1_bytes, p->eigen_gebp_mr);
    return ICP4R_OK;
}

int next_event(std::vector<EventPair>& v, size_t& used, EventPair** out) {
    if (used == v.size()) {
        EventPair e;
        HIP_TRY(hipEventCreate(&e.start));
        HIP_TRY(hipEventCreate(&e.stop));
        v.push_back(e);
    }
    *out = &v[used++];
    return ICP4R_OK;
}

// Size the workspace for a plan and fill WorkArgs.
int setup_work(icp4r_ctx* ctx, const Plan& pl, int npairs, int max_n, int max_m, bool corr, hipStream_t st,
               WorkArgs& w) {
    const int64_t x_stride = (((max_n > 0 ? max_n : 1) + 3) & ~3) + opt(ctx, kOptXpad, 0);
    const int64_t slots = (int64_t)npairs * x_stride;
    HIP_TRY(ctx->X.ensure((size_t)slots * sizeof(float4)));
    HIP_TRY(ctx->nn_key.ensure((size_t)slots * sizeof(NNKey)));
    HIP_TRY(ctx->state.ensure((size_t)npairs * sizeof(PairState)));
    memset(&w, 0, sizeof(w));
    w.tile_own = opt(ctx, kOptTileOwn, 1) != 0 ? 1 : 0;
    w.X = static_cast<float4*>(ctx->X.p);
    w.nn_key = static_cast<NNKey*>(ctx->nn_key.p);
    w.state = static_cast<PairState*>(ctx->state.p);
    w.x_stride = x_stride;
    w.splits = pl.splits;
    if (!ctx->evals.p) {
        HIP_TRY(ctx->evals.ensure(kCountBytes));
        HIP_TRY(hipMemsetAsync(ctx->evals.p, 0, kCountBytes, st));
    }
    // the NN work counters: diagnostics, off unless asked for (plan option counters = 1, or per-kernel
    // timing on): their per-wave atomics at every search launch's end cost C1 2 %, C2 1.4 % (round 6)
    w.evals = (opt(ctx, kOptCounters, 0) != 0 || ctx->kernel_timing) ? static_cast<unsigned long long*>(ctx->evals.p)
                                                                      : nullptr;
    if (opt(ctx, kOptPhaseTicks, 0)) {
        // (see the kernels' debug tick slots; then kPassTickSlots per NN pass)
        const size_t nt = (size_t)pass_tick_base(npairs) + (size_t)kMaxTickPasses * kPassTickSlots;
        if (ctx->ticks.cap < nt * sizeof(uint64_t)) {
            HIP_TRY(ctx->ticks.ensure(nt * sizeof(uint64_t)));
            HIP_TRY(hipMemsetAsync(ctx->ticks.p, 0, nt * sizeof(uint64_t), st));
        }
        w.ticks = static_cast<uint64_t*>(ctx->ticks.p);
    }
    if (corr && !pl.cache) {  // with the cached-neighbour test the update reads X and nn_t instead
        HIP_TRY(ctx->corr.ensure((size_t)slots * 2 * sizeof(float4)));
        w.corr = static_cast<float4*>(ctx->corr.p);
    }
    if (pl.pruned) {
        const int64_t span = (int64_t)pl.leaf * kSuper;
        w.leaf = pl.leaf;
        w.kd_index = opt(ctx, kOptKd, 3);  // bit 0: targets, bit 1: sources (0: Morton for both)
        w.t_stride = ((max_m > 0 ? max_m : 1) + span - 1) / span * span;
        w.b_stride = w.t_stride / pl.leaf;
        w.sb_stride = w.b_stride / kSuper;
        HIP_TRY(ctx->tsort.ensure((size_t)npairs * w.t_stride * sizeof(float4)));
        HIP_TRY(ctx->tinv.ensure((size_t)npairs * w.t_stride * sizeof(int32_t)));
        HIP_TRY(ctx->tbox.ensure((size_t)npairs * 2 * w.b_stride * sizeof(float4)));
        HIP_TRY(ctx->sbox.ensure((size_t)npairs * 2 * w.sb_stride * sizeof(float4)));
        HIP_TRY(ctx->sperm.ensure((size_t)slots * sizeof(int32_t)));
        w.tsort = static_cast<float4*>(ctx->tsort.p);
        w.tinv = static_cast<int32_t*>(ctx->tinv.p);
        w.tbox = static_cast<float4*>(ctx->tbox.p);
        w.sbox = static_cast<float4*>(ctx->sbox.p);
        w.sperm = static_cast<int32_t*>(ctx->sperm.p);
        HIP_TRY(ctx->kdn.ensure((size_t)npairs * (kKdnStride + 8) * sizeof(uint32_t)));
        w.kdn = static_cast<uint32_t*>(ctx->kdn.p);
        w.tbb = reinterpret_cast<float*>(w.kdn + (size_t)npairs * kKdnStride);
        // a target too large for the in-LDS kd build, for few pairs: its Morton sort on several
        // workgroups (one 8192-point chunk each) before index_refine_kernel re-orders every chunk
        // (plan option morton_mwg = 0: one workgroup per target, as for the batches)
        constexpr int kChunk = 8192;
        const int64_t mog = (w.t_stride + kChunk - 1) / kChunk;
        if ((w.kd_index & 1) && w.t_stride > kChunk && (pl.leaf == 16 || pl.leaf == 32) &&
            npairs * mog <= 2048 && opt(ctx, kOptMortonMwg, 1)) {
            HIP_TRY(ctx->mo_hist.ensure((size_t)npairs * mog * (1u << 14) * sizeof(uint16_t)));
            w.mo_hist = static_cast<uint16_t*>(ctx->mo_hist.p);
            w.mo_groups = (int32_t)mog;
            HIP_TRY(ctx->mo_rep.ensure((size_t)npairs * (1u << 14) * sizeof(int32_t)));
            w.mo_rep = static_cast<int32_t*>(ctx->mo_rep.p);
        }
        if (pl.solo) {  // the query list and the cached-neighbour state (solo_kernel)
            HIP_TRY(ctx->qv.ensure((size_t)slots * sizeof(float4)));
            HIP_TRY(ctx->qm.ensure((size_t)slots * sizeof(uint2)));
            HIP_TRY(ctx->nn_lu.ensure((size_t)slots * sizeof(float)));
            HIP_TRY(ctx->nn_t.ensure((size_t)slots * sizeof(float4)));
            HIP_TRY(ctx->sq.ensure((size_t)slots * sizeof(float4)));
            HIP_TRY(ctx->sm.ensure((size_t)slots * sizeof(uint2)));
            w.qv = static_cast<float4*>(ctx->qv.p);
            w.qm = static_cast<uint2*>(ctx->qm.p);
            w.nn_u = static_cast<float*>(ctx->nn_lu.p);
            w.nn_t = static_cast<float4*>(ctx->nn_t.p);
            w.sq = static_cast<float4*>(ctx->sq.p);
            w.sm = static_cast<uint2*>(ctx->sm.p);
            // (the test's per-pair count and, for an overflowing miss list, its bitmap: written only)
            w.need_stride = (x_stride + 31) / 32;
            HIP_TRY(ctx->need.ensure((size_t)npairs * w.need_stride * sizeof(uint32_t)));
            HIP_TRY(ctx->miss_cnt.ensure((size_t)npairs * sizeof(int32_t)));
            w.need = static_cast<uint32_t*>(ctx->need.p);
            w.miss_cnt = static_cast<int32_t*>(ctx->miss_cnt.p);
            w.defer_xform = 1;
        }
        if (pl.lds) {
            HIP_TRY(ctx->plist.ensure((size_t)npairs * ((x_stride + 63) / 64) * sizeof(int32_t)));
            HIP_TRY(ctx->plist_n.ensure(4 * kMaxGroups * sizeof(int32_t)));  // per group: items, queue, part size
            w.plist = static_cast<int32_t*>(ctx->plist.p);
            HIP_TRY(ctx->qv.ensure((size_t)slots * sizeof(float4)));
            HIP_TRY(ctx->qm.ensure((size_t)slots * sizeof(uint2)));
            w.qv = static_cast<float4*>(ctx->qv.p);
            w.qm = static_cast<uint2*>(ctx->qm.p);
            w.plist_n = static_cast<int32_t*>(ctx->plist_n.p);
            w.queue = w.plist_n + 1;
            // (plist_n[3] of every group: the fused order's arrival counter, zeroed per registration by
            // init_kernel)
            HIP_TRY(ctx->owork.ensure((size_t)npairs * sizeof(int32_t)));
            w.owork = static_cast<int32_t*>(ctx->owork.p);
        }
        if (pl.cache) {
            w.need_stride = (x_stride + 31) / 32;
            HIP_TRY(ctx->nn_lu.ensure((size_t)slots * sizeof(float)));
            HIP_TRY(ctx->nn_t.ensure((size_t)slots * sizeof(float4)));
            w.nn_t = static_cast<float4*>(ctx->nn_t.p);
            HIP_TRY(ctx->sq.ensure((size_t)slots * sizeof(float4)));
            HIP_TRY(ctx->sm.ensure((size_t)slots * sizeof(uint2)));

            HIP_TRY(ctx->need.ensure((size_t)npairs * w.need_stride * sizeof(uint32_t)));
            HIP_TRY(ctx->miss_cnt.ensure((size_t)npairs * sizeof(int32_t)));
            w.nn_u = static_cast<float*>(ctx->nn_lu.p);
            w.defer_xform = 1;
            w.sq = static_cast<float4*>(ctx->sq.p);
            w.sm = static_cast<uint2*>(ctx->sm.p);

            w.need = static_cast<uint32_t*>(ctx->need.p);
            w.miss_cnt = static_cast<int32_t*>(ctx->miss_cnt.p);
            w.part_size = opt(ctx, kOptPart, kDefaultPartSize);
            if (w.part_size != 0 && w.part_size < 64) w.part_size = 64;
            w.stage_sel = std::max(0, opt(ctx, kOptStageSel, kDefaultStageSel));
            // (a fresh registration starts from zero: init_kernel clears the pair's bitmap and count —
            // three memset launches per batch, and their boundaries, fewer)
        }
    }
    return ICP4R_OK;
}

// One NN pass over every active pair, timed with events: the roofline's kernel is the batched
// search (nn_lds_kernel) or, for the other plans, the NN launch itself.
int nn_pass(icp4r_ctx* ctx, const Plan& pl, const PairArgs& a, const WorkArgs& w0, int npairs, int max_n,
            int fitness_pass, int first, hipStream_t st, int ncu, int test_fused, int pass, int ordered) {
    EventPair* ne;
    int r;
    WorkArgs w = w0;  // debug: the pass' own event slots (plan option phase_ticks = 1)
    w.pass_ticks = (w0.ticks && pass >= 0 && pass < kMaxTickPasses)
                       ? w0.ticks + pass_tick_base(npairs) + (int64_t)pass * kPassTickSlots
                       : nullptr;
    // per-kernel events only when asked for (icp4r_set_kernel_timing: each record between two kernels
    // costs device time); the batch events around a registration are always recorded
    const bool kev = ctx->kernel_timing;
    EventPair none;
    none.start = none.stop = nullptr;
    if (kev) {
        if ((r = next_event(ctx->nn_events, ctx->nn_used, &ne))) return r;
    } else {
        ne = &none;
    }
    if (pl.lds) {
        NNLdsEvents ev;
        ev.search_start = ne->start;
        ev.search_stop = ne->stop;
        if (kev && pl.cache && !first && !test_fused) {
            EventPair* te;
            if ((r = next_event(ctx->test_events, ctx->test_used, &te))) return r;
            ev.test_start = te->start;
            ev.test_stop = te->stop;
        }
        HIP_TRY(launch_nn_lds(a, w, npairs, max_n, fitness_pass, first, ncu > 0 ? ncu : ctx->ncu, st, ev, test_fused,
                              ordered));
        return ICP4R_OK;
    }
    if (pl.tile) {  // the events bracket nn_tile_kernel itself (not its seed / record kernels)
        HIP_TRY(launch_nn_tile(a, w, npairs, max_n, pl.max_m, fitness_pass, first, pl.tile_run, st, ne->start, ne->stop));
        return ICP4R_OK;
    }
    if (kev) HIP_TRY(hipEventRecord(ne->start, st));
    if (pl.pruned) {
        HIP_TRY(launch_nn_pruned(pl.q, pl.chunk_sb, pl.chunks, a, w, npairs, max_n, fitness_pass, first, st));
    } else {
        if (pl.splits > 1) HIP_TRY(hipMemsetAsync(w.nn_key, 0xFF, (size_t)npairs * w.x_stride * sizeof(NNKey), st));
        HIP_TRY(launch_nn(pl.q, pl.packed, a, w, npairs, max_n, fitness_pass, st));
    }
    if (kev) HIP_TRY(hipEventRecord(ne->stop, st));
    return ICP4R_OK;
}

static_assert(sizeof(icp4r_ctx::aux_stream) / sizeof(hipStream_t) == kMaxGroups, "aux streams");

// Pairs [p0, p0 + np) of a batch as a batch of their own: every per-pair array offset by p0, the
// pass-scoped lists / counters of group g in their own slots.
void group_view(const PairArgs& a, const WorkArgs& w, int p0, int g, PairArgs& ag, WorkArgs& wg) {
    ag = a;
    ag.src_off += p0;
    ag.src_n += p0;
    ag.tgt_off += p0;
    ag.tgt_n += p0;
    if (ag.guess) ag.guess += (int64_t)p0 * 16;
    ag.results += p0;
    wg = w;
    const int64_t xs = (int64_t)p0 * w.x_stride;
    wg.X += xs;
    wg.nn_key += xs;
    wg.state += p0;
    if (wg.corr) wg.corr += xs * 2;
    if (wg.tsort) {
        wg.tsort += (int64_t)p0 * w.t_stride;
        wg.tinv += (int64_t)p0 * w.t_stride;
        wg.tbox += (int64_t)p0 * 2 * w.b_stride;
        wg.sbox += (int64_t)p0 * 2 * w.sb_stride;
        wg.sperm += xs;
        if (wg.kdn) wg.kdn += (int64_t)p0 * kKdnStride;
        if (wg.tbb) wg.tbb += (int64_t)p0 * 8;
        if (wg.mo_hist) wg.mo_hist += (int64_t)p0 * w.mo_groups * (1 << 14);
        if (wg.mo_rep) wg.mo_rep += (int64_t)p0 * (1 << 14);
    }
    if (wg.nn_u) {
        wg.nn_u += xs;
        wg.nn_t += xs;
        wg.sq += xs;
        wg.sm += xs;
        wg.need += (int64_t)p0 * w.need_stride;
        wg.miss_cnt += p0;
    }
    if (wg.plist) {
        wg.qv += xs;
        wg.qm += xs;
        wg.plist += (int64_t)p0 * ((w.x_stride + 63) / 64);
        wg.plist_n += 4 * g;
        wg.queue = wg.plist_n + 1;
        wg.owork += p0;
    }
    if (g > 0) wg.ticks = nullptr;  // debug slots are pair-0 / global
}

// The whole registration of a device-resident batch as one stream-ordered launch sequence.
// Large batched (LDS-plan) batches run as `groups` independent pair groups on their own streams,
// forked from and joined back into `st`: a group's HBM-bound kernels (cache test, fold) overlap the
// latency/issue-bound search of another (ICP4R_GROUPS, default kDefaultGroups).
int run_pairs(icp4r_ctx* ctx, const PairArgs& a, int npairs, int max_n, int max_m, int max_iterations,
              int nn_mode, hipStream_t st) {
    if (npairs <= 0) return ICP4R_OK;
    const int mn = max_n > 0 ? max_n : 1;
    const bool pcl = a.kp.numerics == kNumericsPCL;
    const Plan pl = make_plan(ctx, npairs, mn, max_m, nn_mode, true, pcl);
    WorkArgs w;
    int rc;
    if ((rc = setup_work(ctx, pl, npairs, max_n, max_m, pcl && !pl.solo, st, w))) return rc;
    // sources ordered by their target's kd tree (src_order_kernel) on the batched plan, where its
    // better first-pass seeds and one kd build per pair pay (C3 +2.9 %); a single pair's extra launch
    // does not (C1 0.75 -> 0.80 ms), so the unbatched plans build the source's own tree
    w.src_by_tgt = (pl.pruned && pl.lds) ? (opt(ctx, kOptSrcOrder, 1) != 0 ? 1 : 0)
                                         : (pl.pruned && opt(ctx, kOptSrcOrder, 0) != 0 ? 1 : 0);
    w.stage_first = (w.src_by_tgt && (pl.lds || pl.solo) && w.qv && w.qm) ? 1 : 0;
    // multi-tile plan (the scan-to-map target), PCL numerics: seeds written by the update's transform
    w.seed_next = (pl.tile && pl.chunks > 1 && pcl && w.corr && opt(ctx, kOptFuseSeed, 1) != 0) ? 1 : 0;
    // one-tile plan (C1, C2), PCL numerics: the update's transformCloud(T_inc) deferred into the next
    // search, which reads every query anyway (nn_tile_kernel; plan option tile_defer = 0: the update does it)
    if (pl.tile && pl.chunks == 1 && !pl.solo && pcl && w.corr && opt(ctx, kOptTileOwn, 1) != 0 &&
        opt(ctx, kOptTileDefer, 1) != 0)
        w.defer_xform = 1;
    EventPair* be;
    if ((rc = next_event(ctx->batch_events, ctx->batch_used, &be))) return rc;
    HIP_TRY(hipEventRecord(be->start, st));
    if (pl.solo) {  // init, the two kd builds, then every iteration and the fitness pass in one launch
        icp4r_host::Range solo_range("icp4r solo registration");
        HIP_TRY(launch_init(a, w, npairs, st));
        HIP_TRY(launch_index(a, w, npairs, st));
        const bool kev = ctx->kernel_timing;
        EventPair* ne = nullptr;
        if (kev) {
            if ((rc = next_event(ctx->nn_events, ctx->nn_used, &ne))) return rc;
            HIP_TRY(hipEventRecord(ne->start, st));
        }
        HIP_TRY(launch_solo(a, w, npairs, max_n, max_iterations > 0 ? max_iterations : 1, st));
        if (kev) HIP_TRY(hipEventRecord(ne->stop, st));
        HIP_TRY(hipEventRecord(be->stop, st));
        return ICP4R_OK;
    }
    // (at most kMaxGroups: a process has GPU_MAX_HW_QUEUES = 4 hardware queues, and a fourth group
    // shares one with the third, whose kernels then serialise — DESIGN.md §5; icp4r_set_plan_option
    // refuses more)
    int groups = pl.lds ? opt(ctx, kOptGroups, kDefaultGroups) : 1;
    if (groups < 1) groups = 1;
    if (groups > kMaxGroups) groups = kMaxGroups;
    while (groups > 1 && npairs / groups < kLdsMinPairs / 2) --groups;
    PairArgs ag[kMaxGroups];
    WorkArgs wg[kMaxGroups];
    hipStream_t gs[kMaxGroups];
    int gn[kMaxGroups];
    for (int g = 0; g < groups; ++g) {
        const int p0 = (int)((int64_t)npairs * g / groups), p1 = (int)((int64_t)npairs * (g + 1) / groups);
        gn[g] = p1 - p0;
        group_view(a, w, p0, g, ag[g], wg[g]);
        gs[g] = st;
        if (g > 0) {
            if (!ctx->aux_stream[g]) HIP_TRY(hipStreamCreateWithFlags(&ctx->aux_stream[g], hipStreamNonBlocking));
            if (!ctx->fork_ev[g]) HIP_TRY(hipEventCreateWithFlags(&ctx->fork_ev[g], hipEventDisableTiming));
            gs[g] = ctx->aux_stream[g];
        }
    }
    for (int g = 1; g < groups; ++g) HIP_TRY(hipStreamWaitEvent(gs[g], be->start, 0));  // fork
    // persistent search grid per group: CUs / groups (ICP4R_SEARCH_CU_DIV overrides), so the other
    // groups' kernels find CUs without a 150-KB search workgroup on them (C3: 2 groups on 128 CUs
    // each 91.5k pairs/s, on 256 CUs each 89.5k, one group 88.4k — measured in one session)
    const int cdiv = opt(ctx, kOptSearchCuDiv, groups);
    const int search_cu = cdiv > 1 ? (ctx->ncu + cdiv - 1) / cdiv : 0;
    for (int g = 0; g < groups; ++g) {
        HIP_TRY(launch_init(ag[g], wg[g], gn[g], gs[g]));
        if (pl.pruned) HIP_TRY(launch_index(ag[g], wg[g], gn[g], gs[g]));
    }
    // PCL's do { ... } while (!converged): at least one iteration even for max_iterations == 0.
    const int iters = max_iterations > 0 ? max_iterations : 1;
    // the cached-neighbour test of iteration passes 2.. runs in the tail of the previous update
    // (fold_update_kernel, PCL numerics; plan option fuse_test = 0: its own kernel)
    const bool fuse = pl.lds && pl.cache && pcl && opt(ctx, kOptFuseTest, 1) != 0;
    // ... and the work list of those passes is built by the update's last workgroup (plan option fuse_order = 0:
    // nn_order_kernel)
    const bool ford = fuse && opt(ctx, kOptFuseOrder, 1) != 0;
    // ... and folds the next pass A's source centroid sums over the X it writes, so that pass A reads
    // nn_t only (every correspondence kept, unweighted, no MSE criterion).  Off unless plan option sums_tail = 1:
    // the three n-long chains are serial, and in pass A they run beside the other chains for free, while
    // in the tail they lengthen the pair's critical path (C3: update 177 -> 190 us)
    for (int g = 0; g < groups; ++g)
        wg[g].sums_tail = (fuse && a.kp.huber_delta == INFINITY && a.kp.max_d2 >= FLT_MAX && !a.kp.need_mse &&
                           opt(ctx, kOptSumsTail, 0) != 0)
                              ? 1
                              : 0;
    // ... and the batched update holds each pair on chip (fold_update_res_kernel: sources <= kResMaxN,
    // unweighted, no distance threshold — PCL's defaults; plan option res_update = 0: fold_update_kernel)
    for (int g = 0; g < groups; ++g)
        wg[g].res_update = (fuse && pcl && mn <= kResMaxN && !wg[g].sums_tail && a.kp.huber_delta == INFINITY &&
                             a.kp.max_d2 >= FLT_MAX && opt(ctx, kOptResUpdate, kDefaultResUpdate) != 0)
                                ? 1
                                : 0;
    const bool kev = ctx->kernel_timing;  // per-kernel events (icp4r_set_kernel_timing; nn_pass: the same)
    // at most one pair per CU: the update in one 1024-thread workgroup per pair, its sigma panels side
    // by side (plan option wide_update = 0: fold_update_kernel's 256 threads)
    const bool wide = pcl && !fuse && npairs <= ctx->ncu && opt(ctx, kOptWideUpdate, 1) != 0;
    // ... with the records held in registers from pass A to pass B for sources of at most kHeldMaxN
    // points (fold_update_held_kernel; plan option held_update = 0: fold_update_wide_kernel)
    for (int g = 0; g < groups; ++g)
        wg[g].held_update = (wide && mn <= kHeldMaxN && opt(ctx, kOptHeldUpdate, kDefaultHeldUpdate) != 0) ? 1 : 0;
    // ... which, on the multi-tile plan (the scan-to-map target), forms the correspondence records in
    // its pass A instead of corr_kernel after every search (plan option fold_keys = 0: corr_kernel)
    if (wide && pl.tile && !pl.lds && w.corr && (pl.chunks > 1 || !w.tile_own) && opt(ctx, kOptFoldKeys, 1) != 0)
        for (int g = 0; g < groups; ++g) wg[g].fold_keys = 1;
    char pass_name[48];
    for (int it = 0; it < iters; ++it) {
        snprintf(pass_name, sizeof(pass_name), "icp4r ICP pass %d", it + 1);
        icp4r_host::Range pass_range(pass_name);
        for (int g = 0; g < groups; ++g) {
            const int ncu_g = search_cu > 0 ? search_cu : ctx->ncu;
            if ((rc = nn_pass(ctx, pl, ag[g], wg[g], gn[g], mn, 0, it == 0, gs[g], search_cu, fuse && it > 0, it,
                              ford && it > 0)))
                return rc;
            EventPair* ue = nullptr;
            if (kev) {
                if ((rc = next_event(ctx->upd_events, ctx->upd_used, &ue))) return rc;
                HIP_TRY(hipEventRecord(ue->start, gs[g]));
            }
            HIP_TRY(launch_update(ag[g], wg[g], gn[g], mn, pcl && !pl.pruned, gs[g], fuse && it + 1 < iters,
                                  ford && it + 1 < iters ? ncu_g : 0, wide));
            if (kev) HIP_TRY(hipEventRecord(ue->stop, gs[g]));
        }
    }
    icp4r_host::Range fit_range("icp4r fitness pass");
    for (int g = 0; g < groups; ++g) {
        // the fitness pass' cached-neighbour test runs inside fitness_prep_kernel when fused; on the
        // one-tile plan (no cache, no seeds) the search forms X := final * input itself, one launch and
        // one boundary fewer (plan option fit_xform = 0: fitness_prep_kernel)
        const int ftest = fuse && a.kp.compute_fitness ? 1 : 0;
        wg[g].fit_xform = (a.kp.compute_fitness && pl.tile && !pl.lds && pl.max_m <= kLdsMaxTargets && wg[g].tile_own &&
                           !wg[g].nn_u && !wg[g].seed_next && opt(ctx, kOptFitXform, 1) != 0)
                              ? 1
                              : 0;
        if ((a.kp.compute_fitness || a.aligned) && !wg[g].fit_xform)
            HIP_TRY(launch_fitness_prep(ag[g], wg[g], gn[g], gs[g], ftest));
        if (a.kp.compute_fitness && (rc = nn_pass(ctx, pl, ag[g], wg[g], gn[g], mn, 1, 0, gs[g], search_cu, ftest, iters)))
            return rc;
        HIP_TRY(launch_finish(ag[g], wg[g], gn[g], gs[g]));
    }
    for (int g = 1; g < groups; ++g) {  // join
        HIP_TRY(hipEventRecord(ctx->fork_ev[g], gs[g]));
        HIP_TRY(hipStreamWaitEvent(st, ctx->fork_ev[g], 0));
    }
    HIP_TRY(hipEventRecord(be->stop, st));
    return ICP4R_OK;
}

// Exact 1-NN of n host queries (optionally transformed by T, column-major) in a host target: the
// registration's own NN path (init = transformCloud(query, T); index; one NN pass), keys copied
// back.  Used by icp4r_nearest and icp4r_fitness.
int nearest_keys(icp4r_ctx* ctx, const float* query, int32_t n, int32_t qstride, const float* tgt, int32_t m,
                 int32_t tstride, const float* T, std::vector<NNKey>& keys) {
    std::vector<float> hq, ht;
    pack_host(query, n, qstride, hq);
    pack_host(tgt, m, tstride, ht);
    hipStream_t st = ctx->stream;
    const int64_t zero64 = 0;
    HIP_TRY(ctx->src.ensure(hq.size() * 4));
    HIP_TRY(ctx->tgt.ensure(ht.size() * 4));
    HIP_TRY(ctx->src_off.ensure(16));
    HIP_TRY(ctx->tgt_off.ensure(16));
    HIP_TRY(ctx->src_n.ensure(16));
    HIP_TRY(ctx->tgt_n.ensure(16));
    HIP_TRY(ctx->guess.ensure(64));
    HIP_TRY(ctx->results.ensure(sizeof(icp4r_result)));
    HIP_TRY(hipMemcpyAsync(ctx->src.p, hq.data(), hq.size() * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->tgt.p, ht.data(), ht.size() * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->src_off.p, &zero64, 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->tgt_off.p, &zero64, 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->src_n.p, &n, 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->tgt_n.p, &m, 4, hipMemcpyHostToDevice, st));
    if (T) HIP_TRY(hipMemcpyAsync(ctx->guess.p, T, 64, hipMemcpyHostToDevice, st));
    PairArgs a;
    memset(&a, 0, sizeof(a));
    a.src = static_cast<const float4*>(ctx->src.p);
    a.tgt = static_cast<const float4*>(ctx->tgt.p);
    a.src_off = static_cast<const int64_t*>(ctx->src_off.p);
    a.tgt_off = static_cast<const int64_t*>(ctx->tgt_off.p);
    a.src_n = static_cast<const int32_t*>(ctx->src_n.p);
    a.tgt_n = static_cast<const int32_t*>(ctx->tgt_n.p);
    a.guess = T ? static_cast<const float*>(ctx->guess.p) : nullptr;
    a.results = static_cast<Result*>(ctx->results.p);
    int rc;
    if ((rc = make_kparams(nullptr, &a.kp))) return rc;
    const Plan pl = make_plan(ctx, 1, n, m, ICP4R_NN_AUTO);
    WorkArgs w;
    if ((rc = setup_work(ctx, pl, 1, n, m, false, st, w))) return rc;
    HIP_TRY(launch_init(a, w, 1, st));
    if (pl.pruned) HIP_TRY(launch_index(a, w, 1, st));
    if ((rc = nn_pass(ctx, pl, a, w, 1, n, 0, 1, st, 0, 0, -1))) return rc;
    PairState ps;
    keys.resize((size_t)n);
    HIP_TRY(hipMemcpyAsync(&ps, w.state, sizeof(ps), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(keys.data(), w.nn_key, (size_t)n * sizeof(NNKey), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (ps.phase == kPhaseInvalid) return fail(ps.status, "non-finite coordinate in the query or target cloud");
    return ICP4R_OK;
}

int events_avg(std::vector<EventPair>& v, size_t used, double* avg_ms) {
    double tot = 0.0;
    for (size_t i = 0; i < used; ++i) {
        HIP_TRY(hipEventSynchronize(v[i].stop));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, v[i].start, v[i].stop));
        tot += ms;
    }
    *avg_ms = used ? tot / (double)used : 0.0;
    return ICP4R_OK;
}

}  // namespace icp4r_pipe

using namespace icp4r_pipe;

extern "C" {

const char* icp4r_version(void) { return "icp4r 0.2.0 (gfx950, HIP)"; }
int icp4r_abi_version(void) { return ICP4R_ABI_VERSION; }
const char* icp4r_last_error(void) { return icp4r_host::g_last_error.c_str(); }

void icp4r_params_default(icp4r_params* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->max_iterations = 10;                       // Registration::max_iterations_
    p->min_correspondences = 3;                   // Registration::min_number_correspondences_
    p->max_correspondence_distance = sqrt(DBL_MAX);  // Registration::corr_dist_threshold_
    p->transformation_epsilon = 0.0;
    p->transformation_rotation_epsilon = 0.0;
    p->euclidean_fitness_epsilon = -DBL_MAX;
    p->mse_threshold_absolute = 1e-12;            // DefaultConvergenceCriteria
    p->max_iterations_similar_transforms = 0;
    p->numerics = ICP4R_NUMERICS_PCL;
    p->nn_mode = ICP4R_NN_AUTO;
    p->compute_fitness = 1;
    p->huber_delta = INFINITY;
    p->fitness_max_range = DBL_MAX;
}

int icp4r_device_count(int* count) {
    if (!count) return fail(ICP4R_E_INVALID, "count is NULL");
    HIP_TRY(hipGetDeviceCount(count));
    return ICP4R_OK;
}

int icp4r_create(icp4r_ctx** out, int device) {
    if (!out) return fail(ICP4R_E_INVALID, "out is NULL");
    *out = nullptr;
    if (device == ICP4R_NO_DEVICE) {  // plan queries and plan options only: no HIP call, no stream
        icp4r_ctx* c = new icp4r_ctx();
        c->device = ICP4R_NO_DEVICE;
        *out = c;
        return ICP4R_OK;
    }
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(ICP4R_E_INVALID, "device %d out of range (%d devices)", device, n);
    HIP_TRY(hipSetDevice(device));
    icp4r_ctx* c = new icp4r_ctx();
    c->device = device;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0) c->ncu = ncu;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(ICP4R_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    *out = c;
    return ICP4R_OK;
}

int icp4r_destroy(icp4r_ctx* ctx) {
    if (!ctx) return ICP4R_OK;
    for (icp4r_comm* c : ctx->comms) icp4r_host::comm_detach(c);
    if (ctx->device == ICP4R_NO_DEVICE) {
        delete ctx;
        return ICP4R_OK;
    }
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (int g = 0; g < kMaxGroups; ++g) {
        if (ctx->aux_stream[g]) (void)hipStreamDestroy(ctx->aux_stream[g]);
        if (ctx->fork_ev[g]) (void)hipEventDestroy(ctx->fork_ev[g]);
    }
    for (DevBuf* b : {&ctx->src, &ctx->tgt, &ctx->src_off, &ctx->src_n, &ctx->tgt_off, &ctx->tgt_n, &ctx->guess,
                      &ctx->aligned, &ctx->results, &ctx->T, &ctx->X, &ctx->nn_key,
                      &ctx->state, &ctx->tsort, &ctx->tinv, &ctx->tbox, &ctx->sbox, &ctx->sperm, &ctx->evals, &ctx->corr, &ctx->ticks, &ctx->nn_lu, &ctx->nn_t, &ctx->kdn, &ctx->sq, &ctx->sm, &ctx->qv, &ctx->qm, &ctx->need,
                      &ctx->miss_cnt, &ctx->plist, &ctx->plist_n, &ctx->owork, &ctx->ego_rec, &ctx->ego_off, &ctx->ego_cnt, &ctx->ego_feat,
                      &ctx->ego_pd, &ctx->ego_scores, &ctx->ego_res, &ctx->ego_mask, &ctx->ego_xyzi, &ctx->gicp_gs,
                      &ctx->gicp_cov_src, &ctx->gicp_cov_tgt, &ctx->gicp_mah, &ctx->gicp_active, &ctx->gicp_part, &ctx->gicp_sidx})
        b->release();
    for (auto* v : {&ctx->nn_events, &ctx->test_events, &ctx->upd_events, &ctx->batch_events, &ctx->gicp_events})
        for (auto& ev : *v) {
            (void)hipEventDestroy(ev.start);
            (void)hipEventDestroy(ev.stop);
        }
    if (ctx->gicp_hflag) (void)hipHostFree(ctx->gicp_hflag);
    if (ctx->gicp_fork) (void)hipEventDestroy(ctx->gicp_fork);
    if (ctx->gicp_join) (void)hipEventDestroy(ctx->gicp_join);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return ICP4R_OK;
}

int icp4r_align(icp4r_ctx* ctx, const float* src, int32_t n, int32_t src_stride_bytes, const float* tgt, int32_t m,
                int32_t tgt_stride_bytes, const float* guess, const icp4r_params* params, icp4r_result* out,
                float* aligned_out, int32_t out_stride_bytes) {
    if (!ctx || !out) return fail(ICP4R_E_INVALID, "ctx/out is NULL");
    icp4r_host::Range range("icp4r_align");
    int rc;
    if ((rc = check_cloud(src, n, src_stride_bytes, "source"))) return rc;
    if ((rc = check_cloud(tgt, m, tgt_stride_bytes, "target"))) return rc;
    if (aligned_out && (out_stride_bytes < 12 || out_stride_bytes % 4))
        return fail(ICP4R_E_INVALID, "aligned_out stride %d bytes", out_stride_bytes);
    KParams kp;
    if ((rc = make_kparams(params, &kp))) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    std::vector<float> hs, ht;
    pack_host(src, n, src_stride_bytes, hs);
    pack_host(tgt, m, tgt_stride_bytes, ht);
    const int64_t zero64 = 0;
    HIP_TRY(ctx->src.ensure(hs.size() * sizeof(float)));
    HIP_TRY(ctx->tgt.ensure(ht.size() * sizeof(float)));
    HIP_TRY(ctx->src_off.ensure(16));
    HIP_TRY(ctx->tgt_off.ensure(16));
    HIP_TRY(ctx->src_n.ensure(16));
    HIP_TRY(ctx->tgt_n.ensure(16));
    HIP_TRY(ctx->guess.ensure(16 * sizeof(float)));
    HIP_TRY(ctx->results.ensure(sizeof(icp4r_result)));
    HIP_TRY(ctx->aligned.ensure(hs.size() * sizeof(float)));
    hipStream_t st = ctx->stream;
    HIP_TRY(hipMemcpyAsync(ctx->src.p, hs.data(), hs.size() * sizeof(float), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->tgt.p, ht.data(), ht.size() * sizeof(float), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->src_off.p, &zero64, 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->tgt_off.p, &zero64, 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->src_n.p, &n, 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->tgt_n.p, &m, 4, hipMemcpyHostToDevice, st));
    if (guess) HIP_TRY(hipMemcpyAsync(ctx->guess.p, guess, 16 * sizeof(float), hipMemcpyHostToDevice, st));
    PairArgs a;
    a.src = static_cast<const float4*>(ctx->src.p);
    a.tgt = static_cast<const float4*>(ctx->tgt.p);
    a.src_off = static_cast<const int64_t*>(ctx->src_off.p);
    a.tgt_off = static_cast<const int64_t*>(ctx->tgt_off.p);
    a.src_n = static_cast<const int32_t*>(ctx->src_n.p);
    a.tgt_n = static_cast<const int32_t*>(ctx->tgt_n.p);
    a.guess = guess ? static_cast<const float*>(ctx->guess.p) : nullptr;
    a.aligned = aligned_out ? static_cast<float4*>(ctx->aligned.p) : nullptr;
    a.results = static_cast<Result*>(ctx->results.p);
    a.kp = kp;
    const int iters = params ? params->max_iterations : 10;
    if ((rc = run_pairs(ctx, a, 1, n, m, iters, params ? params->nn_mode : ICP4R_NN_AUTO, st))) return rc;
    HIP_TRY(hipMemcpyAsync(out, ctx->results.p, sizeof(icp4r_result), hipMemcpyDeviceToHost, st));
    std::vector<float> ha;
    if (aligned_out && n > 0) {
        ha.resize((size_t)n * 4);
        HIP_TRY(hipMemcpyAsync(ha.data(), ctx->aligned.p, ha.size() * sizeof(float), hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (aligned_out && n > 0) {
        unsigned char* o = reinterpret_cast<unsigned char*>(aligned_out);
        for (int32_t i = 0; i < n; ++i) {
            float* q = reinterpret_cast<float*>(o + (size_t)i * out_stride_bytes);
            q[0] = ha[4 * (size_t)i];
            q[1] = ha[4 * (size_t)i + 1];
            q[2] = ha[4 * (size_t)i + 2];
            if (out_stride_bytes >= 16) q[3] = ha[4 * (size_t)i + 3];
        }
    }
    if (out->status != ICP4R_OK) {
        const char* what = out->status == ICP4R_E_TOO_FEW_CORR ? "Not enough correspondences found. Relax your threshold parameters."
                           : out->status == ICP4R_E_EMPTY      ? "No input target dataset was given!"
                           : out->status == ICP4R_E_NONFINITE  ? "non-finite coordinate in an input cloud"
                                                               : "registration failed";
        return fail(out->status, "[icp4r::IterativeClosestPoint::computeTransformation] %s", what);
    }
    return ICP4R_OK;
}

int icp4r_align_batch_device(icp4r_ctx* ctx, const icp4r_batch* b, const icp4r_params* params, icp4r_result* results,
                             void* hip_stream) {
    if (!ctx || !b || !results) return fail(ICP4R_E_INVALID, "ctx/batch/results is NULL");
    icp4r_host::Range range("icp4r_align_batch_device");
    if (b->npairs < 0) return fail(ICP4R_E_INVALID, "npairs < 0");
    if (b->npairs == 0) return ICP4R_OK;
    if (!b->src || !b->tgt || !b->src_off || !b->src_n || !b->tgt_off || !b->tgt_n)
        return fail(ICP4R_E_INVALID, "batch has a NULL device array");
    if (b->max_src_n < 0 || b->max_tgt_n < 0) return fail(ICP4R_E_INVALID, "negative max sizes");
    KParams kp;
    int rc;
    if ((rc = make_kparams(params, &kp))) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    PairArgs a;
    a.src = reinterpret_cast<const float4*>(b->src);
    a.tgt = reinterpret_cast<const float4*>(b->tgt);
    a.src_off = b->src_off;
    a.src_n = b->src_n;
    a.tgt_off = b->tgt_off;
    a.tgt_n = b->tgt_n;
    a.guess = b->guess;
    a.aligned = reinterpret_cast<float4*>(b->aligned);
    a.results = reinterpret_cast<Result*>(results);
    a.kp = kp;
    hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->stream;
    return run_pairs(ctx, a, b->npairs, b->max_src_n, b->max_tgt_n, params ? params->max_iterations : 10,
                     params ? params->nn_mode : ICP4R_NN_AUTO, st);
}

int icp4r_align_batch_host(icp4r_ctx* ctx, const float* src, const int64_t* src_off, const int32_t* src_n,
                           const float* tgt, const int64_t* tgt_off, const int32_t* tgt_n, int32_t npairs,
                           const float* guess, const icp4r_params* params, icp4r_result* results) {
    if (!ctx || !results || npairs < 0) return fail(ICP4R_E_INVALID, "bad arguments");
    icp4r_host::Range range("icp4r_align_batch_host");
    if (npairs == 0) return ICP4R_OK;
    if (!src_off || !src_n || !tgt_off || !tgt_n) return fail(ICP4R_E_INVALID, "NULL offset/count array");
    // only the point ranges the pairs cover are uploaded, offsets rebased to them (a shard of a larger
    // host batch, icp4r_align_batch_multi, uploads its own points only)
    int64_t s_lo = INT64_MAX, s_hi = 0, t_lo = INT64_MAX, t_hi = 0;
    int32_t max_n = 0, max_m = 0;
    for (int32_t p = 0; p < npairs; ++p) {
        if (src_n[p] < 0 || tgt_n[p] < 0 || src_off[p] < 0 || tgt_off[p] < 0)
            return fail(ICP4R_E_INVALID, "pair %d: negative offset/count", p);
        if (src_n[p] > 0) {
            s_lo = std::min<int64_t>(s_lo, src_off[p]);
            s_hi = std::max<int64_t>(s_hi, src_off[p] + src_n[p]);
        }
        if (tgt_n[p] > 0) {
            t_lo = std::min<int64_t>(t_lo, tgt_off[p]);
            t_hi = std::max<int64_t>(t_hi, tgt_off[p] + tgt_n[p]);
        }
        if (src_n[p] > max_n) max_n = src_n[p];
        if (tgt_n[p] > max_m) max_m = tgt_n[p];
    }
    if (s_lo > s_hi) s_lo = s_hi = 0;
    if (t_lo > t_hi) t_lo = t_hi = 0;
    const int64_t ns = s_hi - s_lo, nt = t_hi - t_lo;
    if ((ns > 0 && !src) || (nt > 0 && !tgt)) return fail(ICP4R_E_INVALID, "NULL cloud data");
    std::vector<int64_t> so((size_t)npairs), to((size_t)npairs);
    for (int32_t p = 0; p < npairs; ++p) {
        so[p] = src_n[p] > 0 ? src_off[p] - s_lo : 0;
        to[p] = tgt_n[p] > 0 ? tgt_off[p] - t_lo : 0;
    }
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    HIP_TRY(ctx->src.ensure((size_t)(ns > 0 ? ns : 1) * 16));
    HIP_TRY(ctx->tgt.ensure((size_t)(nt > 0 ? nt : 1) * 16));
    HIP_TRY(ctx->src_off.ensure((size_t)npairs * 8));
    HIP_TRY(ctx->tgt_off.ensure((size_t)npairs * 8));
    HIP_TRY(ctx->src_n.ensure((size_t)npairs * 4));
    HIP_TRY(ctx->tgt_n.ensure((size_t)npairs * 4));
    HIP_TRY(ctx->results.ensure((size_t)npairs * sizeof(icp4r_result)));
    if (guess) HIP_TRY(ctx->guess.ensure((size_t)npairs * 64));
    if (ns > 0) HIP_TRY(hipMemcpyAsync(ctx->src.p, src + 4 * s_lo, (size_t)ns * 16, hipMemcpyHostToDevice, st));
    if (nt > 0) HIP_TRY(hipMemcpyAsync(ctx->tgt.p, tgt + 4 * t_lo, (size_t)nt * 16, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->src_off.p, so.data(), (size_t)npairs * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->tgt_off.p, to.data(), (size_t)npairs * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->src_n.p, src_n, (size_t)npairs * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->tgt_n.p, tgt_n, (size_t)npairs * 4, hipMemcpyHostToDevice, st));
    if (guess) HIP_TRY(hipMemcpyAsync(ctx->guess.p, guess, (size_t)npairs * 64, hipMemcpyHostToDevice, st));
    icp4r_batch b;
    memset(&b, 0, sizeof(b));
    b.src = static_cast<const float*>(ctx->src.p);
    b.tgt = static_cast<const float*>(ctx->tgt.p);
    b.src_off = static_cast<const int64_t*>(ctx->src_off.p);
    b.tgt_off = static_cast<const int64_t*>(ctx->tgt_off.p);
    b.src_n = static_cast<const int32_t*>(ctx->src_n.p);
    b.tgt_n = static_cast<const int32_t*>(ctx->tgt_n.p);
    b.guess = guess ? static_cast<const float*>(ctx->guess.p) : nullptr;
    b.npairs = npairs;
    b.max_src_n = max_n;
    b.max_tgt_n = max_m;
    int rc = icp4r_align_batch_device(ctx, &b, params, static_cast<icp4r_result*>(ctx->results.p), st);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(results, ctx->results.p, (size_t)npairs * sizeof(icp4r_result), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return ICP4R_OK;
}

int icp4r_nearest(icp4r_ctx* ctx, const float* query, int32_t n, int32_t query_stride_bytes, const float* tgt,
                  int32_t m, int32_t tgt_stride_bytes, int32_t* idx_out, float* d2_out) {
    if (!ctx || (n > 0 && (!idx_out || !d2_out))) return fail(ICP4R_E_INVALID, "NULL argument");
    int rc;
    if ((rc = check_cloud(query, n, query_stride_bytes, "query"))) return rc;
    if ((rc = check_cloud(tgt, m, tgt_stride_bytes, "target"))) return rc;
    if (m == 0) return fail(ICP4R_E_EMPTY, "empty target");
    if (n == 0) return ICP4R_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    std::vector<NNKey> keys;
    if ((rc = nearest_keys(ctx, query, n, query_stride_bytes, tgt, m, tgt_stride_bytes, nullptr, keys))) return rc;
    for (int32_t i = 0; i < n; ++i) {
        idx_out[i] = key_idx(keys[i]);
        d2_out[i] = key_d2(keys[i]);
    }
    return ICP4R_OK;
}

int icp4r_fitness(icp4r_ctx* ctx, const float* src, int32_t n, int32_t src_stride_bytes, const float* tgt, int32_t m,
                  int32_t tgt_stride_bytes, const float* T, double max_range, double* fitness) {
    if (!ctx || !T || !fitness) return fail(ICP4R_E_INVALID, "NULL argument");
    int rc;
    if ((rc = check_cloud(src, n, src_stride_bytes, "source"))) return rc;
    if ((rc = check_cloud(tgt, m, tgt_stride_bytes, "target"))) return rc;
    *fitness = DBL_MAX;
    if (m == 0) return fail(ICP4R_E_EMPTY, "empty target");
    if (n == 0) return ICP4R_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    std::vector<NNKey> keys;
    if ((rc = nearest_keys(ctx, src, n, src_stride_bytes, tgt, m, tgt_stride_bytes, T, keys))) return rc;
    // Registration::getFitnessScore: sequential double sum over points with d2 <= max_range
    double sum = 0.0;
    int nr = 0;
    for (int32_t i = 0; i < n; ++i) {
        const float d2 = key_d2(keys[i]);
        if (d2 <= max_range) {
            sum += d2;
            ++nr;
        }
    }
    *fitness = nr > 0 ? sum / nr : DBL_MAX;
    return ICP4R_OK;
}

int icp4r_synchronize(icp4r_ctx* ctx, void* hip_stream) {
    if (!ctx) return fail(ICP4R_E_INVALID, "ctx is NULL");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipStreamSynchronize(hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->stream));
    return ICP4R_OK;
}

int icp4r_kernel_time_ms(icp4r_ctx* ctx, double* avg_ms, int32_t* launches) {
    if (!ctx || !avg_ms) return fail(ICP4R_E_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(ctx->device));
    int rc = events_avg(ctx->nn_events, ctx->nn_used, avg_ms);
    if (launches) *launches = (int32_t)ctx->nn_used;
    return rc;
}

int icp4r_batch_time_ms(icp4r_ctx* ctx, double* avg_ms, int32_t* calls) {
    if (!ctx || !avg_ms) return fail(ICP4R_E_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(ctx->device));
    int rc = events_avg(ctx->batch_events, ctx->batch_used, avg_ms);
    if (calls) *calls = (int32_t)ctx->batch_used;
    return rc;
}

int icp4r_stage_time_ms(icp4r_ctx* ctx, int32_t stage, double* avg_ms, int32_t* launches) {
    if (!ctx || !avg_ms) return fail(ICP4R_E_INVALID, "NULL argument");
    std::vector<EventPair>* v;
    size_t used;
    switch (stage) {
        case ICP4R_STAGE_NN: v = &ctx->nn_events; used = ctx->nn_used; break;
        case ICP4R_STAGE_NN_TEST: v = &ctx->test_events; used = ctx->test_used; break;
        case ICP4R_STAGE_UPDATE: v = &ctx->upd_events; used = ctx->upd_used; break;
        case ICP4R_STAGE_BATCH: v = &ctx->batch_events; used = ctx->batch_used; break;
        case ICP4R_STAGE_GICP_COV: v = &ctx->gicp_events; used = ctx->gicp_used; break;
        default: return fail(ICP4R_E_INVALID, "unknown stage %d", stage);
    }
    HIP_TRY(hipSetDevice(ctx->device));
    int rc = events_avg(*v, used, avg_ms);
    if (launches) *launches = (int32_t)used;
    return rc;
}

int icp4r_set_kernel_timing(icp4r_ctx* ctx, int32_t enable) {
    if (!ctx) return fail(ICP4R_E_INVALID, "ctx is NULL");
    ctx->kernel_timing = enable != 0;
    return ICP4R_OK;
}

int icp4r_kernel_time_reset(icp4r_ctx* ctx) {
    if (!ctx) return fail(ICP4R_E_INVALID, "ctx is NULL");
    ctx->nn_used = 0;
    ctx->test_used = 0;
    ctx->upd_used = 0;
    ctx->batch_used = 0;
    ctx->gicp_used = 0;
    if (ctx->evals.p) {
        HIP_TRY(hipSetDevice(ctx->device));
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipMemset(ctx->evals.p, 0, kCountBytes));
    }
    return ICP4R_OK;
}

// Plan options: per-context values of icp4r_pipe::PlanOpt.  Ranges are checked where a
// value would pick a wrong plan rather than fall back to a default.
namespace {
int plan_opt_index(const char* name) {
    if (!name) return -1;
    for (int k = 0; k < kNumPlanOpts; ++k)
        if (strcmp(name, kPlanOptNames[k]) == 0) return k;
    return -1;
}
}  // namespace

int icp4r_set_plan_option(icp4r_ctx* ctx, const char* name, int32_t value) {
    if (!ctx) return fail(ICP4R_E_INVALID, "ctx is NULL");
    const int k = plan_opt_index(name);
    if (k < 0) return fail(ICP4R_E_INVALID, "unknown plan option '%s'", name ? name : "(null)");
    if (k == kOptGroups && (value < 1 || value > kMaxGroups))
        return fail(ICP4R_E_INVALID,
                    "plan option groups = %d: 1..%d (a fourth pair group shares a hardware queue with the third, "
                    "and its kernels serialise)",
                    value, kMaxGroups);
    if (k == kOptXpad && (value < 0 || value > 1 << 20)) return fail(ICP4R_E_INVALID, "plan option xpad = %d", value);
    if (k == kOptSearchCuDiv && value < 0) return fail(ICP4R_E_INVALID, "plan option search_cu_div = %d", value);
    ctx->plan_val[k] = value;
    ctx->plan_set |= 1ull << k;
    return ICP4R_OK;
}

int icp4r_get_plan_option(const icp4r_ctx* ctx, const char* name, int32_t* value, int32_t* is_set) {
    if (!ctx || !value) return fail(ICP4R_E_INVALID, "NULL argument");
    const int k = plan_opt_index(name);
    if (k < 0) return fail(ICP4R_E_INVALID, "unknown plan option '%s'", name ? name : "(null)");
    const bool set = (ctx->plan_set >> k) & 1ull;
    *value = set ? ctx->plan_val[k] : INT32_MIN;
    if (!set) {  // the default in effect (what the plan code falls back to)
        static const int32_t dflt[kNumPlanOpts] = {
            0 /*nn_q: per plan*/, kDefaultLeaf, 0 /*chunk_sb: auto*/, -1 /*nn_lds: auto*/, 1, 1, 0 /*tile_run: auto*/,
            -1 /*solo: auto*/, 0, 0, 3, 1, kDefaultPartSize, -1 /*src_order: per plan*/, 1, 1, 1, kDefaultGroups,
            0 /*search_cu_div: groups*/, 1, 1, 0, 1, 0, 0, 1, kGicpSpec, kGicpGrid,
            0 /*gicp_knn_lanes: auto*/, kDefaultResUpdate, kDefaultHeldUpdate, 1, 0, kDefaultStageSel};
        *value = dflt[k];
    }
    if (is_set) *is_set = set ? 1 : 0;
    return ICP4R_OK;
}

int icp4r_reset_plan_options(icp4r_ctx* ctx) {
    if (!ctx) return fail(ICP4R_E_INVALID, "ctx is NULL");
    ctx->plan_set = 0;
    return ICP4R_OK;
}

int icp4r_plan(const icp4r_ctx* ctx, int32_t npairs, int32_t max_src_n, int32_t max_tgt_n, int32_t nn_mode,
               int32_t numerics, icp4r_plan_info* out) {
    if (npairs <= 0 || max_src_n < 0 || max_tgt_n < 0 || !out) return fail(ICP4R_E_INVALID, "bad shape");
    if (nn_mode < ICP4R_NN_AUTO || nn_mode > ICP4R_NN_PRUNED) return fail(ICP4R_E_INVALID, "unknown nn_mode %d", nn_mode);
    if (numerics != ICP4R_NUMERICS_PCL && numerics != ICP4R_NUMERICS_F64)
        return fail(ICP4R_E_INVALID, "unknown numerics mode %d", numerics);
    const bool pcl = numerics == ICP4R_NUMERICS_PCL;
    const Plan pl = make_plan(ctx, npairs, max_src_n > 0 ? max_src_n : 1, max_tgt_n, nn_mode, true, pcl);
    out->pruned = pl.pruned ? 1 : 0;
    out->solo = pl.solo ? 1 : 0;
    // run_pairs' choice: no solo plan, no fused cache test, at most one pair per CU of the context's
    // device (256 without a context), PCL numerics
    const int ncu = ctx ? ctx->ncu : 256;
    const bool fuse = pl.lds && pl.cache && pcl && opt(ctx, kOptFuseTest, 1) != 0;
    out->wide_update = (pcl && !pl.solo && !fuse && npairs <= ncu && opt(ctx, kOptWideUpdate, 1) != 0) ? 1 : 0;
    out->held_update = (out->wide_update && max_src_n <= kHeldMaxN && opt(ctx, kOptHeldUpdate, kDefaultHeldUpdate) != 0) ? 1 : 0;
    out->res_update = (fuse && max_src_n <= kResMaxN && opt(ctx, kOptSumsTail, 0) == 0 && opt(ctx, kOptResUpdate, kDefaultResUpdate) != 0) ? 1 : 0;
    out->q = pl.q;
    out->splits = pl.splits;
    out->leaf = pl.leaf;
    out->lds = pl.lds ? 1 : 0;
    out->cache = pl.cache ? 1 : 0;
    out->nn_blocks = pl.blocks;
    return ICP4R_OK;
}

int icp4r_nn_counters(icp4r_ctx* ctx, uint64_t* evaluations, uint64_t* box_tests) {
    if (!ctx || !evaluations) return fail(ICP4R_E_INVALID, "NULL argument");
    uint64_t v[kNumCounters];
    int rc = read_counters(ctx, v);
    if (rc) return rc;
    *evaluations = v[0];
    if (box_tests) *box_tests = v[1];
    return ICP4R_OK;
}

int icp4r_nn_cache_hits(icp4r_ctx* ctx, uint64_t* hits) {
    if (!ctx || !hits) return fail(ICP4R_E_INVALID, "NULL argument");
    uint64_t v[kNumCounters];
    int rc = read_counters(ctx, v);
    if (rc) return rc;
    *hits = v[2];
    return ICP4R_OK;
}

int icp4r_nn_stats(icp4r_ctx* ctx, icp4r_nn_stats_t* out) {
    if (!ctx || !out) return fail(ICP4R_E_INVALID, "NULL argument");
    uint64_t v[kNumCounters];
    int rc = read_counters(ctx, v);
    if (rc) return rc;
    memset(out, 0, sizeof(*out));
    out->evaluations = v[0];
    out->box_tests = v[1];
    out->cache_hits = v[2];
    out->cache_tested = v[3];
    out->records_written_by_test = v[4];
    out->tested_in_update = v[5];
    out->hits_in_update = v[6];
    out->second_chance_hits = v[7];
    return ICP4R_OK;
}

// Internal debug hook (not in icp4r.h): the last fold_update phase timestamps of pair 0 (100 MHz
// ticks; needs plan option phase_ticks = 1 on the context when the registration ran).
int icp4r__debug_ticks(icp4r_ctx* ctx, uint64_t* out, int32_t k) {
    if (!ctx || !out || k <= 0 || (size_t)k * sizeof(uint64_t) > ctx->ticks.cap) return fail(ICP4R_E_INVALID, "bad arguments");
    if (!ctx->ticks.p) return fail(ICP4R_E_INVALID, "phase ticks not enabled (plan option phase_ticks = 1)");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, ctx->ticks.p, (size_t)k * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return ICP4R_OK;
}

// Internal test hook (not part of the public ABI in icp4r.h): the device float Umeyama rotation of
// k row-major 3x3 matrices, host buffers.
int icp4r__test_rot_f32(icp4r_ctx* ctx, const float* sigma, float* R, int32_t k) {
    if (!ctx || !sigma || !R || k <= 0) return fail(ICP4R_E_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(ctx->T.ensure((size_t)k * 9 * 4 * 2));
    float* d = static_cast<float*>(ctx->T.p);
    HIP_TRY(hipMemcpyAsync(d, sigma, (size_t)k * 36, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(launch_rot_f32(d, d + 9 * (size_t)k, k, ctx->stream));
    HIP_TRY(hipMemcpyAsync(R, d + 9 * (size_t)k, (size_t)k * 36, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return ICP4R_OK;
}

}  // extern "C"
