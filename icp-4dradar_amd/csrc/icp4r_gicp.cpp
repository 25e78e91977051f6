// icp4r_gicp.cpp — C ABI of the generalized ICP (include/icp4r/icp4r_gicp.h).
//
// FastGICPSingleThread::align (reference: src/radar_odometry.cpp:398-411) as one stream-ordered
// launch sequence per batch, on the ICP core's device machinery:
//
//   init_kernel + gicp_init        validate, X := guess * src, x0 := guess, lambda := -1
//   covariances x 2                source and target (calculate_covariances): k-NN over each cloud's
//                                  Morton index (pruned plans; the target's stays for the NN passes)
//                                  or brute force
//   repeat                         NN pass (exact 1-NN of X in the target) + the iteration's three
//                                  kernels over slices of the source (Mahalanobis and H / g, the last
//                                  slice solving the LM trials; the trials' errors, the last slice
//                                  deciding x0; X := float(x0) src);
//                                  every 4 iterations the host reads how many pairs still iterate
//   fitness_prep + NN + finish     getFitnessScore and the results, as the ICP path
//
// No CPU fallback: every entry fails with ICP4R_E_HIP if the device path cannot run.
#include <float.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <sched.h>
#include <string.h>

#include <vector>

#include "icp4r/icp4r_gicp.h"
#include "icp4r_batch.hpp"
#include "icp4r_host.hpp"
#include "icp4r_internal.hpp"

using namespace icp4r;
using icp4r_host::DevBuf;
using icp4r_host::EventPair;
using icp4r_host::fail;

namespace {

// Iterations between the active-pair checks. A check's count lands in pinned host memory and the host
// reads it only after queueing the next run of iterations (one check of lookahead): the device never
// waits for the host, and at most one run of iterations (early-exit launches) follows the last one.
// (Every 4 with a blocking read had left the device idle ~37 µs per check on the map call.)
constexpr int kActiveCheck = 2;

// The count check `seq` wrote into the pinned slot, once it has; an error if the stream drained without
// it.  A value with another sequence number is a stale one — an earlier call's check still in flight
// when this call reset the slot (the device API returns before its queued work has run) — and is
// waited past.  The loop yields the core between polls.
int wait_active(volatile int64_t* slot, uint32_t seq, hipStream_t st, int32_t* out) {
    auto mine = [&](int64_t v) { return v != -1 && (uint32_t)((uint64_t)v >> 32) == seq; };
    for (;;) {
        const int64_t v = __atomic_load_n(slot, __ATOMIC_ACQUIRE);
        if (mine(v)) {
            *out = (int32_t)(uint32_t)v;
            return ICP4R_OK;
        }
        const hipError_t q = hipStreamQuery(st);
        if (q == hipSuccess) {
            const int64_t v2 = __atomic_load_n(slot, __ATOMIC_ACQUIRE);
            if (!mine(v2)) return fail(ICP4R_E_HIP, "GICP active-pair check %u not written", seq);
            *out = (int32_t)(uint32_t)v2;
            return ICP4R_OK;
        }
        if (q != hipErrorNotReady) return fail(ICP4R_E_HIP, "hipStreamQuery: %s", hipGetErrorString(q));
        sched_yield();
    }
}

int check_params(const icp4r_gicp_params* p) {
    if (p->k_correspondences < 1 || p->k_correspondences > 32)
        return fail(ICP4R_E_INVALID, "k_correspondences %d outside [1, 32]", p->k_correspondences);
    if (p->max_iterations < 0) return fail(ICP4R_E_INVALID, "max_iterations < 0");
    if (p->lm_max_iterations < 0) return fail(ICP4R_E_INVALID, "lm_max_iterations < 0");
    if (p->regularization < ICP4R_GICP_REG_NONE || p->regularization > ICP4R_GICP_REG_FROBENIUS)
        return fail(ICP4R_E_INVALID, "unknown regularization %d", p->regularization);
    if (!(p->rotation_epsilon > 0) || !(p->transformation_epsilon > 0))
        return fail(ICP4R_E_INVALID, "convergence epsilons must be > 0");
    if (!(p->max_correspondence_distance > 0)) return fail(ICP4R_E_INVALID, "max_correspondence_distance must be > 0");
    return ICP4R_OK;
}

// Brute force or pruned k-NN for the covariances: brute force where the plan does not prune, or with
// plan option gicp_cov_brute = 1 (A/B and the equality test). (Brute force by default for small
// grids measured slower even for a single 8k scan: the map call 1.27 -> 1.36 ms with its source by
// brute force, an 8k pair at k = 20 0.96 -> 2.07 ms — every candidate ran the insertion chain in
// some lane of the wave.)
bool cov_brute(int opt_val, const icp4r_pipe::Plan& pl) { return !pl.pruned || opt_val == 1; }

// k-NN covariances of the clouds (cloud, off, cnt) of npairs pairs: brute force, or pruned over an
// index of each cloud (index_kernel with the cloud as its target; w's index buffers must fit max_n
// points).
// is_tgt: the cloud is the pairs' target, whose boxes init_kernel found (w.tbb): its index is the one
// the NN passes search, on the plan's strides (the multi-workgroup Morton sort where the plan has it).
// Otherwise (the source) the index is built on strides of the cloud's own size (the in-LDS kd build
// for up to 8192 points, not a Morton sort refined chunk by chunk on the target's strides).
int cov_pass(const icp4r_pipe::Plan& pl, const PairArgs& a, const WorkArgs& w, const float4* cloud, const int64_t* off,
             const int32_t* cnt, int npairs, int max_n, int64_t stride, int k, int reg, double* out, hipStream_t st,
             bool brute, bool is_tgt, int lanes) {
    if (!brute) {
        PairArgs ai = a;
        ai.tgt = cloud;
        ai.tgt_off = off;
        ai.tgt_n = cnt;
        WorkArgs wi = w;
        if (!is_tgt) {
            wi.tbb = nullptr;  // (init_kernel's target boxes: the index finds the cloud's own)
            wi.mo_hist = nullptr;
            wi.mo_rep = nullptr;
            const int64_t span = (int64_t)w.leaf * kSuper;
            const int64_t ts = ((max_n > 0 ? max_n : 1) + span - 1) / span * span;
            if (ts < w.t_stride) {
                wi.t_stride = ts;
                wi.b_stride = ts / w.leaf;
                wi.sb_stride = wi.b_stride / kSuper;
            }
        }
        HIP_TRY(launch_index(ai, wi, npairs, st));
        HIP_TRY(launch_gicp_knn_cov(cloud, off, cnt, wi, npairs, max_n, stride, k, reg, out, lanes, st));
    } else {
        HIP_TRY(launch_gicp_cov(cloud, off, cnt, npairs, max_n, stride, k, reg, out, lanes, st));
    }
    return ICP4R_OK;
}

// The registration of a device-resident batch (pointers in `a`), results into a.results.
int run_gicp(icp4r_ctx* ctx, const PairArgs& a, int npairs, int max_n, int max_m, const icp4r_gicp_params& gp,
             hipStream_t st) {
    using namespace icp4r_pipe;
    if (npairs <= 0) return ICP4R_OK;
    const int mn = max_n > 0 ? max_n : 1;
    const int mm = max_m > 0 ? max_m : 1;
    // pruned plans index the source too (its k-NN covariances): the index strides fit both clouds,
    // and the batched search, which stages t_stride targets, only runs when those fit its LDS
    const int idx_both = max_n > max_m ? max_n : max_m;
    Plan pl = make_plan(ctx, npairs, mn, max_m, ICP4R_NN_AUTO, idx_both <= kLdsMaxTargets);
    pl.cache = false;  // the iteration kernels move X without maintaining the cached-neighbour bounds
    WorkArgs w;
    int rc;
    const int idx_m = pl.pruned ? idx_both : max_m;
    if ((rc = setup_work(ctx, pl, npairs, max_n, idx_m, false, st, w))) return rc;
    const int64_t xs = w.x_stride;
    const int64_t ts = mm;
    HIP_TRY(ctx->gicp_gs.ensure((size_t)npairs * sizeof(GicpState)));
    HIP_TRY(ctx->gicp_cov_src.ensure((size_t)npairs * xs * 6 * sizeof(double)));
    HIP_TRY(ctx->gicp_cov_tgt.ensure((size_t)npairs * ts * 6 * sizeof(double)));
    HIP_TRY(ctx->gicp_mah.ensure((size_t)npairs * xs * 6 * sizeof(double)));
    HIP_TRY(ctx->gicp_active.ensure(sizeof(int32_t)));
    const size_t lin_b = (size_t)npairs * kGicpMaxSlices * kGicpSys * sizeof(double);
    const size_t err_b = (size_t)npairs * kGicpMaxSlices * kGicpSpec * sizeof(double);
    const size_t cand_b = (size_t)npairs * sizeof(GicpCand);
    HIP_TRY(ctx->gicp_part.ensure(lin_b + err_b + cand_b + (size_t)npairs * sizeof(int32_t)));
    GicpArgs g;
    g.gs = static_cast<GicpState*>(ctx->gicp_gs.p);
    g.cov_src = static_cast<const double*>(ctx->gicp_cov_src.p);
    g.cov_tgt = static_cast<const double*>(ctx->gicp_cov_tgt.p);
    g.mah = static_cast<double*>(ctx->gicp_mah.p);
    g.part_lin = static_cast<double*>(ctx->gicp_part.p);
    g.part_err = g.part_lin + lin_b / sizeof(double);
    g.cand = reinterpret_cast<GicpCand*>(g.part_err + err_b / sizeof(double));
    g.cnt = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(g.cand) + cand_b);
    g.t_stride = ts;
    const float thr = (float)fmin(gp.max_correspondence_distance, (double)FLT_MAX);
    g.max_d2 = (double)(thr * thr);  // corr_dist_threshold_ * corr_dist_threshold_ (float)
    g.rot_eps = gp.rotation_epsilon;
    g.trans_eps = gp.transformation_epsilon;
    g.lm_init = gp.lm_init_lambda_factor;
    g.lm_max_iterations = gp.lm_max_iterations;
    g.max_iterations = gp.max_iterations;
    // (plan option gicp_spec: trials per speculative pass; fewer only for the test that the one-by-one
    // trials decide identically)
    const int spec = opt(ctx, kOptGicpSpec, kGicpSpec);
    g.spec = spec < 0 ? 0 : spec > kGicpSpec ? kGicpSpec : spec;
    // (plan option gicp_grid: how many workgroups share the slices; the sums do not depend on it)
    const int grid = opt(ctx, kOptGicpGrid, kGicpGrid);
    g.grid = grid < 1 ? 1 : grid;

    EventPair* be;
    if ((rc = next_event(ctx->batch_events, ctx->batch_used, &be))) return rc;
    HIP_TRY(hipEventRecord(be->start, st));
    HIP_TRY(launch_init(a, w, npairs, st));
    HIP_TRY(launch_gicp_init(a.guess, g.gs, npairs, st));
    HIP_TRY(hipMemsetAsync(g.cnt, 0, (size_t)npairs * sizeof(int32_t), st));
    // per-stage events only with icp4r_set_kernel_timing (each record between kernels costs device time)
    const bool kev = ctx->kernel_timing;
    EventPair* ce = nullptr;
    if (kev && (rc = next_event(ctx->gicp_events, ctx->gicp_used, &ce))) return rc;
    double* cs = static_cast<double*>(ctx->gicp_cov_src.p);
    double* ct = static_cast<double*>(ctx->gicp_cov_tgt.p);
    const bool brute = cov_brute(opt(ctx, kOptGicpCovBrute, 0), pl);
    const int knn_lanes = opt(ctx, kOptGicpKnnLanes, 0);
    if (kev) HIP_TRY(hipEventRecord(ce->start, st));
    if (!brute) {
        // The source's index on buffers of its own and its k-NN covariances on the aux stream, beside the
        // target's chain (index, refinement, k-NN) on st: both chains are latency-bound on few pairs
        // (the map call: the 8k source's kd build and walk ~120 µs under the submap's ~240).
        hipStream_t aux = ctx->aux_stream[0];
        if (!aux) {
            HIP_TRY(hipStreamCreateWithFlags(&ctx->aux_stream[0], hipStreamNonBlocking));
            aux = ctx->aux_stream[0];
        }
        if (!ctx->gicp_fork) HIP_TRY(hipEventCreateWithFlags(&ctx->gicp_fork, hipEventDisableTiming));
        if (!ctx->gicp_join) HIP_TRY(hipEventCreateWithFlags(&ctx->gicp_join, hipEventDisableTiming));
        WorkArgs ws = w;
        const int64_t span = (int64_t)w.leaf * kSuper;
        ws.t_stride = ((int64_t)mn + span - 1) / span * span;
        ws.b_stride = ws.t_stride / w.leaf;
        ws.sb_stride = ws.b_stride / kSuper;
        ws.tbb = nullptr;  // (init_kernel's are the target's boxes: the build finds the source's own)
        ws.mo_hist = nullptr;
        ws.mo_rep = nullptr;
        ws.kdn = nullptr;  // (no tree for a source order to descend)
        ws.src_by_tgt = 0;
        ws.ticks = nullptr;
        const size_t n_ts = (size_t)npairs * ws.t_stride, n_b = (size_t)npairs * 2 * ws.b_stride,
                     n_sb = (size_t)npairs * 2 * ws.sb_stride, n_q = w.qv ? (size_t)npairs * w.x_stride : 0;
        HIP_TRY(ctx->gicp_sidx.ensure((n_ts + n_b + n_sb + n_q) * sizeof(float4) + n_ts * sizeof(int32_t)));
        float4* sb = static_cast<float4*>(ctx->gicp_sidx.p);
        ws.tsort = sb;
        ws.tbox = sb + n_ts;
        ws.sbox = ws.tbox + n_b;
        ws.qv = w.qv ? ws.sbox + n_sb : nullptr;  // (the kd build's key scratch: the target's is in use)
        ws.tinv = reinterpret_cast<int32_t*>(ws.sbox + n_sb + n_q);
        PairArgs as = a;
        as.tgt = a.src;
        as.tgt_off = a.src_off;
        as.tgt_n = a.src_n;
        HIP_TRY(hipEventRecord(ctx->gicp_fork, st));
        HIP_TRY(hipStreamWaitEvent(aux, ctx->gicp_fork, 0));
        HIP_TRY(launch_index_cloud(as, ws, npairs, aux));
        HIP_TRY(launch_gicp_knn_cov(a.src, a.src_off, a.src_n, ws, npairs, mn, xs, gp.k_correspondences,
                                    gp.regularization, cs, knn_lanes, aux));
        HIP_TRY(hipEventRecord(ctx->gicp_join, aux));
        rc = cov_pass(pl, a, w, a.tgt, a.tgt_off, a.tgt_n, npairs, mm, ts, gp.k_correspondences, gp.regularization,
                      ct, st, brute, true, knn_lanes);
        // joined on every path: a failed target pass must not leave the source's chain (which writes
        // gicp_cov_src and gicp_sidx) running past the call
        const hipError_t je = hipStreamWaitEvent(st, ctx->gicp_join, 0);
        if (rc) return rc;
        HIP_TRY(je);
    } else {
        if ((rc = cov_pass(pl, a, w, a.src, a.src_off, a.src_n, npairs, mn, xs, gp.k_correspondences,
                           gp.regularization, cs, st, brute, false, knn_lanes)))
            return rc;
        if ((rc = cov_pass(pl, a, w, a.tgt, a.tgt_off, a.tgt_n, npairs, mm, ts, gp.k_correspondences,
                           gp.regularization, ct, st, brute, true, knn_lanes)))
            return rc;
    }
    if (pl.pruned && brute) HIP_TRY(launch_index(a, w, npairs, st));
    if (kev) HIP_TRY(hipEventRecord(ce->stop, st));
    int32_t* active = static_cast<int32_t*>(ctx->gicp_active.p);
    if (!ctx->gicp_hflag) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ctx->gicp_hflag), 2 * sizeof(int64_t), hipHostMallocCoherent));
    volatile int64_t* hf = ctx->gicp_hflag;
    int nchk = 0, prev_slot = -1;
    uint32_t prev_seq = 0;
    for (int it = 0; it < gp.max_iterations; ++it) {
        if ((rc = nn_pass(ctx, pl, a, w, npairs, mn, 0, it == 0, st))) return rc;
        EventPair* ue = nullptr;
        if (kev) {
            if ((rc = next_event(ctx->upd_events, ctx->upd_used, &ue))) return rc;
            HIP_TRY(hipEventRecord(ue->start, st));
        }
        HIP_TRY(launch_gicp_iter(a, w, g, npairs, mn, it, st));
        if (kev) HIP_TRY(hipEventRecord(ue->stop, st));
        if ((it + 1) % kActiveCheck == 0 && it + 1 < gp.max_iterations) {
            const int slot = nchk++ & 1;  // (the previous check's slot is the other one; the one before
            hf[slot] = -1;                // was read before that check was queued)
            const uint32_t seq = ++ctx->gicp_seq;
            HIP_TRY(launch_gicp_active(w.state, npairs, active, const_cast<int64_t*>(hf + slot), seq, st));
            if (prev_slot >= 0) {
                int32_t h = 0;
                if ((rc = wait_active(hf + prev_slot, prev_seq, st, &h))) return rc;
                if (h == 0) break;
            }
            prev_slot = slot;
            prev_seq = seq;
        }
    }
    if (a.kp.compute_fitness || a.aligned) HIP_TRY(launch_fitness_prep(a, w, npairs, st));
    if (a.kp.compute_fitness && (rc = nn_pass(ctx, pl, a, w, npairs, mn, 1, 0, st))) return rc;
    HIP_TRY(launch_finish(a, w, npairs, st));
    HIP_TRY(hipEventRecord(be->stop, st));
    return ICP4R_OK;
}

int gicp_kparams(const icp4r_gicp_params& gp, KParams* kp) {
    icp4r_params ip;
    icp4r_params_default(&ip);
    ip.compute_fitness = gp.compute_fitness;
    int rc = icp4r_pipe::make_kparams(&ip, kp);
    if (rc) return rc;
    kp->fit_max_range = DBL_MAX;  // Registration::getFitnessScore() default
    return ICP4R_OK;
}

}  // namespace

extern "C" {

void icp4r_gicp_params_default(icp4r_gicp_params* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->k_correspondences = 20;
    p->max_iterations = 64;
    p->rotation_epsilon = 2e-3;
    p->transformation_epsilon = 5e-4;
    p->max_correspondence_distance = FLT_MAX;
    p->regularization = ICP4R_GICP_REG_PLANE;
    p->lm_max_iterations = 10;
    p->lm_init_lambda_factor = 1e-9;
    p->compute_fitness = 1;
}

int icp4r_gicp_align_batch_device(icp4r_ctx* ctx, const icp4r_batch* b, const icp4r_gicp_params* params,
                                  icp4r_result* results, void* hip_stream) {
    if (!ctx || !b || !results) return fail(ICP4R_E_INVALID, "ctx/batch/results is NULL");
    if (b->npairs < 0) return fail(ICP4R_E_INVALID, "npairs < 0");
    if (b->npairs == 0) return ICP4R_OK;
    if (!b->src || !b->tgt || !b->src_off || !b->src_n || !b->tgt_off || !b->tgt_n)
        return fail(ICP4R_E_INVALID, "batch has a NULL device array");
    if (b->max_src_n < 0 || b->max_tgt_n < 0) return fail(ICP4R_E_INVALID, "negative max sizes");
    icp4r_gicp_params gp;
    if (params) gp = *params;
    else icp4r_gicp_params_default(&gp);
    int rc;
    if ((rc = check_params(&gp))) return rc;
    PairArgs a;
    if ((rc = gicp_kparams(gp, &a.kp))) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    a.src = reinterpret_cast<const float4*>(b->src);
    a.tgt = reinterpret_cast<const float4*>(b->tgt);
    a.src_off = b->src_off;
    a.src_n = b->src_n;
    a.tgt_off = b->tgt_off;
    a.tgt_n = b->tgt_n;
    a.guess = b->guess;
    a.aligned = reinterpret_cast<float4*>(b->aligned);
    a.results = reinterpret_cast<Result*>(results);
    hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->stream;
    return run_gicp(ctx, a, b->npairs, b->max_src_n, b->max_tgt_n, gp, st);
}

int icp4r_gicp_align(icp4r_ctx* ctx, const float* src, int32_t n, int32_t src_stride_bytes, const float* tgt,
                     int32_t m, int32_t tgt_stride_bytes, const float* guess, const icp4r_gicp_params* params,
                     icp4r_result* out, float* aligned_out, int32_t out_stride_bytes) {
    using namespace icp4r_host;
    if (!ctx || !out) return fail(ICP4R_E_INVALID, "ctx/out is NULL");
    int rc;
    if ((rc = check_cloud(src, n, src_stride_bytes, "source"))) return rc;
    if ((rc = check_cloud(tgt, m, tgt_stride_bytes, "target"))) return rc;
    if (aligned_out && (out_stride_bytes < 12 || out_stride_bytes % 4))
        return fail(ICP4R_E_INVALID, "aligned_out stride %d bytes", out_stride_bytes);
    HIP_TRY(hipSetDevice(ctx->device));
    std::vector<float> hs, ht;
    pack_host(src, n, src_stride_bytes, hs);
    pack_host(tgt, m, tgt_stride_bytes, ht);
    const int64_t zero64 = 0;
    HIP_TRY(ctx->src.ensure(hs.size() * sizeof(float) + 16));
    HIP_TRY(ctx->tgt.ensure(ht.size() * sizeof(float) + 16));
    HIP_TRY(ctx->src_off.ensure(16));
    HIP_TRY(ctx->tgt_off.ensure(16));
    HIP_TRY(ctx->src_n.ensure(16));
    HIP_TRY(ctx->tgt_n.ensure(16));
    HIP_TRY(ctx->guess.ensure(16 * sizeof(float)));
    HIP_TRY(ctx->results.ensure(sizeof(icp4r_result)));
    HIP_TRY(ctx->aligned.ensure(hs.size() * sizeof(float) + 16));
    hipStream_t st = ctx->stream;
    if (!hs.empty()) HIP_TRY(hipMemcpyAsync(ctx->src.p, hs.data(), hs.size() * sizeof(float), hipMemcpyHostToDevice, st));
    if (!ht.empty()) HIP_TRY(hipMemcpyAsync(ctx->tgt.p, ht.data(), ht.size() * sizeof(float), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->src_off.p, &zero64, 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->tgt_off.p, &zero64, 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->src_n.p, &n, 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->tgt_n.p, &m, 4, hipMemcpyHostToDevice, st));
    if (guess) HIP_TRY(hipMemcpyAsync(ctx->guess.p, guess, 16 * sizeof(float), hipMemcpyHostToDevice, st));
    icp4r_batch b;
    memset(&b, 0, sizeof(b));
    b.src = static_cast<const float*>(ctx->src.p);
    b.tgt = static_cast<const float*>(ctx->tgt.p);
    b.src_off = static_cast<const int64_t*>(ctx->src_off.p);
    b.tgt_off = static_cast<const int64_t*>(ctx->tgt_off.p);
    b.src_n = static_cast<const int32_t*>(ctx->src_n.p);
    b.tgt_n = static_cast<const int32_t*>(ctx->tgt_n.p);
    b.guess = guess ? static_cast<const float*>(ctx->guess.p) : nullptr;
    b.aligned = aligned_out ? static_cast<float*>(ctx->aligned.p) : nullptr;
    b.npairs = 1;
    b.max_src_n = n;
    b.max_tgt_n = m;
    if ((rc = icp4r_gicp_align_batch_device(ctx, &b, params, static_cast<icp4r_result*>(ctx->results.p), st))) return rc;
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
        const char* what = out->status == ICP4R_E_EMPTY ? "No input target dataset was given!"
                           : out->status == ICP4R_E_NONFINITE ? "non-finite coordinate in an input cloud"
                                                              : "registration failed";
        return fail(out->status, "[icp4r::FastGICP::computeTransformation] %s", what);
    }
    return ICP4R_OK;
}

int icp4r_gicp_covariances(icp4r_ctx* ctx, const float* cloud, int32_t n, int32_t stride_bytes, int32_t k,
                           int32_t regularization, double* cov_out) {
    using namespace icp4r_host;
    if (!ctx || (!cov_out && n > 0)) return fail(ICP4R_E_INVALID, "ctx/cov_out is NULL");
    if (k < 1 || k > 32) return fail(ICP4R_E_INVALID, "k %d outside [1, 32]", k);
    if (regularization < ICP4R_GICP_REG_NONE || regularization > ICP4R_GICP_REG_FROBENIUS)
        return fail(ICP4R_E_INVALID, "unknown regularization %d", regularization);
    int rc;
    if ((rc = check_cloud(cloud, n, stride_bytes, "cloud"))) return rc;
    if (n == 0) return ICP4R_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    std::vector<float> hc;
    pack_host(cloud, n, stride_bytes, hc);
    const int64_t zero64 = 0;
    hipStream_t st = ctx->stream;
    HIP_TRY(ctx->src.ensure(hc.size() * sizeof(float)));
    HIP_TRY(ctx->src_off.ensure(16));
    HIP_TRY(ctx->src_n.ensure(16));
    HIP_TRY(ctx->gicp_cov_src.ensure((size_t)n * 6 * sizeof(double)));
    HIP_TRY(hipMemcpyAsync(ctx->src.p, hc.data(), hc.size() * sizeof(float), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->src_off.p, &zero64, 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->src_n.p, &n, 4, hipMemcpyHostToDevice, st));
    PairArgs a;
    memset(&a, 0, sizeof(a));
    a.src = a.tgt = static_cast<const float4*>(ctx->src.p);
    a.src_off = a.tgt_off = static_cast<const int64_t*>(ctx->src_off.p);
    a.src_n = a.tgt_n = static_cast<const int32_t*>(ctx->src_n.p);
    const icp4r_pipe::Plan pl = icp4r_pipe::make_plan(ctx, 1, n, n, ICP4R_NN_AUTO);
    WorkArgs w;
    if ((rc = icp4r_pipe::setup_work(ctx, pl, 1, n, n, false, st, w))) return rc;
    HIP_TRY(hipMemsetAsync(w.state, 0, sizeof(PairState), st));  // phase = active: index_kernel runs
    if ((rc = cov_pass(pl, a, w, a.src, a.src_off, a.src_n, 1, n, n, k, regularization,
                       static_cast<double*>(ctx->gicp_cov_src.p), st,
                       cov_brute(icp4r_pipe::opt(ctx, icp4r_pipe::kOptGicpCovBrute, 0), pl), false,
                       icp4r_pipe::opt(ctx, icp4r_pipe::kOptGicpKnnLanes, 0))))
        return rc;
    std::vector<double> h6((size_t)n * 6);
    HIP_TRY(hipMemcpyAsync(h6.data(), ctx->gicp_cov_src.p, h6.size() * sizeof(double), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    static const int idx[9] = {0, 1, 2, 1, 3, 4, 2, 4, 5};
    for (int32_t i = 0; i < n; ++i)
        for (int t = 0; t < 9; ++t) cov_out[(size_t)i * 9 + t] = h6[(size_t)i * 6 + idx[t]];
    return ICP4R_OK;
}

}  // extern "C"
