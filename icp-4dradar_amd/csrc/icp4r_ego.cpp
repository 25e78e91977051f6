// icp4r_ego.cpp — C ABI of the radar ego-velocity estimator (include/icp4r/icp4r_ego.h).
//
// Host entry points for the reference node's per-frame parse / fitSineRansac / static split /
// least squares (src/iterative_closest_point.cpp:354-431) over the kernels of icp4r_ego.hip.  No CPU
// fallback: every entry fails with ICP4R_E_HIP if the device path cannot run.
#include <hip/hip_runtime.h>
#include <string.h>

#include <vector>

#include "icp4r/icp4r_ego.h"
#include "icp4r_host.hpp"
#include "icp4r_internal.hpp"

using icp4r::EgoArgs;
using icp4r_host::fail;

namespace {

int check_params(const icp4r_ego_params* p) {
    if (!p) return ICP4R_OK;
    if (!(p->sigma > 0)) return fail(ICP4R_E_INVALID, "sigma must be > 0");
    if (p->dynamic_threshold != p->dynamic_threshold) return fail(ICP4R_E_INVALID, "dynamic_threshold is NaN");
    return ICP4R_OK;
}

int hyps_for(const icp4r_ego_params& p, int32_t max_n) { return p.iterations > 0 ? p.iterations : (int)(max_n * 0.2); }

// Workspace for nscans scans of at most max_n points; fills the EgoArgs buffers.
int setup(icp4r_ctx* ctx, const icp4r_ego_params& p, int32_t nscans, int32_t max_n, EgoArgs& e) {
    const int64_t stride = max_n > 0 ? max_n : 1;
    const int32_t H = hyps_for(p, max_n);
    HIP_TRY(ctx->ego_feat.ensure((size_t)nscans * stride * sizeof(float4)));
    HIP_TRY(ctx->ego_pd.ensure((size_t)nscans * stride * sizeof(double4)));
    HIP_TRY(ctx->ego_scores.ensure((size_t)nscans * (H > 0 ? H : 1) * sizeof(int32_t)));
    e.stride = stride;
    e.feat = static_cast<float4*>(ctx->ego_feat.p);
    e.pd = static_cast<double4*>(ctx->ego_pd.p);
    e.scores = static_cast<int32_t*>(ctx->ego_scores.p);
    e.max_h = H > 0 ? H : 0;
    e.iterations = p.iterations;
    e.sigma = p.sigma;
    e.dyn = p.dynamic_threshold;
    e.seed = p.seed;
    return ICP4R_OK;
}

// Upload one host scan (n records) with off = 0, cnt = n.
int upload_one(icp4r_ctx* ctx, const float* records, int32_t n, EgoArgs& e) {
    const int64_t zero = 0;
    HIP_TRY(ctx->ego_rec.ensure((size_t)(n > 0 ? n : 1) * 5 * sizeof(float)));
    HIP_TRY(ctx->ego_off.ensure(sizeof(int64_t)));
    HIP_TRY(ctx->ego_cnt.ensure(sizeof(int32_t)));
    if (n > 0)
        HIP_TRY(hipMemcpyAsync(ctx->ego_rec.p, records, (size_t)n * 5 * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->ego_off.p, &zero, sizeof(zero), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->ego_cnt.p, &n, sizeof(n), hipMemcpyHostToDevice, ctx->stream));
    e.rec = static_cast<const float*>(ctx->ego_rec.p);
    e.off = static_cast<const int64_t*>(ctx->ego_off.p);
    e.cnt = static_cast<const int32_t*>(ctx->ego_cnt.p);
    return ICP4R_OK;
}

}  // namespace

extern "C" {

void icp4r_ego_params_default(icp4r_ego_params* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->iterations = 0;           // (int)(PointsNum * 0.2) — iterative_closest_point.cpp:389
    p->sigma = 0.5;              // fitSineRansac's default — :89
    p->dynamic_threshold = 0.2;  // :396
    p->seed = 0x1CB4D12A5EEDull;
}

int icp4r_radar_features(icp4r_ctx* ctx, const float* records, int32_t n, float* xyzi_out, float* feat_out) {
    if (!ctx) return fail(ICP4R_E_INVALID, "ctx is NULL");
    if (n < 0 || (n > 0 && !records)) return fail(ICP4R_E_INVALID, "bad scan (n = %d)", n);
    if (n == 0) return ICP4R_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    icp4r_ego_params p;
    icp4r_ego_params_default(&p);
    EgoArgs e;
    memset(&e, 0, sizeof(e));
    int rc;
    if ((rc = setup(ctx, p, 1, n, e)) || (rc = upload_one(ctx, records, n, e))) return rc;
    float4* xyzi = nullptr;
    if (xyzi_out) {
        HIP_TRY(ctx->ego_xyzi.ensure((size_t)n * sizeof(float4)));
        xyzi = static_cast<float4*>(ctx->ego_xyzi.p);
    }
    HIP_TRY(icp4r::launch_ego_features(e, 1, n, xyzi, ctx->stream));
    if (feat_out) HIP_TRY(hipMemcpyAsync(feat_out, e.feat, (size_t)n * sizeof(float4), hipMemcpyDeviceToHost, ctx->stream));
    if (xyzi_out) HIP_TRY(hipMemcpyAsync(xyzi_out, xyzi, (size_t)n * sizeof(float4), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return ICP4R_OK;
}

int icp4r_ego_velocity(icp4r_ctx* ctx, const float* records, int32_t n, const icp4r_ego_params* params,
                       icp4r_ego_result* out, uint8_t* static_mask_out, double* scores_out) {
    if (!ctx || !out) return fail(ICP4R_E_INVALID, "NULL argument");
    if (n < 0 || (n > 0 && !records)) return fail(ICP4R_E_INVALID, "bad scan (n = %d)", n);
    int rc;
    if ((rc = check_params(params))) return rc;
    icp4r_ego_params p;
    icp4r_ego_params_default(&p);
    if (params) p = *params;
    HIP_TRY(hipSetDevice(ctx->device));
    EgoArgs e;
    memset(&e, 0, sizeof(e));
    if ((rc = setup(ctx, p, 1, n, e)) || (rc = upload_one(ctx, records, n, e))) return rc;
    HIP_TRY(ctx->ego_res.ensure(sizeof(icp4r_ego_result)));
    e.results = static_cast<icp4r_ego_result*>(ctx->ego_res.p);
    if (static_mask_out && n > 0) {
        HIP_TRY(ctx->ego_mask.ensure((size_t)n));
        e.mask = static_cast<uint8_t*>(ctx->ego_mask.p);
    }
    HIP_TRY(icp4r::launch_ego(e, 1, n > 0 ? n : 1, nullptr, ctx->stream));
    HIP_TRY(hipMemcpyAsync(out, e.results, sizeof(*out), hipMemcpyDeviceToHost, ctx->stream));
    if (e.mask) HIP_TRY(hipMemcpyAsync(static_mask_out, e.mask, (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    std::vector<int32_t> sc;
    const int H = n > 0 ? hyps_for(p, n) : 0;
    if (scores_out && H > 0) {
        sc.resize((size_t)H);
        HIP_TRY(hipMemcpyAsync(sc.data(), e.scores, (size_t)H * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    for (int h = 0; h < (int)sc.size(); ++h) scores_out[h] = (double)sc[(size_t)h];
    if (n == 0) return fail(ICP4R_E_EMPTY, "empty scan");
    return ICP4R_OK;
}

int icp4r_ego_velocity_batch_device(icp4r_ctx* ctx, const float* records, const int64_t* off, const int32_t* cnt,
                                    int32_t nscans, int32_t max_n, const icp4r_ego_params* params,
                                    icp4r_ego_result* results, uint8_t* static_mask, void* hip_stream) {
    if (!ctx || !results || nscans < 0 || max_n < 0) return fail(ICP4R_E_INVALID, "bad arguments");
    if (nscans == 0) return ICP4R_OK;
    if (!records || !off || !cnt) return fail(ICP4R_E_INVALID, "NULL device array");
    int rc;
    if ((rc = check_params(params))) return rc;
    icp4r_ego_params p;
    icp4r_ego_params_default(&p);
    if (params) p = *params;
    HIP_TRY(hipSetDevice(ctx->device));
    EgoArgs e;
    memset(&e, 0, sizeof(e));
    if ((rc = setup(ctx, p, nscans, max_n, e))) return rc;
    e.rec = records;
    e.off = off;
    e.cnt = cnt;
    e.results = results;
    e.mask = static_mask;
    hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->stream;
    HIP_TRY(icp4r::launch_ego(e, nscans, max_n > 0 ? max_n : 1, nullptr, st));
    return ICP4R_OK;
}

}  // extern "C"
