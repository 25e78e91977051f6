// icp4r_host.hpp — host-side pieces shared by the C-ABI translation units (icp4r_capi.cpp,
// icp4r_map.cpp): error reporting, device buffers and the context.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "icp4r/icp4r.h"

namespace icp4r_host {

// Records a printf-style message for icp4r_last_error() (thread-local) and returns `code`.
int fail(int code, const char* fmt, ...);

#define HIP_TRY(expr)                                                                                 \
    do {                                                                                              \
        hipError_t _e = (expr);                                                                       \
        if (_e != hipSuccess)                                                                         \
            return ::icp4r_host::fail(ICP4R_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e),    \
                                      __FILE__, __LINE__);                                            \
    } while (0)

// Grow-only device allocation.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
            cap = 0;
        }
        size_t want = bytes < 256 ? 256 : bytes;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// roctx, loaded at first use (dlopen of librocprofiler-sdk-roctx.so.1): the deployed library needs no
// profiler SDK; without it the ranges are no-ops.
struct RoctxApi {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
};
const RoctxApi& roctx();

// A roctx range over a host scope (SURVEY.md §5 "Tracing"): the entry points and every ICP pass show
// up as named ranges in `rocprofv3 --marker-trace` beside the kernels they launched.  Without a
// profiler attached a push / pop is a few tens of ns.
struct Range {
    explicit Range(const char* name) {
        if (roctx().push) roctx().push(name);
    }
    ~Range() {
        if (roctx().pop) roctx().pop();
    }
    Range(const Range&) = delete;
    Range& operator=(const Range&) = delete;
};

struct EventPair {
    hipEvent_t start = nullptr, stop = nullptr;
};

// Validates a host cloud argument (count, pointer, stride).
int check_cloud(const float* c, int64_t n, int32_t stride, const char* what);

// Repacks n host points of `stride_bytes` into float4 (x, y, z, 4th float or 0).
void pack_host(const float* c, int64_t n, int32_t stride_bytes, std::vector<float>& out);

}  // namespace icp4r_host

struct icp4r_comm;
namespace icp4r_host {
// icp4r_destroy: the context is gone; the communicator keeps working on explicit streams only
void comm_detach(icp4r_comm* c);
}  // namespace icp4r_host

struct icp4r_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // run_pairs' pair groups 1.. run on their own streams, joined back into the launch stream
    hipStream_t aux_stream[3] = {};  // icp4r::kMaxGroups (static_assert in icp4r_capi.cpp)
    hipEvent_t fork_ev[3] = {};
    // staging for the host-buffer entry points
    icp4r_host::DevBuf src, tgt, src_off, src_n, tgt_off, tgt_n, guess, aligned, results, T;
    // batch workspace
    icp4r_host::DevBuf X, nn_key, state, tsort, tinv, tbox, sbox, sperm, corr, ticks, nn_lu, nn_t, kdn, sq, sm, qv, qm, need,
        miss_cnt, plist, plist_n, owork, mo_hist, mo_rep;  // nn_lu holds U (float) per source point
    int ncu = 256;  // compute units of the device (persistent launches)
    bool kernel_timing = false;  // per-kernel events (icp4r_set_kernel_timing)
    // plan options (icp4r_set_plan_option; icp4r_pipe::PlanOpt): values, and which are set
    int32_t plan_val[64] = {};  // (indexed by the plan option enum; kNumPlanOpts <= 64)
    uint64_t plan_set = 0;
    // RCCL communicators created on this context (icp4r_multi.cpp): detached by icp4r_destroy
    std::vector<icp4r_comm*> comms;
    // HIP events on the launch stream: the dominant NN kernel (the batched search, or the whole NN
    // launch of the other plans), the cache-test kernel, the update kernel, whole registrations
    std::vector<icp4r_host::EventPair> nn_events, test_events, upd_events, batch_events;
    size_t nn_used = 0, test_used = 0, upd_used = 0, batch_used = 0;
    icp4r_host::DevBuf evals;  // per-wave counter slots (kCountSlots x kCountStride u64), summed by the host
    // radar ego velocity (icp4r_ego.cpp): staging and workspace
    icp4r_host::DevBuf ego_rec, ego_off, ego_cnt, ego_feat, ego_pd, ego_scores, ego_res, ego_mask, ego_xyzi;
    // generalized ICP (icp4r_gicp.cpp): per-pair LM state, covariances, Mahalanobis, active count
    icp4r_host::DevBuf gicp_gs, gicp_cov_src, gicp_cov_tgt, gicp_mah, gicp_active, gicp_part;
    int64_t* gicp_hflag = nullptr;  // pinned host slots the active-pair checks write (hipHostMalloc):
                                    // (check sequence << 32) | active count
    uint32_t gicp_seq = 0;          // the last active-pair check's sequence number (grows across calls)
    icp4r_host::DevBuf gicp_sidx;   // the source's own index (its k-NN covariances, beside the target's)
    hipEvent_t gicp_fork = nullptr, gicp_join = nullptr;
    std::vector<icp4r_host::EventPair> gicp_events;  // covariance launches (the iterations time as UPDATE)
    size_t gicp_used = 0;
};
