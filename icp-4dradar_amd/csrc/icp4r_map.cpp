// icp4r_map.cpp — C ABI of the scan-to-map store (include/icp4r/icp4r_map.h).
//
// Host-side mirror of the reference's ikd-Tree as radar_odometry.cpp uses it (:92, :347-348,
// :382-396): an append-only float4 store in HBM that grows by doubling, and Sector_Search as a
// device stream compaction (icp4r_map.hip).  No CPU fallback: every entry fails with
// ICP4R_E_HIP if the device path cannot run.
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <vector>

#include "icp4r/icp4r_map.h"
#include "icp4r_host.hpp"
#include "icp4r_internal.hpp"

using icp4r_host::check_cloud;
using icp4r_host::DevBuf;
using icp4r_host::EventPair;
using icp4r_host::fail;
using icp4r_host::pack_host;

struct icp4r_map {
    icp4r_ctx* ctx = nullptr;
    float4* pts = nullptr;  // [cap] insertion order
    int64_t n = 0, cap = 0;
    DevBuf staging, counts, offsets, total, out;
    std::vector<EventPair> events;
    size_t used = 0;
};

namespace {

// Grow the store to hold `need` points, keeping the first map->n (doubling: amortised O(1) append).
int grow(icp4r_map* m, int64_t need) {
    if (need <= m->cap) return ICP4R_OK;
    int64_t cap = m->cap > 0 ? m->cap : (int64_t)1 << 16;
    while (cap < need) cap *= 2;
    float4* p = nullptr;
    HIP_TRY(hipMalloc(&p, (size_t)cap * sizeof(float4)));
    if (m->n > 0) {
        hipError_t e = hipMemcpyAsync(p, m->pts, (size_t)m->n * sizeof(float4), hipMemcpyDeviceToDevice, m->ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(m->ctx->stream);
        if (e != hipSuccess) {
            (void)hipFree(p);
            return fail(ICP4R_E_HIP, "map grow: %s", hipGetErrorString(e));
        }
    }
    if (m->pts) HIP_TRY(hipFree(m->pts));
    m->pts = p;
    m->cap = cap;
    return ICP4R_OK;
}

// Upload n host points (any stride) as float4 into the staging buffer.
int stage(icp4r_map* m, const float* pts, int64_t n, int32_t stride, std::vector<float>& h) {
    pack_host(pts, n, stride, h);
    HIP_TRY(m->staging.ensure((size_t)(n > 0 ? n : 1) * sizeof(float4)));
    if (n > 0) HIP_TRY(hipMemcpyAsync(m->staging.p, h.data(), (size_t)n * sizeof(float4), hipMemcpyHostToDevice, m->ctx->stream));
    return ICP4R_OK;
}

int sector_launch(icp4r_map* m, const float* center, float radius, float heading, float4* out, int32_t* count,
                  hipStream_t st) {
    if (!center) return fail(ICP4R_E_INVALID, "center is NULL");
    if (!(radius >= 0.0f)) return fail(ICP4R_E_INVALID, "radius must be >= 0");
    const int64_t nblk = icp4r::sector_blocks(m->n);
    HIP_TRY(m->counts.ensure((size_t)(nblk > 0 ? nblk : 1) * sizeof(int32_t)));
    HIP_TRY(m->offsets.ensure((size_t)(nblk > 0 ? nblk : 1) * sizeof(int32_t)));
    icp4r::SectorArgs a;
    a.cx = center[0];
    a.cy = center[1];
    a.cz = center[2];
    a.radius = radius;
    a.heading = heading;
    if (m->used == m->events.size()) {
        EventPair e;
        HIP_TRY(hipEventCreate(&e.start));
        HIP_TRY(hipEventCreate(&e.stop));
        m->events.push_back(e);
    }
    EventPair& ev = m->events[m->used++];
    HIP_TRY(hipEventRecord(ev.start, st));
    HIP_TRY(icp4r::launch_sector(m->pts, m->n, a, static_cast<int32_t*>(m->counts.p),
                                 static_cast<int32_t*>(m->offsets.p), count, out, st));
    HIP_TRY(hipEventRecord(ev.stop, st));
    return ICP4R_OK;
}

}  // namespace

extern "C" {

int icp4r_map_create(icp4r_ctx* ctx, icp4r_map** out) {
    if (!ctx || !out) return fail(ICP4R_E_INVALID, "ctx/out is NULL");
    *out = nullptr;
    if (ctx->device < 0) return fail(ICP4R_E_INVALID, "icp4r_map_create: a context without a device");
    icp4r_map* m = new icp4r_map();
    m->ctx = ctx;
    *out = m;
    return ICP4R_OK;
}

int icp4r_map_destroy(icp4r_map* m) {
    if (!m) return ICP4R_OK;
    (void)hipSetDevice(m->ctx->device);
    (void)hipStreamSynchronize(m->ctx->stream);
    if (m->pts) (void)hipFree(m->pts);
    for (DevBuf* b : {&m->staging, &m->counts, &m->offsets, &m->total, &m->out}) b->release();
    for (auto& e : m->events) {
        (void)hipEventDestroy(e.start);
        (void)hipEventDestroy(e.stop);
    }
    delete m;
    return ICP4R_OK;
}

int icp4r_map_add_points(icp4r_map* m, const float* pts, int64_t n, int32_t stride_bytes, int32_t downsample_on) {
    if (!m) return fail(ICP4R_E_INVALID, "map is NULL");
    if (downsample_on)
        return fail(ICP4R_E_INVALID, "Add_Points with downsample_on is not on this path (radar_odometry.cpp:390 passes false)");
    int rc;
    if ((rc = check_cloud(pts, n, stride_bytes, "points"))) return rc;
    if (n == 0) return ICP4R_OK;
    HIP_TRY(hipSetDevice(m->ctx->device));
    if ((rc = grow(m, m->n + n))) return rc;
    std::vector<float> h;
    pack_host(pts, n, stride_bytes, h);
    HIP_TRY(hipMemcpyAsync(m->pts + m->n, h.data(), (size_t)n * sizeof(float4), hipMemcpyHostToDevice, m->ctx->stream));
    HIP_TRY(hipStreamSynchronize(m->ctx->stream));  // h goes out of scope
    m->n += n;
    return ICP4R_OK;
}

int icp4r_map_build(icp4r_map* m, const float* pts, int64_t n, int32_t stride_bytes) {
    if (!m) return fail(ICP4R_E_INVALID, "map is NULL");
    int rc;
    if ((rc = check_cloud(pts, n, stride_bytes, "points"))) return rc;
    m->n = 0;  // KD_TREE::Build replaces the tree
    return icp4r_map_add_points(m, pts, n, stride_bytes, 0);
}

int icp4r_map_add_scan(icp4r_map* m, const float* scan, int64_t n, int32_t stride_bytes, const double* R,
                       const double* t, float* world_out) {
    if (!m || !R || !t) return fail(ICP4R_E_INVALID, "map/R/t is NULL");
    int rc;
    if ((rc = check_cloud(scan, n, stride_bytes, "scan"))) return rc;
    if (n == 0) return ICP4R_OK;
    HIP_TRY(hipSetDevice(m->ctx->device));
    if ((rc = grow(m, m->n + n))) return rc;
    std::vector<float> h;
    if ((rc = stage(m, scan, n, stride_bytes, h))) return rc;
    icp4r::Mat3x4d M;
    memcpy(M.R, R, sizeof(M.R));
    memcpy(M.t, t, sizeof(M.t));
    HIP_TRY(icp4r::launch_associate(static_cast<const float4*>(m->staging.p), n, M, m->pts + m->n, m->ctx->stream));
    if (world_out)
        HIP_TRY(hipMemcpyAsync(world_out, m->pts + m->n, (size_t)n * sizeof(float4), hipMemcpyDeviceToHost, m->ctx->stream));
    HIP_TRY(hipStreamSynchronize(m->ctx->stream));
    m->n += n;
    return ICP4R_OK;
}

int icp4r_map_size(const icp4r_map* m, int64_t* n) {
    if (!m || !n) return fail(ICP4R_E_INVALID, "NULL argument");
    *n = m->n;
    return ICP4R_OK;
}

int icp4r_map_sector_search(icp4r_map* m, const float* center, float radius, float heading_deg, float* out,
                            int64_t out_cap, int64_t* out_n) {
    if (!m || !out_n || (out_cap > 0 && !out)) return fail(ICP4R_E_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(m->ctx->device));
    hipStream_t st = m->ctx->stream;
    HIP_TRY(m->out.ensure((size_t)(m->n > 0 ? m->n : 1) * sizeof(float4)));
    HIP_TRY(m->total.ensure(sizeof(int32_t)));
    int rc;
    if ((rc = sector_launch(m, center, radius, heading_deg, static_cast<float4*>(m->out.p),
                            static_cast<int32_t*>(m->total.p), st)))
        return rc;
    int32_t cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, m->total.p, sizeof(cnt), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    *out_n = cnt;
    if (cnt > out_cap) return fail(ICP4R_E_TOO_LARGE, "sector search kept %d points, out_cap %lld", cnt, (long long)out_cap);
    if (cnt > 0) {
        HIP_TRY(hipMemcpyAsync(out, m->out.p, (size_t)cnt * sizeof(float4), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    return ICP4R_OK;
}

int icp4r_map_sector_search_device(icp4r_map* m, const float* center, float radius, float heading_deg, float* d_out,
                                   int32_t* d_count, void* hip_stream) {
    if (!m || !d_out || !d_count) return fail(ICP4R_E_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(m->ctx->device));
    hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : m->ctx->stream;
    return sector_launch(m, center, radius, heading_deg, reinterpret_cast<float4*>(d_out), d_count, st);
}

int icp4r_map_points_device(icp4r_map* m, const float** d_points, int64_t* n) {
    if (!m || !d_points || !n) return fail(ICP4R_E_INVALID, "NULL argument");
    *d_points = reinterpret_cast<const float*>(m->pts);
    *n = m->n;
    return ICP4R_OK;
}

int icp4r_map_time_ms(icp4r_map* m, double* avg_ms, int32_t* calls) {
    if (!m || !avg_ms) return fail(ICP4R_E_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(m->ctx->device));
    double tot = 0.0;
    for (size_t i = 0; i < m->used; ++i) {
        HIP_TRY(hipEventSynchronize(m->events[i].stop));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, m->events[i].start, m->events[i].stop));
        tot += ms;
    }
    *avg_ms = m->used ? tot / (double)m->used : 0.0;
    if (calls) *calls = (int32_t)m->used;
    return ICP4R_OK;
}

int icp4r_map_time_reset(icp4r_map* m) {
    if (!m) return fail(ICP4R_E_INVALID, "map is NULL");
    m->used = 0;
    return ICP4R_OK;
}

}  // extern "C"
