// icp4r_map.hip — scan-to-map store kernels for gfx950 (include/icp4r/icp4r_map.h).
//
// The reference keeps its radar map in an ikd-Tree and, per scan, takes the submap with
// Sector_Search — a full traversal with a per-point keep test (ikd_Tree.cpp:1098-1140).  Here the
// map is an append-only float4 array in HBM and the query is a stable stream compaction at HBM
// bandwidth: count per 4096-point block -> exclusive scan of the block counts -> ordered write.
// Both passes read the map once (16 B/point) and the write pass stores the kept points (16 B each).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "icp4r_internal.hpp"

namespace icp4r {

constexpr int kSecWG = 256;
constexpr int kSecPer = 16;                  // points per thread
constexpr int kSecBlock = kSecWG * kSecPer;  // points per workgroup
constexpr double kPi = 3.14159265358979323846;  // glibc's M_PI (math.h), the reference's constant

// KD_TREE::calc_dist (ikd_Tree.cpp:1427-1431): float, ((dx*dx + dy*dy) + dz*dz), unfused.
__device__ __forceinline__ float map_calc_dist(float ax, float ay, float az, float bx, float by, float bz) {
    const float dx = ax - bx, dy = ay - by, dz = az - bz;
    float d = dx * dx;
    d = d + dy * dy;
    d = d + dz * dz;
    return d;
}

// KD_TREE::calc_heading (ikd_Tree.cpp:1434-1448): float asinf / sqrtf (ikd_Tree.h's `using namespace
// std` picks the float overloads), `* 180` in float, `/ M_PI` and `180 +` in double, stored as float.
__device__ __forceinline__ float map_calc_heading(float ax, float ay, float az, float bx, float by, float bz) {
    const float r = (ax - bx) / sqrtf(map_calc_dist(ax, ay, az, bx, by, bz));
    float h;
    if (ay - by < 0.0f)
        h = (float)(180.0 + (double)(asinf(r) * 180.0f) / kPi);
    else
        h = (float)((double)(-asinf(r) * 180.0f) / kPi);
    if (h > 180.0f && h < 360.0f) h = h - 360.0f;
    return h;
}

// Search_by_sector's keep test (ikd_Tree.cpp:1114-1116), precedence included; nothing is deleted.
__device__ __forceinline__ bool sector_keep(const float4 p, const SectorArgs& a) {
    const float dh = fabsf(map_calc_heading(p.x, p.y, p.z, a.cx, a.cy, a.cz) - a.heading);
    return (map_calc_dist(p.x, p.y, p.z, a.cx, a.cy, a.cz) <= a.radius * a.radius && dh < 60.0f) || (dh > 300.0f);
}

// pointAssociateToMap (radar_odometry.cpp:137-145): p_w = Rtrans * p + t_w_curr in double, per row
// ((R0*x + R1*y) + R2*z) + t (Eigen's packet order), cast to float; intensity copied.
__global__ __launch_bounds__(256) void associate_kernel(const float4* __restrict__ in, int64_t n, Mat3x4d M,
                                                        float4* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 v = in[i];
    const double x = v.x, y = v.y, z = v.z;
    double w[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        double s = M.R[3 * r] * x;
        s = s + M.R[3 * r + 1] * y;
        s = s + M.R[3 * r + 2] * z;
        w[r] = s + M.t[r];
    }
    out[i] = make_float4((float)w[0], (float)w[1], (float)w[2], v.w);
}

__global__ __launch_bounds__(kSecWG) void sector_count_kernel(const float4* __restrict__ map, int64_t n,
                                                              SectorArgs a, int32_t* __restrict__ counts) {
    __shared__ int32_t wsum[kSecWG / 64];
    const int64_t base = (int64_t)blockIdx.x * kSecBlock;
    int c = 0;
#pragma unroll 4
    for (int k = 0; k < kSecPer; ++k) {
        const int64_t i = base + k * kSecWG + threadIdx.x;
        if (i < n && sector_keep(map[i], a)) ++c;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < kSecWG / 64; ++w) t += wsum[w];
        counts[blockIdx.x] = t;
    }
}

// Exclusive scan of the block counts by one workgroup (tiles of 1024); total -> *total.
__global__ __launch_bounds__(1024) void sector_scan_kernel(const int32_t* __restrict__ counts, int nblk,
                                                           int32_t* __restrict__ offsets, int32_t* __restrict__ total) {
    __shared__ int32_t wsum[16];
    __shared__ int32_t carry;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int b0 = 0; b0 < nblk; b0 += 1024) {
        const int i = b0 + tid;
        const int v = i < nblk ? counts[i] : 0;
        int incl = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_up(incl, off, 64);
            if (lane >= off) incl += o;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        int wbase = 0;
        for (int w = 0; w < wave; ++w) wbase += wsum[w];
        const int c0 = carry;
        if (i < nblk) offsets[i] = c0 + wbase + incl - v;
        __syncthreads();
        if (tid == 1023) carry = c0 + wbase + incl;
        __syncthreads();
    }
    if (tid == 0) *total = carry;
}

// Ordered write: within a block, round k covers 256 consecutive points, wave w its 64, lane its one
// — so ranks taken round by round, wave by wave, lane by lane are insertion order.
__global__ __launch_bounds__(kSecWG) void sector_write_kernel(const float4* __restrict__ map, int64_t n,
                                                              SectorArgs a, const int32_t* __restrict__ offsets,
                                                              float4* __restrict__ out) {
    __shared__ int32_t wcnt[kSecWG / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t base = (int64_t)blockIdx.x * kSecBlock;
    int32_t run = offsets[blockIdx.x];
    for (int k = 0; k < kSecPer; ++k) {
        const int64_t i = base + k * kSecWG + tid;
        float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
        bool keep = false;
        if (i < n) {
            p = map[i];
            keep = sector_keep(p, a);
        }
        const uint64_t m = __ballot(keep);
        if (lane == 0) wcnt[wave] = __builtin_popcountll(m);
        __syncthreads();
        int before = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kSecWG / 64; ++w) {
            before += w < wave ? wcnt[w] : 0;
            tot += wcnt[w];
        }
        if (keep) {
            const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            out[run + before + (int32_t)r] = p;
        }
        run += tot;
        __syncthreads();
    }
}

hipError_t launch_associate(const float4* in, int64_t n, const Mat3x4d& M, float4* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(associate_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, n, M, out);
    return hipGetLastError();
}

int64_t sector_blocks(int64_t n) { return (n + kSecBlock - 1) / kSecBlock; }

hipError_t launch_sector(const float4* map, int64_t n, const SectorArgs& a, int32_t* counts, int32_t* offsets,
                         int32_t* total, float4* out, hipStream_t st) {
    const int64_t nblk = sector_blocks(n);
    if (nblk == 0) return hipMemsetAsync(total, 0, sizeof(int32_t), st);
    hipLaunchKernelGGL(sector_count_kernel, dim3((unsigned)nblk), dim3(kSecWG), 0, st, map, n, a, counts);
    hipLaunchKernelGGL(sector_scan_kernel, dim3(1), dim3(1024), 0, st, counts, (int)nblk, offsets, total);
    hipLaunchKernelGGL(sector_write_kernel, dim3((unsigned)nblk), dim3(kSecWG), 0, st, map, n, a, offsets, out);
    return hipGetLastError();
}

}  // namespace icp4r
