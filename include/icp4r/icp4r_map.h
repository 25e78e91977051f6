/*
 * icp4r_map.h — device-resident scan-to-map store and sector query.
 *
 * Replaces the reference's ikd-Tree map as radar_odometry uses it (a KD_TREE<pcl::PointXYZI>):
 *
 *   radar_odometry.cpp:92       KD_TREE<PointXYZI> ikd_Tree(0.3, 0.6, 0.5)   -> icp4r_map_create
 *   radar_odometry.cpp:347      ikd_Tree.Build(src->points)                  -> icp4r_map_build
 *   radar_odometry.cpp:348      ikd_Tree.set_downsample_param(0.5)           -> (no effect: the node
 *                               only calls Add_Points(.., false), which never downsamples)
 *   radar_odometry.cpp:382-390  pointAssociateToMap per point + Add_Points(scan_map, false)
 *                                                                            -> icp4r_map_add_scan
 *                               (or icp4r_map_add_points for world-frame points)
 *   radar_odometry.cpp:396      ikd_Tree.Sector_Search(p_now, 80, heading, SubMap->points)
 *                                                                            -> icp4r_map_sector_search
 *   third_party/ikd-Tree/ikd_Tree.cpp:415-419 (Sector_Search), 422-497 (Add_Points),
 *   1098-1140 (Search_by_sector), 1427-1448 (calc_dist, calc_heading)
 *
 * On this path nothing is ever deleted and Sector_Search visits every node, so the store is an
 * append-only float4 (x, y, z, intensity) array in HBM and the query is a full filter at HBM
 * bandwidth, kept in insertion order (ikd-Tree returns the same SET in its tree's pre-order).  The
 * keep test is the reference's, C precedence included:
 *
 *   (d2 <= r*r && |h - heading| < 60) || |h - heading| > 300
 *
 * with d2 and h = calc_heading(p, center) (degrees, 0 along +y, +90 along -x) in the reference's
 * float/double mix.  Points with |dh| > 300 are kept whatever their distance (the reference's
 * operator-precedence quirk); a point AT the centre has h = NaN and is never kept.
 */
#ifndef ICP4R_MAP_H
#define ICP4R_MAP_H

#include "icp4r/icp4r.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct icp4r_map icp4r_map;

/* A map store on the context's device (uses the context's stream; one map per context is
 * typical, several are allowed).  Destroy it before its context. */
int icp4r_map_create(icp4r_ctx* ctx, icp4r_map** out);
int icp4r_map_destroy(icp4r_map* map);

/* KD_TREE::Build: replace the contents with n points (x, y, z[, intensity]) of stride_bytes. */
int icp4r_map_build(icp4r_map* map, const float* pts, int64_t n, int32_t stride_bytes);

/* KD_TREE::Add_Points(points, downsample_on): append.  downsample_on must be 0 — the node's only
 * call (radar_odometry.cpp:390); the voxel-downsampling insert is not part of this path
 * (ICP4R_E_INVALID). */
int icp4r_map_add_points(icp4r_map* map, const float* pts, int64_t n, int32_t stride_bytes, int32_t downsample_on);

/* pointAssociateToMap + Add_Points(.., false) for one scan: p_w = R * p + t in double (R row-major
 * 3x3 = Rtrans, t = t_w_curr; per row ((R0*x + R1*y) + R2*z) + t), stored as float, intensity
 * copied.  world_out (optional, host, n x 4 floats) receives the world-frame scan (`scan_map`). */
int icp4r_map_add_scan(icp4r_map* map, const float* scan, int64_t n, int32_t stride_bytes, const double* R,
                       const double* t, float* world_out);

int icp4r_map_size(const icp4r_map* map, int64_t* n);

/* KD_TREE::Sector_Search(center, radius, heading_deg, Storage): the kept points, insertion order,
 * to host memory (float4 each).  Writes at most out_cap points; *out_n = the number kept (if it
 * exceeds out_cap the call returns ICP4R_E_TOO_LARGE and writes nothing).  Synchronous. */
int icp4r_map_sector_search(icp4r_map* map, const float* center, float radius, float heading_deg, float* out,
                            int64_t out_cap, int64_t* out_n);

/* Device-resident variant for scan-to-map registration: writes the kept points (float4) to d_out
 * (device, capacity >= icp4r_map_size) and their count to *d_count (device int32 — usable directly
 * as icp4r_batch.tgt_n).  Asynchronous on hip_stream (NULL = the context's stream). */
int icp4r_map_sector_search_device(icp4r_map* map, const float* center, float radius, float heading_deg,
                                   float* d_out, int32_t* d_count, void* hip_stream);

/* The stored points (device, float4, insertion order) and their count. */
int icp4r_map_points_device(icp4r_map* map, const float** d_points, int64_t* n);

/* Average device time (HIP events) of the sector-search launches since the last
 * icp4r_map_time_reset, and how many there were. */
int icp4r_map_time_ms(icp4r_map* map, double* avg_ms, int32_t* calls);
int icp4r_map_time_reset(icp4r_map* map);

#ifdef __cplusplus
}
#endif

#endif /* ICP4R_MAP_H */
