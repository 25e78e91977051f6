/*
 * map_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the scan-to-map submap path of the reference's radar_odometry node
 * (SURVEY.md §8f rank 1): the ikd-Tree map store as radar_odometry.cpp uses it and its
 * Sector_Search query.
 *
 *   radar_odometry.cpp:92        KD_TREE<pcl::PointXYZI> ikd_Tree(0.3, 0.6, 0.5);
 *   radar_odometry.cpp:347-348   ikd_Tree.Build(src->points); set_downsample_param(0.5);
 *   radar_odometry.cpp:384-390   pointAssociateToMap(...) per point; ikd_Tree.Add_Points(scan_map, false);
 *   radar_odometry.cpp:396       ikd_Tree.Sector_Search(p_now, RADAR_RADIUS (80), heading, SubMap);
 *   third_party/ikd-Tree/ikd_Tree.cpp:415-419, 1098-1140, 1427-1448
 *
 * On this path nothing is ever deleted (Add_Points(.., false) only inserts, Build replaces), and
 * Sector_Search visits every node (its box pruning is commented out, ikd_Tree.cpp:1103-1113), so the
 * map is an append-only point list and the query is a full filter.  Output order: ikd-Tree returns a
 * pre-order traversal of its current (rebalanced) tree; the restatement returns insertion order —
 * the SAME SET, in a defined order.
 *
 * Parity status: UNPINNED by the reference (no tests or fixtures for this path; ikd_Tree.cpp needs
 * PCL headers, absent here, so it is not built).  Pinned by analytic known-answer tests
 * (tests/test_map.py).  The only library function on the path is asinf (glibc here; ROCm ocml on
 * the device): the two may differ by an ulp, which can flip only points within ~1e-4 deg of a
 * sector edge (|dh| = 60 or 300) — the GPU tests allow exactly that, nothing else.
 */
#ifndef MAP_ORACLE_H
#define MAP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* KD_TREE::calc_dist (ikd_Tree.cpp:1427-1431): float, ((dx*dx + dy*dy) + dz*dz). */
float oracle_calc_dist(const float* a, const float* b);

/* KD_TREE::calc_heading (ikd_Tree.cpp:1434-1448): degrees, float asinf/sqrtf, x180/M_PI in double. */
float oracle_calc_heading(const float* a, const float* b);

/* Search_by_sector's keep test (ikd_Tree.cpp:1114-1116), C precedence included:
 *   (!deleted && d2 <= r*r && |h - heading| < 60) || |h - heading| > 300       (deleted == 0 here) */
int oracle_sector_keep(const float* p, const float* center, float radius, float heading);

/* Sector_Search over an append-only map of n points (x, y, z at stride_floats): writes the indices
 * of the kept points in insertion order to out_idx (capacity n) and returns their count. */
int64_t oracle_sector_search(const float* map, int64_t n, int32_t stride_floats, const float* center, float radius,
                             float heading, int64_t* out_idx);

/* pointAssociateToMap (radar_odometry.cpp:137-145): point_w = Rtrans * p + t_w_curr in double
 * (R row-major 3x3; each row ((R0*x + R1*y) + R2*z) + t, Eigen's packet order), then cast to float;
 * intensity copied.  in/out: n points, 4 floats each (x, y, z, intensity). */
void oracle_associate_to_map(const float* in, int64_t n, const double* R, const double* t, float* out);

#ifdef __cplusplus
}
#endif
#endif
