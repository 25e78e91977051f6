/*
 * icp4r_ego.h — C ABI of the radar ego-velocity estimator and the scan parser (SURVEY.md §8f
 * ranks 2-3): the per-frame work the reference node does around its ICP call, on the GPU.
 *
 * Replaces, in /root/reference/src/iterative_closest_point.cpp:
 *
 *     read_radar_data(path)                                         // :64-82   (host: icp4r/replay)
 *     parse: distance, arfa, beta per RadarPoint_Info2              // :354-385 -> icp4r_radar_features
 *     fitSineRansac(point_src_cloud, A_src, b_src, PointsNum * 0.2) // :389, :85-128
 *     static / dynamic split (delta > 0.2)                          // :391-407
 *     Vxyz = (K^T K)^-1 K^T Vr over the static points                // :410-431
 *                                                                   //   -> icp4r_ego_velocity[_batch_device]
 *
 * Semantics follow the reference operation by operation (float features with the float overloads
 * of atan2 / asin / sqrt, PCL 1.8's DEG2RAD = x * 0.017453293 in double, double model and LSQ) with
 * three deliberate departures, all reference bugs: hypothesis points are drawn
 * reproducibly (SplitMix64 of seed + k, mod n) instead of from a re-seeded std::random_device;
 * the draw is in [0, n) instead of the inclusive [0, n] that reads one past the end; n is an int,
 * not a wrapping uint16_t.  The result carries the best score fitSineRansac never returns.
 *
 * Conventions as icp4r.h: int status returns, icp4r_last_error(), one context per host thread.
 */
#ifndef ICP4R_EGO_H
#define ICP4R_EGO_H

#include <stdint.h>

#include "icp4r.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct icp4r_ego_params {
    int32_t iterations;       /* RANSAC hypotheses; <= 0: (int)(0.2 * n) as the node passes (:389)  */
    int32_t reserved0;
    double sigma;             /* inlier threshold |delta| < sigma;          node default 0.5 (:89)   */
    double dynamic_threshold; /* delta > this -> dynamic point;             node: 0.2 (:396)         */
    uint64_t seed;            /* hypothesis stream (SplitMix64 of seed + k)                          */
    int32_t reserved[8];
} icp4r_ego_params;

typedef struct icp4r_ego_result {
    double A;             /* A_best (0 when no hypothesis scored > 0, as the node's initial value) */
    double b;             /* b_best                                                                */
    double v[3];          /* Vxyz                                                                  */
    double score;         /* best inlier count                                                     */
    int32_t n;            /* points in the scan                                                    */
    int32_t n_static;     /* points with delta <= dynamic_threshold                                */
    int32_t iterations;   /* hypotheses evaluated                                                  */
    int32_t best;         /* index of the winning hypothesis, -1 if none                           */
    int32_t status;       /* icp4r_status of this scan                                             */
    int32_t reserved;
} icp4r_ego_result; /* 72 bytes */

void icp4r_ego_params_default(icp4r_ego_params* p);

/* The node's parse (:373-384) of n 5-float records [x, y, z, intensity, v_r] (host buffers):
 * xyzi_out (optional, n x 4: the PointXYZI fill, :404-406) and feat_out (optional, n x 4: distance,
 * arfa, beta — degrees, float — and v_r). */
int icp4r_radar_features(icp4r_ctx* ctx, const float* records, int32_t n, float* xyzi_out, float* feat_out);

/* Ego velocity of one scan from host records.  static_mask_out (optional, n bytes: 1 = static),
 * scores_out (optional, one double per hypothesis: its inlier count). */
int icp4r_ego_velocity(icp4r_ctx* ctx, const float* records, int32_t n, const icp4r_ego_params* params,
                       icp4r_ego_result* out, uint8_t* static_mask_out, double* scores_out);

/* Many scans, device-resident, asynchronous on hip_stream (NULL = the context's stream):
 * records: device, concatenated 5-float records; off/cnt: device[nscans] (first record, count);
 * max_n: host-known upper bound of cnt[]; results: device[nscans]; static_mask: device (one byte
 * per record, same indexing as records) or NULL.  Scan s uses the seed params->seed + (s << 32). */
int icp4r_ego_velocity_batch_device(icp4r_ctx* ctx, const float* records, const int64_t* off, const int32_t* cnt,
                                    int32_t nscans, int32_t max_n, const icp4r_ego_params* params,
                                    icp4r_ego_result* results, uint8_t* static_mask, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* ICP4R_EGO_H */
