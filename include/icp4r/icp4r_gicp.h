/*
 * icp4r_gicp.h — C ABI of the generalized-ICP registration the reference's radar_odometry node runs
 * on its scan-to-map path.
 *
 * Replaces /root/reference/src/radar_odometry.cpp:398-411:
 *
 *     fast_gicp::FastGICPSingleThread<pcl::PointXYZI, pcl::PointXYZI> fgicp_st;   // :399
 *     fgicp_st.clearTarget(); fgicp_st.clearSource();                              // :400-401
 *     fgicp_st.setInputTarget(SubMap); fgicp_st.setInputSource(scan_map);          // :402-403
 *     fgicp_st.setCorrespondenceRandomness(5);                                     // :404
 *     fgicp_st.align(*Final);                                                      // :405
 *     fgicp_st.getFitnessScore(); fgicp_st.hasConverged();                          // :406-408
 *     fgicp_st.getFinalTransformation().cast<double>();                            // :411
 *
 * fast_gicp (koide3/fast_gicp; included at radar_odometry.cpp:31-32, not vendored, not in this
 * image) is restated from its published algorithm: per-point covariances from the k nearest
 * neighbours of the same cloud, regularised to the PLANE model U diag(1, 1, 1e-3) Uᵀ; per iteration
 * exact nearest-neighbour correspondences of the float-transformed source, Mahalanobis weights
 * (C_B + R C_A Rᵀ)⁻¹, the Gauss-Newton system JᵀMJ / JᵀMe with J = [skew(T a), -I], and
 * Levenberg-Marquardt steps (lambda from 1e-9 max|diag H|, at most 10 trials, so3 exponential
 * update); converged when |R_delta - I| < 2e-3 and |t_delta| < 5e-4 elementwise, at most 64
 * iterations.  The C ABI shares icp4r.h's context, conventions and result struct.
 *
 * Parity status: UNPINNED by the reference (fast_gicp is absent; the node needs ROS).  Pinned by
 * the C restatement oracle/gicp_oracle.c and known-answer tests (tests/test_gicp.py).
 */
#ifndef ICP4R_GICP_H
#define ICP4R_GICP_H

#include <stdint.h>

#include "icp4r.h"

#ifdef __cplusplus
extern "C" {
#endif

/* fast_gicp::RegularizationMethod */
typedef enum icp4r_gicp_regularization {
    ICP4R_GICP_REG_NONE = 0,
    ICP4R_GICP_REG_MIN_EIG = 1,
    ICP4R_GICP_REG_NORMALIZED_MIN_EIG = 2,
    ICP4R_GICP_REG_PLANE = 3,
    ICP4R_GICP_REG_FROBENIUS = 4
} icp4r_gicp_regularization;

typedef struct icp4r_gicp_params {
    int32_t k_correspondences;          /* setCorrespondenceRandomness;  fast_gicp 20 (the node: 5)   */
    int32_t max_iterations;             /* LsqRegistration::max_iterations_;              64          */
    double rotation_epsilon;            /* LsqRegistration::rotation_epsilon_;            2e-3        */
    double transformation_epsilon;      /* LsqRegistration::transformation_epsilon_;      5e-4        */
    double max_correspondence_distance; /* FastGICP::corr_dist_threshold_;                FLT_MAX     */
    int32_t regularization;             /* icp4r_gicp_regularization;                     PLANE       */
    int32_t lm_max_iterations;          /* LsqRegistration::lm_max_iterations_;           10          */
    double lm_init_lambda_factor;       /* LsqRegistration::lm_init_lambda_factor_;       1e-9        */
    int32_t compute_fitness;            /* 1: Registration::getFitnessScore(DBL_MAX) computed once    */
    int32_t reserved[9];
} icp4r_gicp_params;

void icp4r_gicp_params_default(icp4r_gicp_params* p);

/* FastGICP(SingleThread)::align(output[, guess]) for one pair from host buffers (strides in bytes as
 * icp4r_align).  out->T = final_transformation_ (column-major float), out->iterations =
 * nr_iterations_ (index of the last iteration, as fast_gicp reports it), out->converged,
 * out->fitness = getFitnessScore().  aligned_out: optional transformPointCloud(input, final). */
int icp4r_gicp_align(icp4r_ctx* ctx, const float* src, int32_t n, int32_t src_stride_bytes, const float* tgt,
                     int32_t m, int32_t tgt_stride_bytes, const float* guess, const icp4r_gicp_params* params,
                     icp4r_result* out, float* aligned_out, int32_t out_stride_bytes);

/* The same for a device-resident batch (icp4r_batch layout; results[npairs] in device memory), stream
 * ordered on hip_stream (NULL: the context's stream).  Per pair as icp4r_gicp_align. */
int icp4r_gicp_align_batch_device(icp4r_ctx* ctx, const icp4r_batch* batch, const icp4r_gicp_params* params,
                                  icp4r_result* results, void* hip_stream);

/* FastGICP::calculate_covariances for one cloud (host buffers): cov_out[n][9] row-major 3x3. */
int icp4r_gicp_covariances(icp4r_ctx* ctx, const float* cloud, int32_t n, int32_t stride_bytes, int32_t k,
                           int32_t regularization, double* cov_out);

#ifdef __cplusplus
}
#endif

#endif /* ICP4R_GICP_H */
