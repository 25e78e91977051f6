/*
 * gicp_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of fast_gicp's FastGICPSingleThread as the reference's radar_odometry node calls it
 * (src/radar_odometry.cpp:398-411).  fast_gicp (koide3/fast_gicp, included at
 * radar_odometry.cpp:31-32) is neither vendored nor installed here; its published algorithm is
 * restated (include/icp4r/icp4r_gicp.h has the summary):
 *
 *   calculate_covariances   k nearest neighbours (the point itself included) of each point in its own
 *                           cloud, mean-centred, cov = N Nᵀ / k, regularised (PLANE: U diag(1,1,1e-3) Uᵀ)
 *   update_correspondences  exact 1-NN of the float-transformed source point in the target;
 *                           Mahalanobis M = (C_B + R C_A Rᵀ)⁻¹
 *   linearize               e = b - T a, H = Σ JᵀMJ, g = Σ JᵀMe, J = [skew(T a), -I], y = Σ eᵀMe
 *   step_lm                 lambda = 1e-9 max|diag H| (first step), (H + lambda I) d = -g, delta =
 *                           [so3_exp(d0..2) | d3..5], accept if rho > 0, at most 10 trials
 *   is_converged            max(|R_delta - I| / 2e-3, |t_delta| / 5e-4) < 1
 *
 * Distances are FLANN's L2_Simple float ((dx*dx + dy*dy) + dz*dz); neighbour ties resolve to the
 * lowest index.  Everything else is double.
 *
 * Parity status: UNPINNED by the reference (no fast_gicp, no fixtures).  Pinned by known-answer
 * tests (tests/test_gicp.py): a pair with a known rigid transform and surface structure.
 */
#ifndef GICP_ORACLE_H
#define GICP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gicp_oracle_params {
    int32_t k;              /* k_correspondences_ */
    int32_t max_iterations; /* 64 */
    double rotation_epsilon;
    double transformation_epsilon;
    double max_correspondence_distance;
    int32_t regularization; /* icp4r_gicp_regularization */
    int32_t lm_max_iterations;
    double lm_init_lambda_factor;
} gicp_oracle_params;

typedef struct gicp_oracle_result {
    double T[16];        /* final x0, row-major (double; final_transformation_ = float of it) */
    int32_t iterations;  /* nr_iterations_ */
    int32_t converged;
    int32_t lm_failed;   /* step_lm returned false */
    int32_t n_valid;     /* correspondences of the last linearisation */
} gicp_oracle_result;

void gicp_oracle_params_default(gicp_oracle_params* p);

/* calculate_covariances: cloud n x 4 floats (x, y, z, ·); cov_out n x 9 row-major. */
void gicp_oracle_covariances(const float* cloud, int32_t n, int32_t k, int32_t regularization, double* cov_out);

/* FastGICP align from the identity or guess (row-major 4x4 double, may be NULL). */
int gicp_oracle_align(const float* src, int32_t n, const float* tgt, int32_t m, const double* guess,
                      const gicp_oracle_params* p, gicp_oracle_result* r);

#ifdef __cplusplus
}
#endif
#endif
