/*
 * ego_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference node's radar ego-velocity path, the part
 * of the per-frame loop of src/iterative_closest_point.cpp around the ICP call:
 *
 *   :354-385   parse: x, y, z, intensity, v_r from the 5-float record; distance = sqrt (float),
 *              arfa = atan2(y, x)*180/M_PI, beta = asin(z/distance)*180/M_PI (float overloads,
 *              `* 180` in float, `/ M_PI` in double, stored as float — RadarPoint_Info2, userdefine.h)
 *   :85-128    fitSineRansac(points, A, b, iterations = (int)(0.2 N), sigma = 0.5): two-point sine
 *              model v_r cos(beta) = A cos(arfa + b), inlier count |delta| < sigma, first strict max
 *   :391-407   split: delta > 0.2 (signed) -> dynamic, else static
 *   :410-431   Vxyz = (K^T K)^-1 K^T Vr over the static points, K_i = [ca cb, sa cb, sb]
 *
 * DEG2RAD is PCL 1.8's macro `((x) * 0.017453293)` (pcl_macros.h), applied to the float angle in
 * double.  Every transcendental is glibc's (x86-64), as in the reference.
 *
 * Deliberate departures (reference bugs): the reference draws each hypothesis pair
 * from a freshly seeded std::random_device (non-reproducible) with uniform_int_distribution(0, num)
 * INCLUSIVE (reads points[num], one past the end), and keeps num in a uint16_t (wraps at 65,536).
 * Here hypothesis k uses i1 = h(seed, 2k) mod n, i2 = h(seed, 2k+1) mod n with the SplitMix64 finaliser
 * h (ego_hyp_index), n as int — the GPU draws the same pairs, so runs are reproducible and comparable.
 * fitSineRansac also falls off its end without a return (UB); here it returns the best score.
 *
 * Parity status: UNPINNED by the reference (no tests or fixtures; the node needs ROS/PCL).  Pinned by
 * analytic known-answer tests (a synthetic sequence with a known ego velocity, tests/test_ego.py).
 */
#ifndef EGO_ORACLE_H
#define EGO_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per point: feat[4 i ..] = distance, arfa (deg), beta (deg), v_r — all float, as the node stores them.
 * rec: n records of 5 floats (x, y, z, intensity, v_r). */
void ego_features(const float* rec, int32_t n, float* feat);

/* Index of hypothesis point k of a scan (k = 2h, 2h+1 for hypothesis h): SplitMix64(seed + k) mod n. */
int32_t ego_hyp_index(uint64_t seed, int64_t k, int32_t n);

/* fitSineRansac over features feat (n x 4): returns the best score; A_best/b_best keep their input
 * values when no hypothesis scores > 0 (the node passes 0, 0).  scores (optional): per hypothesis.
 * best_h (optional): index of the winning hypothesis, -1 if none. */
double ego_fit_sine_ransac(const float* feat, int32_t n, int32_t iterations, double sigma, uint64_t seed,
                           double* A_best, double* b_best, double* scores, int32_t* best_h);

/* Split (delta > dyn_threshold -> dynamic) and the normal-equation least squares over the static
 * points.  static_mask (optional, n bytes): 1 = static.  Returns the number of static points;
 * V = (K^T K)^-1 K^T Vr (Eigen 3.3's cofactor 3x3 inverse; NaN/Inf when K^T K is singular). */
int32_t ego_split_lsq(const float* feat, int32_t n, double A, double b, double dyn_threshold, uint8_t* static_mask,
                      double* V);

#ifdef __cplusplus
}
#endif
#endif
