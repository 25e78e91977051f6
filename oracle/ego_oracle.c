/* ego_oracle.c — TEST INFRASTRUCTURE ONLY.  See ego_oracle.h for scope, citations and pinning. */
#include "ego_oracle.h"

#include <math.h>

#ifndef M_PI /* glibc's value (math.h, POSIX) — what the reference's M_PI is */
#define M_PI 3.14159265358979323846
#endif

/* pcl/pcl_macros.h (PCL 1.8): #define DEG2RAD(x) ((x)*0.017453293) */
static double deg2rad(float x) { return (double)x * 0.017453293; }

/* iterative_closest_point.cpp:373-384 */
void ego_features(const float* rec, int32_t n, float* feat) {
    for (int32_t i = 0; i < n; ++i) {
        const float* r = rec + 5 * (int64_t)i;
        const float x = r[0], y = r[1], z = r[2];
        /* std::sqrt(float expression): x*x + y*y + z*z in float, left to right */
        float s = x * x;
        s = s + y * y;
        s = s + z * z;
        const float distance = sqrtf(s);
        const float arfa = (float)((double)(atan2f(y, x) * 180.0f) / M_PI);
        const float beta = (float)((double)(asinf(z / distance) * 180.0f) / M_PI);
        float* f = feat + 4 * (int64_t)i;
        f[0] = distance;
        f[1] = arfa;
        f[2] = beta;
        f[3] = r[4];
    }
}

static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int32_t ego_hyp_index(uint64_t seed, int64_t k, int32_t n) {
    return n > 0 ? (int32_t)(splitmix64(seed + (uint64_t)k) % (uint64_t)n) : 0;
}

/* iterative_closest_point.cpp:85-128 */
double ego_fit_sine_ransac(const float* feat, int32_t n, int32_t iterations, double sigma, uint64_t seed,
                           double* A_best, double* b_best, double* scores, int32_t* best_h) {
    double bestScore = 0.0;
    if (best_h) *best_h = -1;
    for (int32_t i = 0; i < iterations && n > 0; ++i) {
        const float* p1 = feat + 4 * (int64_t)ego_hyp_index(seed, 2 * (int64_t)i, n);
        const float* p2 = feat + 4 * (int64_t)ego_hyp_index(seed, 2 * (int64_t)i + 1, n);
        /* p.v_r = [3], p.beta = [2], p.arfa = [1] */
        const double k = (p1[3] * cos(deg2rad(p1[2]))) / (p2[3] * cos(deg2rad(p2[2])));
        const double b = atan((cos(deg2rad(p1[1])) - k * cos(deg2rad(p2[1]))) /
                              (sin(deg2rad(p1[1])) - k * sin(deg2rad(p2[1]))));
        const double A = cos(deg2rad(p1[2])) * p1[3] / cos((deg2rad(p1[1])) + b);
        double score = 0;
        for (int32_t j = 0; j < n; j++) {
            const float* pj = feat + 4 * (int64_t)j;
            const double delta = (cos(deg2rad(pj[2])) * pj[3]) - (A * cos(deg2rad(pj[1]) + b));
            if (fabs(delta) < sigma) score += 1;
        }
        if (scores) scores[i] = score;
        if (score > bestScore) {
            *A_best = A;
            *b_best = b;
            bestScore = score;
            if (best_h) *best_h = i;
        }
    }
    return bestScore;
}

/* Eigen 3.3 compute_inverse<Matrix3d> (Eigen/src/LU/InverseImpl.h): cofactors of the first column
 * give the determinant, result = cofactor^T / det. */
static void inverse3(const double m[9], double r[9]) {
#define M(i, j) m[3 * (i) + (j)]
    const double c0 = M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1);
    const double c1 = M(2, 1) * M(0, 2) - M(2, 2) * M(0, 1);
    const double c2 = M(0, 1) * M(1, 2) - M(0, 2) * M(1, 1);
    const double det = c0 * M(0, 0) + c1 * M(1, 0) + c2 * M(2, 0);
    const double inv = 1.0 / det;
    r[0] = c0 * inv;
    r[3] = (M(1, 2) * M(2, 0) - M(1, 0) * M(2, 2)) * inv;
    r[6] = (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0)) * inv;
    r[1] = c1 * inv;
    r[4] = (M(2, 2) * M(0, 0) - M(2, 0) * M(0, 2)) * inv;
    r[7] = (M(2, 0) * M(0, 1) - M(2, 1) * M(0, 0)) * inv;
    r[2] = c2 * inv;
    r[5] = (M(0, 2) * M(1, 0) - M(0, 0) * M(1, 2)) * inv;
    r[8] = (M(0, 0) * M(1, 1) - M(0, 1) * M(1, 0)) * inv;
#undef M
}

/* iterative_closest_point.cpp:391-431 */
int32_t ego_split_lsq(const float* feat, int32_t n, double A, double b, double dyn_threshold, uint8_t* static_mask,
                      double* V) {
    double KtK[9] = {0}, KtV[3] = {0};
    int32_t ns = 0;
    for (int32_t i = 0; i < n; ++i) {
        const float* p = feat + 4 * (int64_t)i;
        const double delta = (cos(deg2rad(p[2])) * p[3]) - (A * cos(deg2rad(p[1]) + b));
        const int stat = !(delta > dyn_threshold);
        if (static_mask) static_mask[i] = (uint8_t)stat;
        if (!stat) continue;
        ++ns;
        const double k[3] = {cos(deg2rad(p[1])) * cos(deg2rad(p[2])), sin(deg2rad(p[1])) * cos(deg2rad(p[2])),
                             sin(deg2rad(p[2]))};
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) KtK[3 * r + c] += k[r] * k[c];
            KtV[r] += k[r] * (double)p[3];
        }
    }
    double inv[9];
    inverse3(KtK, inv);
    for (int r = 0; r < 3; ++r) V[r] = inv[3 * r] * KtV[0] + inv[3 * r + 1] * KtV[1] + inv[3 * r + 2] * KtV[2];
    return ns;
}
