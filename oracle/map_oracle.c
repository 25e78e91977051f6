/* map_oracle.c — TEST INFRASTRUCTURE ONLY.  See map_oracle.h for scope, citations and pinning. */
#include "map_oracle.h"

#include <math.h>

#ifndef M_PI /* glibc's value (math.h, POSIX) — what the reference's M_PI is */
#define M_PI 3.14159265358979323846
#endif

/* ikd_Tree.cpp:1427-1431 */
float oracle_calc_dist(const float* a, const float* b) {
    const float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    float dist = dx * dx;
    dist = dist + dy * dy;
    dist = dist + dz * dz;
    return dist;
}

/* ikd_Tree.cpp:1434-1448.  `using namespace std` (ikd_Tree.h:20) makes asin/sqrt of a float the
 * float overloads; `asin(..) * 180` is float * int (float), `/ M_PI` promotes to double, and the
 * result is stored in a float. */
float oracle_calc_heading(const float* a, const float* b) {
    float heading;
    const float r = (a[0] - b[0]) / sqrtf(oracle_calc_dist(a, b));
    if (a[1] - b[1] < 0) {
        heading = (float)(180 + (double)(asinf(r) * 180.0f) / M_PI);
    } else {
        heading = (float)((double)(-asinf(r) * 180.0f) / M_PI);
    }
    if (heading > 180 && heading < 360) heading = heading - 360;
    return heading;
}

/* ikd_Tree.cpp:1114-1116 — note `A && B && C || D`: points with |dh| > 300 are kept whatever
 * their distance (and deletion flag); a point AT the centre has h = NaN and is never kept. */
int oracle_sector_keep(const float* p, const float* center, float radius, float heading) {
    const int deleted = 0;
    const float dh = fabsf(oracle_calc_heading(p, center) - heading);
    return (!deleted && oracle_calc_dist(p, center) <= radius * radius && dh < 60) || (dh > 300);
}

/* ikd_Tree.cpp:415-419 + 1098-1140 (full traversal), in insertion order. */
int64_t oracle_sector_search(const float* map, int64_t n, int32_t stride_floats, const float* center, float radius,
                             float heading, int64_t* out_idx) {
    int64_t k = 0;
    for (int64_t i = 0; i < n; ++i)
        if (oracle_sector_keep(map + i * stride_floats, center, radius, heading)) out_idx[k++] = i;
    return k;
}

/* radar_odometry.cpp:137-145 */
void oracle_associate_to_map(const float* in, int64_t n, const double* R, const double* t, float* out) {
    for (int64_t i = 0; i < n; ++i) {
        const double x = in[4 * i], y = in[4 * i + 1], z = in[4 * i + 2];
        for (int r = 0; r < 3; ++r) {
            double v = R[3 * r] * x;
            v = v + R[3 * r + 1] * y;
            v = v + R[3 * r + 2] * z;
            v = v + t[r];
            out[4 * i + r] = (float)v;
        }
        out[4 * i + 3] = in[4 * i + 3];
    }
}
