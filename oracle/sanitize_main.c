/* Host-only sanitizer driver for the oracle (TEST INFRASTRUCTURE): ASan + UBSan over the kd-tree
 * build/search, both Umeyama paths, the error paths and the fitness pass. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "icp_oracle.h"

static float frand(unsigned* s) {
    *s = *s * 1103515245u + 12345u;
    return ((*s >> 8) & 0xFFFF) / 65535.0f;
}

int main(void) {
    enum { N = 700, M = 650 };
    float* src = malloc(sizeof(float) * 4 * N);
    float* tgt = malloc(sizeof(float) * 4 * M);
    unsigned s = 1;
    for (int i = 0; i < M; ++i)
        for (int k = 0; k < 4; ++k) tgt[4 * i + k] = 80.0f * frand(&s) - 40.0f;
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < 4; ++k) src[4 * i + k] = tgt[4 * (i % M) + k] + 0.05f * (frand(&s) - 0.5f);
    oracle_params p;
    oracle_result r;
    float* out = malloc(sizeof(float) * 4 * N);
    for (int num = 0; num < 2; ++num)
        for (int nn = 0; nn < 2; ++nn) {
            oracle_params_default(&p);
            p.numerics = num;
            p.nn = nn;
            p.max_iterations = 5;
            if (oracle_align(src, N, 4, tgt, M, 4, NULL, &p, &r, out, NULL) != 0) return 1;
        }
    oracle_params_default(&p);
    p.huber_delta = 0.5;
    p.numerics = 1;
    if (oracle_align(src, N, 4, tgt, M, 4, NULL, &p, &r, NULL, NULL) != 0) return 2;
    if (oracle_align(src, N, 4, tgt, 0, 4, NULL, &p, &r, NULL, NULL) != -2) return 3;
    if (oracle_align(src, 2, 4, tgt, M, 4, NULL, &p, &r, NULL, NULL) != -3) return 4;
    int32_t* idx = malloc(sizeof(int32_t) * N);
    float* d2 = malloc(sizeof(float) * N);
    if (oracle_nearest(src, N, 4, tgt, M, 4, 0, idx, d2) != 0) return 5;
    double f = oracle_fitness(src, N, 4, tgt, M, 4, r.T, 1e300, 0);
    if (!isfinite(f)) return 6;
    free(src); free(tgt); free(out); free(idx); free(d2);
    printf("ok\n");
    return 0;
}
