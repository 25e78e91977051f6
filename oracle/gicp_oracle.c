/* gicp_oracle.c — TEST INFRASTRUCTURE ONLY.  See gicp_oracle.h for scope, citations and pinning. */
#include "gicp_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

enum { REG_NONE = 0, REG_MIN_EIG = 1, REG_NORMALIZED_MIN_EIG = 2, REG_PLANE = 3, REG_FROBENIUS = 4 };

void gicp_oracle_params_default(gicp_oracle_params* p) {
    p->k = 20;
    p->max_iterations = 64;
    p->rotation_epsilon = 2e-3;
    p->transformation_epsilon = 5e-4;
    p->max_correspondence_distance = FLT_MAX;
    p->regularization = REG_PLANE;
    p->lm_max_iterations = 10;
    p->lm_init_lambda_factor = 1e-9;
}

static float l2f(const float* a, const float* b) {
    const float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    float d = dx * dx;
    d = d + dy * dy;
    d = d + dz * dz;
    return d;
}

static int key_less(float da, int ia, float db, int ib) { return da < db || (da == db && ia < ib); }

/* symmetric 3x3 eigen-decomposition by cyclic Jacobi: a (row-major) -> eigenvalues w, vectors V
 * (columns), sorted by decreasing eigenvalue */
static void sym_eig3(const double* a_in, double* w, double* V) {
    double a[9];
    memcpy(a, a_in, sizeof(a));
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        /* converged: the off-diagonal mass is below 1e-30 of the diagonal's (~1e-15 relative per
         * element, the double rounding level; waiting for an exact zero took many more sweeps) */
        const double off = a[1] * a[1] + a[2] * a[2] + a[5] * a[5];
        if (off <= 1e-30 * (a[0] * a[0] + a[4] * a[4] + a[8] * a[8])) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                const double apq = a[3 * p + q];
                if (apq == 0.0) continue;
                const double theta = (a[3 * q + q] - a[3 * p + p]) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 3; ++k) { /* A := Jᵀ A J */
                    const double akp = a[3 * k + p], akq = a[3 * k + q];
                    a[3 * k + p] = c * akp - s * akq;
                    a[3 * k + q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    const double apk = a[3 * p + k], aqk = a[3 * q + k];
                    a[3 * p + k] = c * apk - s * aqk;
                    a[3 * q + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    const double vkp = V[3 * k + p], vkq = V[3 * k + q];
                    V[3 * k + p] = c * vkp - s * vkq;
                    V[3 * k + q] = s * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < 3; ++i) w[i] = a[4 * i];
    for (int i = 0; i < 2; ++i) /* sort descending */
        for (int j = i + 1; j < 3; ++j)
            if (w[j] > w[i]) {
                const double tw = w[i];
                w[i] = w[j];
                w[j] = tw;
                for (int k = 0; k < 3; ++k) {
                    const double tv = V[3 * k + i];
                    V[3 * k + i] = V[3 * k + j];
                    V[3 * k + j] = tv;
                }
            }
}

static void inv3(const double* m, double* r) {
    const double c0 = m[4] * m[8] - m[5] * m[7];
    const double c1 = m[7] * m[2] - m[8] * m[1];
    const double c2 = m[1] * m[5] - m[2] * m[4];
    const double det = c0 * m[0] + c1 * m[3] + c2 * m[6];
    const double id = 1.0 / det;
    r[0] = c0 * id;
    r[1] = c1 * id;
    r[2] = c2 * id;
    r[3] = (m[5] * m[6] - m[3] * m[8]) * id;
    r[4] = (m[8] * m[0] - m[6] * m[2]) * id;
    r[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    r[6] = (m[3] * m[7] - m[4] * m[6]) * id;
    r[7] = (m[6] * m[1] - m[7] * m[0]) * id;
    r[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

/* FastGICP::calculate_covariances */
void gicp_oracle_covariances(const float* cloud, int32_t n, int32_t k, int32_t reg, double* cov_out) {
    if (k > n) k = n;
    float* bd = (float*)malloc(sizeof(float) * (size_t)(k > 0 ? k : 1));
    int* bi = (int*)malloc(sizeof(int) * (size_t)(k > 0 ? k : 1));
    for (int32_t i = 0; i < n; ++i) {
        int cnt = 0;
        const float* q = cloud + 4 * (int64_t)i;
        for (int32_t j = 0; j < n; ++j) { /* exact k-NN, (d², index) order */
            const float d = l2f(q, cloud + 4 * (int64_t)j);
            if (cnt == k && !key_less(d, j, bd[k - 1], bi[k - 1])) continue;
            int pos = cnt < k ? cnt++ : k - 1;
            while (pos > 0 && key_less(d, j, bd[pos - 1], bi[pos - 1])) {
                bd[pos] = bd[pos - 1];
                bi[pos] = bi[pos - 1];
                --pos;
            }
            bd[pos] = d;
            bi[pos] = j;
        }
        double mean[3] = {0, 0, 0};
        for (int j = 0; j < cnt; ++j)
            for (int r = 0; r < 3; ++r) mean[r] += (double)cloud[4 * (int64_t)bi[j] + r];
        for (int r = 0; r < 3; ++r) mean[r] /= (double)cnt;
        double c[9] = {0};
        for (int j = 0; j < cnt; ++j) {
            double d[3];
            for (int r = 0; r < 3; ++r) d[r] = (double)cloud[4 * (int64_t)bi[j] + r] - mean[r];
            for (int r = 0; r < 3; ++r)
                for (int s = 0; s < 3; ++s) c[3 * r + s] += d[r] * d[s];
        }
        for (int t = 0; t < 9; ++t) c[t] /= (double)k;
        double* o = cov_out + 9 * (int64_t)i;
        if (reg == REG_NONE) {
            memcpy(o, c, sizeof(c));
        } else if (reg == REG_FROBENIUS) {
            double C[9], Ci[9], nrm = 0.0;
            memcpy(C, c, sizeof(C));
            for (int t = 0; t < 3; ++t) C[4 * t] += 1e-3;
            inv3(C, Ci);
            for (int t = 0; t < 9; ++t) nrm += Ci[t] * Ci[t];
            nrm = sqrt(nrm);
            for (int t = 0; t < 9; ++t) Ci[t] /= nrm;
            inv3(Ci, o);
        } else {
            double w[3], V[9], v[3];
            sym_eig3(c, w, V);
            for (int t = 0; t < 3; ++t) {
                if (reg == REG_PLANE) v[t] = t < 2 ? 1.0 : 1e-3;
                else if (reg == REG_MIN_EIG) v[t] = w[t] > 1e-3 ? w[t] : 1e-3;
                else v[t] = (w[0] != 0.0 ? w[t] / w[0] : 0.0) > 1e-3 ? w[t] / w[0] : 1e-3;
            }
            for (int r = 0; r < 3; ++r)
                for (int s = 0; s < 3; ++s) {
                    double acc = 0.0;
                    for (int t = 0; t < 3; ++t) acc += V[3 * r + t] * v[t] * V[3 * s + t];
                    o[3 * r + s] = acc;
                }
        }
    }
    free(bd);
    free(bi);
}

/* ---- LsqRegistration / FastGICP */
typedef struct {
    double R[9], t[3];
} iso3;

static iso3 iso_mul(const iso3* a, const iso3* b) {
    iso3 o;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) o.R[3 * r + c] = a->R[3 * r] * b->R[c] + a->R[3 * r + 1] * b->R[3 + c] + a->R[3 * r + 2] * b->R[6 + c];
        o.t[r] = a->R[3 * r] * b->t[0] + a->R[3 * r + 1] * b->t[1] + a->R[3 * r + 2] * b->t[2] + a->t[r];
    }
    return o;
}

static void iso_apply(const iso3* T, const double* p, double* o) {
    for (int r = 0; r < 3; ++r) o[r] = T->R[3 * r] * p[0] + T->R[3 * r + 1] * p[1] + T->R[3 * r + 2] * p[2] + T->t[r];
}

/* so3_exp (fast_gicp so3.hpp) -> Eigen Quaternion::toRotationMatrix */
static void so3_exp(const double* w, double* R) {
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double imag, real;
    if (th2 < 1e-10) {
        const double th4 = th2 * th2;
        imag = 0.5 - 1.0 / 48.0 * th2 + 1.0 / 3840.0 * th4;
        real = 1.0 - 1.0 / 8.0 * th2 + 1.0 / 384.0 * th4;
    } else {
        const double th = sqrt(th2), half = 0.5 * th;
        imag = sin(half) / th;
        real = cos(half);
    }
    const double qw = real, qx = imag * w[0], qy = imag * w[1], qz = imag * w[2];
    const double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
    const double twx = tx * qw, twy = ty * qw, twz = tz * qw, txx = tx * qx, txy = ty * qx, txz = tz * qx;
    const double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

static int is_converged(const iso3* d, const gicp_oracle_params* p) {
    double m = 0.0;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            const double v = 1.0 / p->rotation_epsilon * fabs(d->R[3 * r + c] - (r == c ? 1.0 : 0.0));
            if (v > m) m = v;
        }
    for (int r = 0; r < 3; ++r) {
        const double v = 1.0 / p->transformation_epsilon * fabs(d->t[r]);
        if (v > m) m = v;
    }
    return m < 1.0;
}

/* solve (A) x = b for a symmetric positive definite 6x6 by LDLᵀ (no pivoting) */
static void ldlt6(const double* A, const double* b, double* x) {
    double L[36] = {0}, D[6];
    for (int j = 0; j < 6; ++j) {
        double s = A[6 * j + j];
        for (int k = 0; k < j; ++k) s -= L[6 * j + k] * L[6 * j + k] * D[k];
        D[j] = s;
        L[6 * j + j] = 1.0;
        for (int i = j + 1; i < 6; ++i) {
            double t = A[6 * i + j];
            for (int k = 0; k < j; ++k) t -= L[6 * i + k] * L[6 * j + k] * D[k];
            L[6 * i + j] = D[j] != 0.0 ? t / D[j] : t; /* Eigen: a zero pivot leaves its column undivided */
        }
    }
    double y[6];
    for (int i = 0; i < 6; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= L[6 * i + k] * y[k];
        y[i] = s;
    }
    for (int i = 0; i < 6; ++i) y[i] = fabs(D[i]) > DBL_MIN ? y[i] / D[i] : 0.0; /* Eigen's LDLT::solve */
    for (int i = 5; i >= 0; --i) {
        double s = y[i];
        for (int k = i + 1; k < 6; ++k) s -= L[6 * k + i] * x[k];
        x[i] = s;
    }
}

typedef struct {
    const float* src;
    const float* tgt;
    int32_t n, m;
    const double* cs; /* source covariances n x 9 */
    const double* ct; /* target covariances m x 9 */
    int32_t* corr;
    double* mah; /* n x 9 */
    double max_d2;
} gicp_ctx;

/* update_correspondences + linearize (H, g may be NULL: compute_error with cached correspondences) */
static double linearize(gicp_ctx* g, const iso3* T, double* H, double* b, int update) {
    if (update) {
        /* trans_f = trans.cast<float>(): p_f = R_f p + t_f in float, Eigen's order */
        float Rf[9], tf[3];
        for (int t = 0; t < 9; ++t) Rf[t] = (float)T->R[t];
        for (int t = 0; t < 3; ++t) tf[t] = (float)T->t[t];
        for (int32_t i = 0; i < g->n; ++i) {
            const float* a = g->src + 4 * (int64_t)i;
            float q[3];
            for (int r = 0; r < 3; ++r) {
                float s = Rf[3 * r] * a[0];
                s = s + Rf[3 * r + 1] * a[1];
                s = s + Rf[3 * r + 2] * a[2];
                q[r] = s + tf[r];
            }
            float bd = INFINITY;
            int bj = -1;
            for (int32_t j = 0; j < g->m; ++j) {
                const float d = l2f(q, g->tgt + 4 * (int64_t)j);
                if (d < bd) {
                    bd = d;
                    bj = j;
                }
            }
            g->corr[i] = ((double)bd < g->max_d2) ? bj : -1;
            if (g->corr[i] < 0) continue;
            /* RCR = C_B + R C_A Rᵀ; mahalanobis = RCR⁻¹ */
            const double* CA = g->cs + 9 * (int64_t)i;
            const double* CB = g->ct + 9 * (int64_t)g->corr[i];
            double RC[9], RCR[9];
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c)
                    RC[3 * r + c] = T->R[3 * r] * CA[c] + T->R[3 * r + 1] * CA[3 + c] + T->R[3 * r + 2] * CA[6 + c];
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c)
                    RCR[3 * r + c] = CB[3 * r + c] + (RC[3 * r] * T->R[3 * c] + RC[3 * r + 1] * T->R[3 * c + 1] + RC[3 * r + 2] * T->R[3 * c + 2]);
            inv3(RCR, g->mah + 9 * (int64_t)i);
        }
    }
    if (H) {
        memset(H, 0, sizeof(double) * 36);
        memset(b, 0, sizeof(double) * 6);
    }
    double sum = 0.0;
    for (int32_t i = 0; i < g->n; ++i) {
        const int j = g->corr[i];
        if (j < 0) continue;
        const double a[3] = {g->src[4 * (int64_t)i], g->src[4 * (int64_t)i + 1], g->src[4 * (int64_t)i + 2]};
        const double bb[3] = {g->tgt[4 * (int64_t)j], g->tgt[4 * (int64_t)j + 1], g->tgt[4 * (int64_t)j + 2]};
        double ta[3];
        iso_apply(T, a, ta);
        const double e[3] = {bb[0] - ta[0], bb[1] - ta[1], bb[2] - ta[2]};
        const double* M = g->mah + 9 * (int64_t)i;
        double Me[3];
        for (int r = 0; r < 3; ++r) Me[r] = M[3 * r] * e[0] + M[3 * r + 1] * e[1] + M[3 * r + 2] * e[2];
        sum += e[0] * Me[0] + e[1] * Me[1] + e[2] * Me[2];
        if (!H) continue;
        /* J = [skew(ta), -I] (3x6) */
        double J[18];
        J[0] = 0; J[1] = -ta[2]; J[2] = ta[1]; J[3] = -1; J[4] = 0; J[5] = 0;
        J[6] = ta[2]; J[7] = 0; J[8] = -ta[0]; J[9] = 0; J[10] = -1; J[11] = 0;
        J[12] = -ta[1]; J[13] = ta[0]; J[14] = 0; J[15] = 0; J[16] = 0; J[17] = -1;
        double MJ[18];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 6; ++c) MJ[6 * r + c] = M[3 * r] * J[c] + M[3 * r + 1] * J[6 + c] + M[3 * r + 2] * J[12 + c];
        for (int r = 0; r < 6; ++r) {
            for (int c = 0; c < 6; ++c) H[6 * r + c] += J[r] * MJ[c] + J[6 + r] * MJ[6 + c] + J[12 + r] * MJ[12 + c];
            b[r] += J[r] * Me[0] + J[6 + r] * Me[1] + J[12 + r] * Me[2];
        }
    }
    return sum;
}

int gicp_oracle_align(const float* src, int32_t n, const float* tgt, int32_t m, const double* guess,
                      const gicp_oracle_params* p, gicp_oracle_result* r) {
    memset(r, 0, sizeof(*r));
    if (n <= 0 || m <= 0) return -2;
    gicp_ctx g;
    g.src = src;
    g.tgt = tgt;
    g.n = n;
    g.m = m;
    double* cs = (double*)malloc(sizeof(double) * 9 * (size_t)n);
    double* ct = (double*)malloc(sizeof(double) * 9 * (size_t)m);
    g.corr = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    g.mah = (double*)malloc(sizeof(double) * 9 * (size_t)n);
    gicp_oracle_covariances(src, n, p->k, p->regularization, cs);
    gicp_oracle_covariances(tgt, m, p->k, p->regularization, ct);
    g.cs = cs;
    g.ct = ct;
    const float thr = (float)p->max_correspondence_distance;
    g.max_d2 = (double)(thr * thr); /* corr_dist_threshold_ * corr_dist_threshold_ in float */
    iso3 x0;
    for (int rr = 0; rr < 3; ++rr) {
        for (int c = 0; c < 3; ++c) x0.R[3 * rr + c] = guess ? guess[4 * rr + c] : (rr == c ? 1.0 : 0.0);
        x0.t[rr] = guess ? guess[4 * rr + 3] : 0.0;
    }
    double lambda = -1.0;
    int converged = 0, failed = 0, it = 0;
    for (int i = 0; i < p->max_iterations && !converged; ++i) {
        it = i;
        /* step_lm */
        double H[36], b[6];
        const double y0 = linearize(&g, &x0, H, b, 1);
        if (lambda < 0.0) {
            double mx = 0.0;
            for (int k = 0; k < 6; ++k)
                if (fabs(H[7 * k]) > mx) mx = fabs(H[7 * k]);
            lambda = p->lm_init_lambda_factor * mx;
        }
        double nu = 2.0;
        int ok = 0;
        iso3 delta;
        for (int t = 0; t < p->lm_max_iterations; ++t) {
            double A[36], nb[6], d[6];
            memcpy(A, H, sizeof(A));
            for (int k = 0; k < 6; ++k) A[7 * k] += lambda;
            for (int k = 0; k < 6; ++k) nb[k] = -b[k];
            ldlt6(A, nb, d);
            so3_exp(d, delta.R);
            delta.t[0] = d[3];
            delta.t[1] = d[4];
            delta.t[2] = d[5];
            const iso3 xi = iso_mul(&delta, &x0);
            const double yi = linearize(&g, &xi, NULL, NULL, 0);
            double den = 0.0;
            for (int k = 0; k < 6; ++k) den += d[k] * (lambda * d[k] - b[k]);
            const double rho = (y0 - yi) / den;
            if (rho < 0) {
                if (is_converged(&delta, p)) {
                    ok = 1;
                    break;
                }
                lambda = nu * lambda;
                nu = 2 * nu;
                continue;
            }
            x0 = xi;
            const double f = 1 - pow(2 * rho - 1, 3);
            lambda = lambda * (f > 1.0 / 3.0 ? f : 1.0 / 3.0);
            ok = 1;
            break;
        }
        if (!ok) {
            failed = 1;
            break;
        }
        converged = is_converged(&delta, p);
    }
    int nv = 0;
    for (int32_t i = 0; i < n; ++i) nv += g.corr[i] >= 0;
    for (int rr = 0; rr < 3; ++rr) {
        for (int c = 0; c < 3; ++c) r->T[4 * rr + c] = x0.R[3 * rr + c];
        r->T[4 * rr + 3] = x0.t[rr];
    }
    r->T[12] = r->T[13] = r->T[14] = 0.0;
    r->T[15] = 1.0;
    r->iterations = it;
    r->converged = converged;
    r->lm_failed = failed;
    r->n_valid = nv;
    free(cs);
    free(ct);
    free(g.corr);
    free(g.mah);
    return 0;
}
