/*
 * icp_oracle.c — TEST INFRASTRUCTURE ONLY (checker + CPU baseline, never the product).
 *
 * Plain-C restatement of the PCL 1.8.1 default ICP that the reference node runs at
 * /root/reference/src/iterative_closest_point.cpp:510-521.  PCL, FLANN and Eigen are third-party
 * and absent from /root/reference and from this image; the semantics below follow
 * SURVEY.md Appendix A, which restates upstream:
 *   PCL 1.8.1  registration/impl/icp.hpp                       computeTransformation, transformCloud
 *   PCL 1.8.1  registration/impl/registration.hpp              align, getFitnessScore
 *   PCL 1.8.1  registration/impl/correspondence_estimation.hpp determineCorrespondences
 *   PCL 1.8.1  registration/impl/transformation_estimation_svd.hpp (use_umeyama_ = true)
 *   PCL 1.8.1  registration/impl/default_convergence_criteria.hpp  hasConverged
 *   Eigen 3.3  Geometry/Umeyama.h (umeyama, with_scaling = false), JacobiSVD<Matrix3f>
 *   FLANN 1.9  KDTreeSingleIndex (leaf_max_size 15, middle split, eps 0) + L2_Simple<float>
 *
 * Build with -ffp-contract=off: the reference's x86-64 SSE build never fuses multiply-adds, and
 * every float expression below is written in the operation order of the upstream code.
 */
#include "icp_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ST_OK 0
#define ST_E_INVALID (-1)
#define ST_E_EMPTY (-2)
#define ST_E_TOO_FEW_CORR (-3)
#define ST_E_NONFINITE (-4)
#define ST_E_NOMEM (-7)

/* pcl::registration::DefaultConvergenceCriteria::ConvergenceState */
enum { CONV_NOT_CONVERGED = 0, CONV_ITERATIONS, CONV_TRANSFORM, CONV_ABS_MSE, CONV_REL_MSE,
       CONV_NO_CORRESPONDENCES };

void oracle_params_default(oracle_params* p) {
    memset(p, 0, sizeof(*p));
    p->max_iterations = 10;                          /* Registration ctor */
    p->min_correspondences = 3;                      /* Registration ctor */
    p->max_correspondence_distance = sqrt(DBL_MAX);  /* Registration ctor: corr_dist_threshold_ */
    p->transformation_epsilon = 0.0;
    p->transformation_rotation_epsilon = 0.0;
    p->euclidean_fitness_epsilon = -DBL_MAX;
    p->mse_threshold_absolute = 1e-12;               /* DefaultConvergenceCriteria ctor */
    p->max_iterations_similar_transforms = 0;
    p->numerics = ORACLE_NUM_F32;
    p->nn = ORACLE_NN_KDTREE;
    p->compute_fitness = 1;
    p->huber_delta = INFINITY;
    p->fitness_max_range = DBL_MAX;
}

/* ------------------------------------------------------------------------------------------ */
/* FLANN L2_Simple<float>: result += diff*diff over the 3 xyz components, float, unfused.      */
/* (DefaultPointRepresentation<PointXYZI> copies x,y,z only — intensity is ignored.)           */
static inline float l2_simple(const float* a, const float* b) {
    float d0 = a[0] - b[0];
    float r = d0 * d0;
    float d1 = a[1] - b[1];
    r = r + d1 * d1;
    float d2 = a[2] - b[2];
    r = r + d2 * d2;
    return r;
}

/* ------------------------------------------------------------------------------------------ */
/* kd-tree, FLANN KDTreeSingleIndex restated (buildIndex → divideTree/middleSplit_/planeSplit,  */
/* findNeighbors → searchLevel).  Data are reordered into leaf order (FLANN reorder_ = true).  */
typedef struct kd_node {
    int32_t child1, child2; /* -1 for a leaf */
    int32_t left, right;    /* leaf: [left, right) into vind */
    int32_t divfeat;
    float divlow, divhigh;
} kd_node;

typedef struct kd_tree {
    int32_t m;
    float* pts;     /* m*3, leaf order */
    int32_t* vind;  /* leaf order → original index */
    kd_node* nodes;
    int32_t nnodes, cap;
    float root_lo[3], root_hi[3];
} kd_tree;

#define KD_LEAF_MAX 15

static const float* kd_orig_pt(const float* data, int32_t stride, int32_t i) { return data + (size_t)i * stride; }

static void kd_minmax(const float* data, int32_t stride, const int32_t* ind, int32_t count, int feat,
                      float* mn, float* mx) {
    float lo = kd_orig_pt(data, stride, ind[0])[feat], hi = lo;
    for (int32_t i = 1; i < count; ++i) {
        float v = kd_orig_pt(data, stride, ind[i])[feat];
        if (v > hi) hi = v;
        if (v < lo) lo = v;
    }
    *mn = lo;
    *mx = hi;
}

static void kd_plane_split(const float* data, int32_t stride, int32_t* ind, int32_t count, int feat,
                           float cutval, int32_t* lim1, int32_t* lim2) {
    int32_t left = 0, right = count - 1;
    for (;;) {
        while (left <= right && kd_orig_pt(data, stride, ind[left])[feat] < cutval) ++left;
        while (left <= right && kd_orig_pt(data, stride, ind[right])[feat] >= cutval) --right;
        if (left > right) break;
        int32_t t = ind[left]; ind[left] = ind[right]; ind[right] = t;
        ++left; --right;
    }
    *lim1 = left;
    right = count - 1;
    for (;;) {
        while (left <= right && kd_orig_pt(data, stride, ind[left])[feat] <= cutval) ++left;
        while (left <= right && kd_orig_pt(data, stride, ind[right])[feat] > cutval) --right;
        if (left > right) break;
        int32_t t = ind[left]; ind[left] = ind[right]; ind[right] = t;
        ++left; --right;
    }
    *lim2 = left;
}

static int32_t kd_new_node(kd_tree* t) {
    if (t->nnodes == t->cap) {
        t->cap = t->cap ? t->cap * 2 : 64;
        t->nodes = (kd_node*)realloc(t->nodes, (size_t)t->cap * sizeof(kd_node));
    }
    return t->nnodes++;
}

/* divideTree: bbox in/out (tight bbox of the subtree on return). */
static int32_t kd_divide(kd_tree* t, const float* data, int32_t stride, int32_t left, int32_t right,
                         float lo[3], float hi[3]) {
    int32_t id = kd_new_node(t);
    if (right - left <= KD_LEAF_MAX) {
        t->nodes[id].child1 = t->nodes[id].child2 = -1;
        t->nodes[id].left = left;
        t->nodes[id].right = right;
        for (int d = 0; d < 3; ++d) {
            lo[d] = hi[d] = kd_orig_pt(data, stride, t->vind[left])[d];
        }
        for (int32_t k = left + 1; k < right; ++k) {
            const float* p = kd_orig_pt(data, stride, t->vind[k]);
            for (int d = 0; d < 3; ++d) {
                if (lo[d] > p[d]) lo[d] = p[d];
                if (hi[d] < p[d]) hi[d] = p[d];
            }
        }
        return id;
    }
    int32_t* ind = t->vind + left;
    int32_t count = right - left;
    /* middleSplit_ */
    const float EPS = 0.00001f;
    float max_span = hi[0] - lo[0];
    for (int d = 1; d < 3; ++d) {
        float span = hi[d] - lo[d];
        if (span > max_span) max_span = span;
    }
    float max_spread = -1.0f;
    int cutfeat = 0;
    for (int d = 0; d < 3; ++d) {
        float span = hi[d] - lo[d];
        if (span > (1 - EPS) * max_span) {
            float mn, mx;
            kd_minmax(data, stride, ind, count, d, &mn, &mx);
            float spread = mx - mn;
            if (spread > max_spread) {
                cutfeat = d;
                max_spread = spread;
            }
        }
    }
    float split_val = (lo[cutfeat] + hi[cutfeat]) / 2;
    float mn, mx, cutval;
    kd_minmax(data, stride, ind, count, cutfeat, &mn, &mx);
    if (split_val < mn) cutval = mn;
    else if (split_val > mx) cutval = mx;
    else cutval = split_val;
    int32_t lim1, lim2, index;
    kd_plane_split(data, stride, ind, count, cutfeat, cutval, &lim1, &lim2);
    if (lim1 > count / 2) index = lim1;
    else if (lim2 < count / 2) index = lim2;
    else index = count / 2;

    float llo[3], lhi[3], rlo[3], rhi[3];
    memcpy(llo, lo, sizeof(llo)); memcpy(lhi, hi, sizeof(lhi));
    memcpy(rlo, lo, sizeof(rlo)); memcpy(rhi, hi, sizeof(rhi));
    lhi[cutfeat] = cutval;
    rlo[cutfeat] = cutval;
    int32_t c1 = kd_divide(t, data, stride, left, left + index, llo, lhi);
    int32_t c2 = kd_divide(t, data, stride, left + index, right, rlo, rhi);
    kd_node* nd = &t->nodes[id];
    nd->child1 = c1;
    nd->child2 = c2;
    nd->divfeat = cutfeat;
    nd->divlow = lhi[cutfeat];
    nd->divhigh = rlo[cutfeat];
    for (int d = 0; d < 3; ++d) {
        lo[d] = llo[d] < rlo[d] ? llo[d] : rlo[d];
        hi[d] = lhi[d] > rhi[d] ? lhi[d] : rhi[d];
    }
    return id;
}

static int kd_build(kd_tree* t, const float* data, int32_t m, int32_t stride) {
    memset(t, 0, sizeof(*t));
    t->m = m;
    t->vind = (int32_t*)malloc((size_t)m * sizeof(int32_t));
    t->pts = (float*)malloc((size_t)m * 3 * sizeof(float));
    if (!t->vind || !t->pts) return ST_E_NOMEM;
    for (int32_t i = 0; i < m; ++i) t->vind[i] = i;
    /* computeBoundingBox */
    for (int d = 0; d < 3; ++d) t->root_lo[d] = t->root_hi[d] = data[d];
    for (int32_t i = 1; i < m; ++i) {
        const float* p = kd_orig_pt(data, stride, i);
        for (int d = 0; d < 3; ++d) {
            if (p[d] < t->root_lo[d]) t->root_lo[d] = p[d];
            if (p[d] > t->root_hi[d]) t->root_hi[d] = p[d];
        }
    }
    float lo[3], hi[3];
    memcpy(lo, t->root_lo, sizeof(lo));
    memcpy(hi, t->root_hi, sizeof(hi));
    kd_divide(t, data, stride, 0, m, lo, hi);
    for (int32_t i = 0; i < m; ++i) memcpy(t->pts + 3 * (size_t)i, kd_orig_pt(data, stride, t->vind[i]), 3 * sizeof(float));
    return ST_OK;
}

static void kd_free(kd_tree* t) {
    free(t->pts);
    free(t->vind);
    free(t->nodes);
    memset(t, 0, sizeof(*t));
}

static _Thread_local int64_t g_leaf_visits; /* per thread: the CPU baseline runs pairs on a thread pool */
int64_t oracle_kdtree_leaf_visits(void) { return g_leaf_visits; }

typedef struct { float best; int32_t idx; } kd_result;

/* searchLevel with eps = 0.  Two documented deviations, both only for exact/near ties:
 *  (1) equal distances resolve to the LOWEST target index (FLANN: first found in traversal);
 *  (2) the subtree lower bound is loosened by 4 ulp before pruning, so float rounding of the
 *      incremental bound can never prune a point that ties the current best.
 * With these the tree returns exactly the brute-force argmin (tests/test_oracle.py checks). */
static void kd_search_level(const kd_tree* t, const float* q, int32_t node, float mindistsq, float dists[3],
                            kd_result* res) {
    const kd_node* nd = &t->nodes[node];
    if (nd->child1 < 0) {
        ++g_leaf_visits;
        for (int32_t i = nd->left; i < nd->right; ++i) {
            float dist = l2_simple(q, t->pts + 3 * (size_t)i);
            int32_t idx = t->vind[i];
            if (dist < res->best || (dist == res->best && idx < res->idx)) {
                res->best = dist;
                res->idx = idx;
            }
        }
        return;
    }
    int idx = nd->divfeat;
    float val = q[idx];
    float diff1 = val - nd->divlow;
    float diff2 = val - nd->divhigh;
    int32_t best_child, other_child;
    float cut_dist;
    if ((diff1 + diff2) < 0) {
        best_child = nd->child1;
        other_child = nd->child2;
        float dd = val - nd->divhigh;
        cut_dist = dd * dd; /* L2_Simple::accum_dist */
    } else {
        best_child = nd->child2;
        other_child = nd->child1;
        float dd = val - nd->divlow;
        cut_dist = dd * dd;
    }
    kd_search_level(t, q, best_child, mindistsq, dists, res);
    float dst = dists[idx];
    mindistsq = mindistsq + cut_dist - dst;
    dists[idx] = cut_dist;
    if (mindistsq * (1.0f - 4.0f * FLT_EPSILON) <= res->best) kd_search_level(t, q, other_child, mindistsq, dists, res);
    dists[idx] = dst;
}

static void kd_nearest(const kd_tree* t, const float* q, int32_t* idx, float* d2) {
    /* computeInitialDistances */
    float dists[3] = {0, 0, 0};
    float distsq = 0;
    for (int d = 0; d < 3; ++d) {
        if (q[d] < t->root_lo[d]) {
            float dd = q[d] - t->root_lo[d];
            dists[d] = dd * dd;
            distsq += dists[d];
        }
        if (q[d] > t->root_hi[d]) {
            float dd = q[d] - t->root_hi[d];
            dists[d] = dd * dd;
            distsq += dists[d];
        }
    }
    kd_result r = {INFINITY, -1};
    kd_search_level(t, q, 0, distsq, dists, &r);
    *idx = r.idx;
    *d2 = r.best;
}

static void brute_nearest(const float* tgt, int32_t m, int32_t stride, const float* q, int32_t* idx, float* d2) {
    float best = INFINITY;
    int32_t bi = -1;
    for (int32_t j = 0; j < m; ++j) {
        float d = l2_simple(q, tgt + (size_t)j * stride);
        if (d < best) { /* strict: first (lowest) index wins ties */
            best = d;
            bi = j;
        }
    }
    *idx = bi;
    *d2 = best;
}

/* ------------------------------------------------------------------------------------------ */
/* Transforms.  icp.hpp transformCloud:  pt_t = tr * (x,y,z,1) with Eigen's lazy packet product */
/* res = c0*x; res = c1*y + res; res = c2*z + res; res = c3*1 + res (SSE: mul then add).       */
/* transforms.hpp transformPointCloud (used by getFitnessScore) evaluates the same order.      */
static inline void xform_pt(const float T[16] /*col-major*/, const float* p, float* o) {
    float x = p[0], y = p[1], z = p[2];
    for (int r = 0; r < 3; ++r) {
        float acc = T[0 * 4 + r] * x;
        acc = T[1 * 4 + r] * y + acc;
        acc = T[2 * 4 + r] * z + acc;
        acc = T[3 * 4 + r] + acc;
        o[r] = acc;
    }
}

/* Matrix4f * Matrix4f (Eigen lazy product, k-ordered unfused accumulation). */
static void mat4_mul_f(const float A[16], const float B[16], float C[16]) {
    float R[16];
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) {
            float acc = A[0 * 4 + i] * B[j * 4 + 0];
            acc = A[1 * 4 + i] * B[j * 4 + 1] + acc;
            acc = A[2 * 4 + i] * B[j * 4 + 2] + acc;
            acc = A[3 * 4 + i] * B[j * 4 + 3] + acc;
            R[j * 4 + i] = acc;
        }
    memcpy(C, R, sizeof(R));
}

static void mat4_identity(float T[16]) {
    memset(T, 0, 16 * sizeof(float));
    T[0] = T[5] = T[10] = T[15] = 1.0f;
}

/* ------------------------------------------------------------------------------------------ */
/* 3x3 SVD by one-sided (Hestenes) Jacobi, generic over float/double.  Singular values sorted  */
/* descending like Eigen::JacobiSVD; U completed for rank < 3.  For rank >= 2 the Umeyama      */
/* rotation U*diag(1,1,s)*V^T is unique, so any exact SVD gives PCL's R up to rounding.        */
#define DEFINE_SVD3(NAME, REAL, SQRT, FABS, TOL, TINY)                                               \
    static void NAME(const REAL A[9] /*row-major*/, REAL U[9], REAL S[3], REAL V[9]) {              \
        REAL W[9];                                                                                   \
        for (int k = 0; k < 9; ++k) W[k] = A[k];                                                     \
        for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0) ? (REAL)1 : (REAL)0;                         \
        static const int P[3] = {0, 0, 1}, Q[3] = {1, 2, 2};                                         \
        for (int sweep = 0; sweep < 40; ++sweep) {                                                   \
            REAL off = 0;                                                                            \
            for (int r = 0; r < 3; ++r) {                                                            \
                int p = P[r], q = Q[r];                                                              \
                REAL al = 0, be = 0, ga = 0;                                                         \
                for (int k = 0; k < 3; ++k) {                                                        \
                    al += W[k * 3 + p] * W[k * 3 + p];                                               \
                    be += W[k * 3 + q] * W[k * 3 + q];                                               \
                    ga += W[k * 3 + p] * W[k * 3 + q];                                               \
                }                                                                                    \
                if (ga == 0) continue;                                                               \
                REAL nrm = SQRT(al * be);                                                            \
                if (nrm == 0) continue;                                                              \
                REAL rel = FABS(ga) / nrm;                                                           \
                if (rel > off) off = rel;                                                            \
                if (rel <= TOL) continue;                                                            \
                REAL zeta = (be - al) / (2 * ga);                                                    \
                REAL t = (zeta >= 0 ? (REAL)1 : (REAL)-1) / (FABS(zeta) + SQRT((REAL)1 + zeta * zeta)); \
                REAL c = (REAL)1 / SQRT((REAL)1 + t * t);                                            \
                REAL s = c * t;                                                                      \
                for (int k = 0; k < 3; ++k) {                                                        \
                    REAL wp = W[k * 3 + p], wq = W[k * 3 + q];                                       \
                    W[k * 3 + p] = c * wp - s * wq;                                                  \
                    W[k * 3 + q] = s * wp + c * wq;                                                  \
                    REAL vp = V[k * 3 + p], vq = V[k * 3 + q];                                       \
                    V[k * 3 + p] = c * vp - s * vq;                                                  \
                    V[k * 3 + q] = s * vp + c * vq;                                                  \
                }                                                                                    \
            }                                                                                        \
            if (off <= TOL) break;                                                                   \
        }                                                                                            \
        REAL sv[3];                                                                                  \
        for (int c = 0; c < 3; ++c)                                                                  \
            sv[c] = SQRT(W[0 * 3 + c] * W[0 * 3 + c] + W[1 * 3 + c] * W[1 * 3 + c] + W[2 * 3 + c] * W[2 * 3 + c]); \
        int ord[3] = {0, 1, 2};                                                                      \
        for (int i = 0; i < 3; ++i)                                                                  \
            for (int j = i + 1; j < 3; ++j)                                                          \
                if (sv[ord[j]] > sv[ord[i]]) {                                                       \
                    int tt = ord[i]; ord[i] = ord[j]; ord[j] = tt;                                   \
                }                                                                                    \
        REAL Vs[9], Ws[9];                                                                           \
        for (int c = 0; c < 3; ++c) {                                                                \
            S[c] = sv[ord[c]];                                                                       \
            for (int k = 0; k < 3; ++k) {                                                            \
                Vs[k * 3 + c] = V[k * 3 + ord[c]];                                                   \
                Ws[k * 3 + c] = W[k * 3 + ord[c]];                                                   \
            }                                                                                        \
        }                                                                                            \
        for (int k = 0; k < 9; ++k) V[k] = Vs[k];                                                    \
        int rank = 0;                                                                                \
        for (int c = 0; c < 3; ++c)                                                                  \
            if (S[c] > TINY * (S[0] > 0 ? S[0] : (REAL)1) && S[c] > 0) rank = c + 1;                 \
        for (int c = 0; c < rank; ++c)                                                               \
            for (int k = 0; k < 3; ++k) U[k * 3 + c] = Ws[k * 3 + c] / S[c];                         \
        if (rank == 0) {                                                                             \
            for (int k = 0; k < 9; ++k) U[k] = (k % 4 == 0) ? (REAL)1 : (REAL)0;                     \
        } else {                                                                                     \
            if (rank == 1) {                                                                         \
                /* any unit vector orthogonal to u0: cross with the least-aligned axis */            \
                int ax = 0;                                                                          \
                REAL amin = FABS(U[0]);                                                              \
                for (int k = 1; k < 3; ++k)                                                          \
                    if (FABS(U[k * 3]) < amin) { amin = FABS(U[k * 3]); ax = k; }                    \
                REAL e[3] = {0, 0, 0};                                                               \
                e[ax] = 1;                                                                           \
                REAL c0 = U[1 * 3] * e[2] - U[2 * 3] * e[1];                                         \
                REAL c1 = U[2 * 3] * e[0] - U[0 * 3] * e[2];                                         \
                REAL c2 = U[0 * 3] * e[1] - U[1 * 3] * e[0];                                         \
                REAL nn = SQRT(c0 * c0 + c1 * c1 + c2 * c2);                                         \
                U[0 * 3 + 1] = c0 / nn; U[1 * 3 + 1] = c1 / nn; U[2 * 3 + 1] = c2 / nn;              \
            }                                                                                        \
            if (rank <= 2) {                                                                         \
                U[0 * 3 + 2] = U[1 * 3 + 0] * U[2 * 3 + 1] - U[2 * 3 + 0] * U[1 * 3 + 1];            \
                U[1 * 3 + 2] = U[2 * 3 + 0] * U[0 * 3 + 1] - U[0 * 3 + 0] * U[2 * 3 + 1];            \
                U[2 * 3 + 2] = U[0 * 3 + 0] * U[1 * 3 + 1] - U[1 * 3 + 0] * U[0 * 3 + 1];            \
            }                                                                                        \
        }                                                                                            \
    }

DEFINE_SVD3(svd3_f64, double, sqrt, fabs, 1e-15, 1e-12)

#define DEFINE_DET3(NAME, REAL)                                                                     \
    static REAL NAME(const REAL M[9]) {                                                             \
        return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +            \
               M[2] * (M[3] * M[7] - M[4] * M[6]);                                                  \
    }
DEFINE_DET3(det3_f64, double)

/* R = U * diag(1,1,s) * V^T with s = -1 iff det(U)*det(V) < 0 (Eigen 3.3 umeyama). */
#define DEFINE_ROT(NAME, REAL, SVD, DET)                                                            \
    static void NAME(const REAL sigma[9], REAL R[9]) {                                              \
        REAL U[9], S[3], V[9];                                                                      \
        SVD(sigma, U, S, V);                                                                        \
        REAL d[3] = {1, 1, 1};                                                                      \
        if (DET(U) * DET(V) < 0) d[2] = -1;                                                         \
        for (int i = 0; i < 3; ++i)                                                                 \
            for (int j = 0; j < 3; ++j) {                                                           \
                REAL acc = 0;                                                                       \
                for (int k = 0; k < 3; ++k) acc += U[i * 3 + k] * d[k] * V[j * 3 + k];              \
                R[i * 3 + j] = acc;                                                                 \
            }                                                                                       \
    }
DEFINE_ROT(rot_f64, double, svd3_f64, det3_f64)

/* ------------------------------------------------------------------------------------------ */
/* PCL's float rotation, restated from Eigen 3.3 (the reference's PCL 1.8.1 / Eigen 3.3.4, SURVEY  */
/* §8c; iterative_closest_point.cpp:514 -> TransformationEstimationSVD -> pcl::umeyama ->          */
/* Eigen::umeyama, Geometry/Umeyama.h):                                                            */
/*   JacobiSVD<Matrix3f> svd(sigma, ComputeFullU | ComputeFullV)   (SVD/JacobiSVD.h compute())    */
/*   S = (1, 1, 1); if (det(U) * det(V) < 0) S(2) = -1;                                            */
/*   R = U * S.asDiagonal() * V^T                                                                   */
/* JacobiSVD for a square matrix takes no QR preconditioner: the matrix is divided by its largest  */
/* |coefficient|, then two-sided 2x2 Jacobi sweeps over (p, q) = (1, 0), (2, 0), (2, 1) run until  */
/* no off-diagonal pair exceeds max(FLT_MIN, 2 eps * the largest |diagonal| seen); each step takes  */
/* real_2x2_jacobi_svd (misc/RealSvd2x2.h): a rotation that symmetrises the 2x2 block, then         */
/* JacobiRotation::makeJacobi (Jacobi/Jacobi.h) for the symmetric block, j_left = rot1 * j_right^T,  */
/* applied to the work matrix's rows and columns and accumulated into U's and V's columns          */
/* (apply_rotation_in_the_plane: x' = c x + s y, y' = -s x + c y; a no-op for c = 1, s = 0).        */
/* Then negative diagonal entries flip U's column, the singular values are scaled back, and a      */
/* selection sort by swaps (maxCoeff: the first maximum; stops at a zero maximum) orders them.     */
/* The product R: Eigen's coefficient-based lazy product of fixed 3x3 operands sums each            */
/* coefficient with the unrolled redux, x0 + (x1 + x2), with x_k = (U(i,k) * S(k)) * V(j,k).        */
/* Every operation in float, unfused, in this order (SSE, no FMA).  Matrices row-major M[r*3+c].   */
typedef struct { float c, s; } jrot_f;

/* apply_rotation_in_the_plane(x, y, (c, s)) over 3 elements of stride `inc` */
static void plane_rot_f(float* x, float* y, int inc, float c, float s) {
    if (c == 1.0f && s == 0.0f) return;
    for (int i = 0; i < 3; ++i) {
        const float xi = x[i * inc], yi = y[i * inc];
        x[i * inc] = c * xi + s * yi;
        y[i * inc] = -s * xi + c * yi;
    }
}

/* misc/RealSvd2x2.h real_2x2_jacobi_svd(matrix, p, q, &j_left, &j_right) */
static void real_2x2_jacobi_svd_f(const float* W, int p, int q, jrot_f* jl, jrot_f* jr) {
    float m00 = W[p * 3 + p], m01 = W[p * 3 + q], m10 = W[q * 3 + p], m11 = W[q * 3 + q];
    jrot_f rot1;
    const float t = m00 + m11;
    const float d = m10 - m01;
    if (fabsf(d) < FLT_MIN) {
        rot1.s = 0.0f;
        rot1.c = 1.0f;
    } else {
        const float u = t / d;
        const float tmp = sqrtf(1.0f + u * u);
        rot1.s = 1.0f / tmp;
        rot1.c = u / tmp;
    }
    /* m.applyOnTheLeft(0, 1, rot1) */
    if (!(rot1.c == 1.0f && rot1.s == 0.0f)) {
        const float x0 = m00, y0 = m10, x1 = m01, y1 = m11;
        m00 = rot1.c * x0 + rot1.s * y0;
        m10 = -rot1.s * x0 + rot1.c * y0;
        m01 = rot1.c * x1 + rot1.s * y1;
        m11 = -rot1.s * x1 + rot1.c * y1;
    }
    (void)m10;
    /* j_right->makeJacobi(m, 0, 1): makeJacobi(x = m(0,0), y = m(0,1), z = m(1,1)) */
    const float deno = 2.0f * fabsf(m01);
    if (deno < FLT_MIN) {
        jr->c = 1.0f;
        jr->s = 0.0f;
    } else {
        const float tau = (m00 - m11) / deno;
        const float w = sqrtf(tau * tau + 1.0f);
        float tt;
        if (tau > 0.0f)
            tt = 1.0f / (tau + w);
        else
            tt = 1.0f / (tau - w);
        const float sign_t = tt > 0.0f ? 1.0f : -1.0f;
        const float n = 1.0f / sqrtf(tt * tt + 1.0f);
        jr->s = -sign_t * (m01 / fabsf(m01)) * fabsf(tt) * n;
        jr->c = n;
    }
    /* *j_left = rot1 * j_right->transpose(): (c1 c2 - s1 s2, c1 s2 + s1 c2) with (c2, s2) = (c_r, -s_r) */
    const float c2 = jr->c, s2 = -jr->s;
    jl->c = rot1.c * c2 - rot1.s * s2;
    jl->s = rot1.c * s2 + rot1.s * c2;
}

static float det3_eigen_f(const float* M) { /* LU/Determinant.h bruteforce_det3_helper */
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

/* JacobiSVD<Matrix3f>(A, ComputeFullU | ComputeFullV).  Returns 0, or -1 for a non-finite A. */
static int eigen_jacobi_svd3_f(const float A[9], float U[9], float S[3], float V[9]) {
    const float precision = 2.0f * FLT_EPSILON, consider_as_zero = FLT_MIN;
    float scale = fabsf(A[0]);
    for (int k = 1; k < 9; ++k) scale = scale < fabsf(A[k]) ? fabsf(A[k]) : scale;
    for (int k = 0; k < 9; ++k) U[k] = V[k] = (k % 4 == 0) ? 1.0f : 0.0f;
    if (!isfinite(scale)) {
        S[0] = S[1] = S[2] = 0.0f;
        return -1;
    }
    if (scale == 0.0f) scale = 1.0f;
    float W[9];
    for (int k = 0; k < 9; ++k) W[k] = A[k] / scale;
    float max_diag = fabsf(W[0]);
    max_diag = max_diag < fabsf(W[4]) ? fabsf(W[4]) : max_diag;
    max_diag = max_diag < fabsf(W[8]) ? fabsf(W[8]) : max_diag;
    int finished = 0;
    while (!finished) {
        finished = 1;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                const float pm = precision * max_diag;
                const float threshold = consider_as_zero < pm ? pm : consider_as_zero;
                if (fabsf(W[p * 3 + q]) > threshold || fabsf(W[q * 3 + p]) > threshold) {
                    finished = 0;
                    jrot_f jl, jr;
                    real_2x2_jacobi_svd_f(W, p, q, &jl, &jr);
                    plane_rot_f(W + p * 3, W + q * 3, 1, jl.c, jl.s); /* W.applyOnTheLeft(p, q, j_left) */
                    plane_rot_f(U + p, U + q, 3, jl.c, jl.s);         /* U.applyOnTheRight(p, q, j_left^T) */
                    plane_rot_f(W + p, W + q, 3, jr.c, -jr.s);        /* W.applyOnTheRight(p, q, j_right) */
                    plane_rot_f(V + p, V + q, 3, jr.c, -jr.s);        /* V.applyOnTheRight(p, q, j_right) */
                    const float ap = fabsf(W[p * 3 + p]), aq = fabsf(W[q * 3 + q]);
                    const float mpq = ap < aq ? aq : ap;
                    max_diag = max_diag < mpq ? mpq : max_diag;
                }
            }
    }
    for (int i = 0; i < 3; ++i) {
        const float a = W[i * 3 + i];
        S[i] = fabsf(a);
        if (a < 0.0f)
            for (int k = 0; k < 3; ++k) U[k * 3 + i] = -U[k * 3 + i];
    }
    for (int i = 0; i < 3; ++i) S[i] *= scale;
    for (int i = 0; i < 3; ++i) {
        int pos = i;
        float mx = S[i];
        for (int k = i + 1; k < 3; ++k)
            if (S[k] > mx) {
                mx = S[k];
                pos = k;
            }
        if (mx == 0.0f) break;
        if (pos != i) {
            float t = S[i];
            S[i] = S[pos];
            S[pos] = t;
            for (int k = 0; k < 3; ++k) {
                t = U[k * 3 + i]; U[k * 3 + i] = U[k * 3 + pos]; U[k * 3 + pos] = t;
                t = V[k * 3 + i]; V[k * 3 + i] = V[k * 3 + pos]; V[k * 3 + pos] = t;
            }
        }
    }
    return 0;
}

/* Eigen::umeyama's rotation (with_scaling = false), Scalar = float. */
static void rot_f32(const float sigma[9], float R[9]) {
    float U[9], S[3], V[9];
    eigen_jacobi_svd3_f(sigma, U, S, V);
    float d[3] = {1.0f, 1.0f, 1.0f};
    if (det3_eigen_f(U) * det3_eigen_f(V) < 0) d[2] = -1.0f;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const float x0 = (U[i * 3 + 0] * d[0]) * V[j * 3 + 0];
            const float x1 = (U[i * 3 + 1] * d[1]) * V[j * 3 + 1];
            const float x2 = (U[i * 3 + 2] * d[2]) * V[j * 3 + 2];
            R[i * 3 + j] = x0 + (x1 + x2);
        }
}

static inline double huber_w(double d2, double delta) {
    if (!(delta < INFINITY)) return 1.0;
    double r = sqrt(d2);
    return r <= delta ? 1.0 : delta / r;
}

/* The depth blocking of the sigma product (Eigen 3.3, single thread).
 *
 * pcl::umeyama (PCL 1.8.1 common/impl/eigen.hpp) forms
 *     sigma = one_over_n * dst_demean * src_demean.transpose()
 * with dst_demean a 3 x n row-major float matrix.  Eigen 3.3 evaluates a product with two small
 * fixed dimensions and a dynamic depth as a GEMM (product_type_selector<Small,Small,Large>) once
 * depth + 3 + 3 >= 20 (generic_product_impl<...,GemmProduct>::evalTo; below that a coefficient-based
 * product, whose vectorised redux order depends on the operands' alignment — not replicated here,
 * those n < 14 registrations use the GEMM form too).  The scalar factor is popped off the lhs
 * (blas_traits of scalar * matrix), so alpha = one_over_n, and sigma is zeroed before the GEMM adds
 * into it.  general_matrix_matrix_product::run walks the depth in panels of kc
 * (computeProductBlockingSizes -> evaluateProductBlockingSizesHeuristic) and calls gebp once per
 * panel; with 3 rows (< LhsProgress = 4) and 3 columns (< nr = 4) gebp takes its scalar tail path
 * ("remaining columns", one coefficient at a time):
 *     C0 = 0; for k in panel: C0 = pmadd(A0, B0, C0) = A0*B0 + C0;   res(i, j) += alpha * C0;
 * so every coefficient is a sequential float chain per panel, the panels added into sigma in order.
 * kc: max_kc = ((l1 - mr*nr*4) / (mr*4 + nr*4)) & ~7 (KcFactor 1, k_peeling 8), then for depth
 * k > max_kc, kc = max_kc when max_kc divides k, else max_kc - 8 * ((max_kc - 1 - k % max_kc) /
 * (8 * (k / max_kc + 1))) — the last panel as large as possible for the same number of panels.
 * Assumptions (the reference's build is not in this image): float, SSE without FMA (packet of 4,
 * gebp_traits<float>::mr = default_mr = 8, nr = 4), L1 data cache 32 KiB as queried by CPUID on
 * the node's x86-64 host: max_kc = 680, and n = 8192 runs 13 panels of kc = 632; n = 2048, 4 of
 * 520; n <= 680 one panel (the plain sequential chain).  eigen_l1_bytes / eigen_gebp_mr override
 * the two host facts; eigen_l1_bytes < 0 turns the blocking off (one panel of depth n). */
int32_t oracle_sigma_max_kc(int32_t l1, int32_t mr) {
    if (l1 < 0) return INT32_MAX;
    if (l1 == 0) l1 = 32768;
    if (mr <= 0) mr = 8;
    const int32_t nr = 4, k_peeling = 8;
    const int32_t k_div = mr * 4 + nr * 4, k_sub = mr * nr * 4;
    int32_t max_kc = ((l1 - k_sub) / k_div) & ~(k_peeling - 1);
    return max_kc < 1 ? 1 : max_kc;
}

int32_t oracle_sigma_kc(int32_t k, int32_t max_kc) {
    if (max_kc <= 0 || k < 48 || k <= max_kc) return k;  /* early return for max(k, 3, 3) < 48; no depth blocking */
    const int32_t r = k % max_kc;
    return r == 0 ? max_kc : max_kc - 8 * ((max_kc - 1 - r) / (8 * (k / max_kc + 1)));
}

/* Umeyama, Scalar = float (Eigen 3.3 Geometry/Umeyama.h as called by
 * TransformationEstimationSVD::estimateRigidTransformation with use_umeyama_).
 * rowwise().sum() on a 3xN column-major matrix has a strided inner access and is a sequential
 * float fold in Eigen 3.3; sigma is the blocked GEMM above: per panel of kc correspondences a
 * sequential float chain of d'_a * s'_b products from +0, added as one_over_n * chain into sigma
 * (from +0) in panel order.  Huber (build-only, no PCL counterpart): the same panels over the
 * products (w * d'_a) * s'_b, one_over_n = 1 / Σw. */
static void umeyama_f32(const float* X, const float* tgt, int32_t tgt_stride, const int32_t* cq,
                        const int32_t* cm, const float* cd2, int32_t n, double huber, int32_t max_kc,
                        float T[16], oracle_trace* tr, int it) {
    float one_over_n;
    float ms[3] = {0, 0, 0}, md[3] = {0, 0, 0};
    float sigma[9] = {0};
    int weighted = huber < INFINITY;
    if (!weighted) {
        one_over_n = 1.0f / (float)n;
        for (int k = 0; k < 3; ++k) {
            float a = X[(size_t)cq[0] * 3 + k], b = tgt[(size_t)cm[0] * tgt_stride + k];
            for (int32_t i = 1; i < n; ++i) {
                a = a + X[(size_t)cq[i] * 3 + k];
                b = b + tgt[(size_t)cm[i] * tgt_stride + k];
            }
            ms[k] = a * one_over_n;
            md[k] = b * one_over_n;
        }
    } else {
        float sw = 0;
        for (int32_t i = 0; i < n; ++i) {
            float w = (float)huber_w(cd2[i], huber);
            sw += w;
            for (int k = 0; k < 3; ++k) {
                ms[k] += w * X[(size_t)cq[i] * 3 + k];
                md[k] += w * tgt[(size_t)cm[i] * tgt_stride + k];
            }
        }
        one_over_n = 1.0f / sw;
        for (int k = 0; k < 3; ++k) { ms[k] *= one_over_n; md[k] *= one_over_n; }
    }
    const int32_t kc = oracle_sigma_kc(n, max_kc);
    for (int32_t k0 = 0; k0 < n; k0 += kc) {
        const int32_t k1 = n - k0 < kc ? n : k0 + kc;
        float c[9] = {0};
        for (int32_t i = k0; i < k1; ++i) {
            float s[3], d[3];
            for (int k = 0; k < 3; ++k) {
                s[k] = X[(size_t)cq[i] * 3 + k] - ms[k];
                d[k] = tgt[(size_t)cm[i] * tgt_stride + k] - md[k];
            }
            if (weighted) {
                const float w = (float)huber_w(cd2[i], huber);
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) c[a * 3 + b] = (w * d[a]) * s[b] + c[a * 3 + b];
            } else {
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) c[a * 3 + b] = d[a] * s[b] + c[a * 3 + b];
            }
        }
        for (int k = 0; k < 9; ++k) sigma[k] = sigma[k] + one_over_n * c[k];
    }
    float R[9];
    rot_f32(sigma, R);
    mat4_identity(T);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) T[j * 4 + i] = R[i * 3 + j];
    for (int i = 0; i < 3; ++i) {
        float rs = R[i * 3 + 0] * ms[0];
        rs = R[i * 3 + 1] * ms[1] + rs;
        rs = R[i * 3 + 2] * ms[2] + rs;
        T[12 + i] = md[i] - rs;
    }
    if (tr) {
        if (tr->sigma) for (int k = 0; k < 9; ++k) tr->sigma[it * 9 + k] = sigma[k];
        if (tr->mu_src) for (int k = 0; k < 3; ++k) tr->mu_src[it * 3 + k] = ms[k];
        if (tr->mu_dst) for (int k = 0; k < 3; ++k) tr->mu_dst[it * 3 + k] = md[k];
    }
}

/* Umeyama in double: the product's arithmetic (icp4r_kernels.hip, solve_pair).  Raw moments
 * Σw, Σw·s, Σw·d, Σw·d·sᵀ accumulated in double from float inputs, then
 * μ = Σw·x / Σw,  sigma = Σw·d·sᵀ/Σw − μd·μsᵀ,  R from the double SVD,  t = μd − R·μs. */
static void umeyama_f64(const float* X, const float* tgt, int32_t tgt_stride, const int32_t* cq,
                        const int32_t* cm, const float* cd2, int32_t n, double huber, float T[16],
                        oracle_trace* tr, int it) {
    double sw = 0, ss[3] = {0, 0, 0}, sd[3] = {0, 0, 0}, sds[9] = {0};
    for (int32_t i = 0; i < n; ++i) {
        double w = huber_w(cd2[i], huber);
        double s[3], d[3];
        for (int k = 0; k < 3; ++k) {
            s[k] = X[(size_t)cq[i] * 3 + k];
            d[k] = tgt[(size_t)cm[i] * tgt_stride + k];
        }
        sw += w;
        for (int k = 0; k < 3; ++k) {
            ss[k] += w * s[k];
            sd[k] += w * d[k];
        }
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) sds[a * 3 + b] += w * d[a] * s[b];
    }
    double ms[3], md[3], sigma[9], R[9];
    for (int k = 0; k < 3; ++k) {
        ms[k] = ss[k] / sw;
        md[k] = sd[k] / sw;
    }
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) sigma[a * 3 + b] = sds[a * 3 + b] / sw - md[a] * ms[b];
    rot_f64(sigma, R);
    mat4_identity(T);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T[j * 4 + i] = (float)R[i * 3 + j];
        T[12 + i] = (float)(md[i] - (R[i * 3 + 0] * ms[0] + R[i * 3 + 1] * ms[1] + R[i * 3 + 2] * ms[2]));
    }
    if (tr) {
        if (tr->sigma) for (int k = 0; k < 9; ++k) tr->sigma[it * 9 + k] = sigma[k];
        if (tr->mu_src) for (int k = 0; k < 3; ++k) tr->mu_src[it * 3 + k] = ms[k];
        if (tr->mu_dst) for (int k = 0; k < 3; ++k) tr->mu_dst[it * 3 + k] = md[k];
    }
}

static int cloud_finite(const float* c, int32_t n, int32_t stride) {
    for (int32_t i = 0; i < n; ++i) {
        const float* p = c + (size_t)i * stride;
        if (!isfinite(p[0]) || !isfinite(p[1]) || !isfinite(p[2])) return 0;
    }
    return 1;
}

typedef struct nn_ctx {
    int mode;
    kd_tree tree;
    const float* tgt;
    int32_t m, stride;
} nn_ctx;

static int nn_init(nn_ctx* c, int mode, const float* tgt, int32_t m, int32_t stride) {
    c->mode = mode;
    c->tgt = tgt;
    c->m = m;
    c->stride = stride;
    memset(&c->tree, 0, sizeof(c->tree));
    if (mode == ORACLE_NN_KDTREE) return kd_build(&c->tree, tgt, m, stride);
    return ST_OK;
}
static inline void nn_query(const nn_ctx* c, const float* q, int32_t* idx, float* d2) {
    if (c->mode == ORACLE_NN_KDTREE) kd_nearest(&c->tree, q, idx, d2);
    else brute_nearest(c->tgt, c->m, c->stride, q, idx, d2);
}
static void nn_free(nn_ctx* c) {
    if (c->mode == ORACLE_NN_KDTREE) kd_free(&c->tree);
}

/* Registration::getFitnessScore(max_range): Y = final * input; mean of NN d² over d² <= max_range. */
static double fitness_with(const nn_ctx* nn, const float* src, int32_t n, int32_t stride, const float T[16],
                           double max_range) {
    double fitness_score = 0.0;
    int32_t nr = 0;
    for (int32_t i = 0; i < n; ++i) {
        float y[3];
        xform_pt(T, src + (size_t)i * stride, y);
        int32_t j;
        float d2;
        nn_query(nn, y, &j, &d2);
        if (d2 <= max_range) {
            fitness_score += d2;
            nr++;
        }
    }
    return nr > 0 ? fitness_score / nr : DBL_MAX;
}

int oracle_nearest(const float* q, int32_t n, int32_t q_stride, const float* tgt, int32_t m, int32_t tgt_stride,
                   int32_t nn_mode, int32_t* idx_out, float* d2_out) {
    if (n < 0 || m <= 0 || !q || !tgt) return ST_E_INVALID;
    nn_ctx nn;
    if (nn_init(&nn, nn_mode, tgt, m, tgt_stride) != ST_OK) return ST_E_NOMEM;
    g_leaf_visits = 0;
    for (int32_t i = 0; i < n; ++i) nn_query(&nn, q + (size_t)i * q_stride, idx_out + i, d2_out + i);
    nn_free(&nn);
    return ST_OK;
}

double oracle_fitness(const float* src, int32_t n, int32_t src_stride, const float* tgt, int32_t m,
                      int32_t tgt_stride, const float* T, double max_range, int32_t nn_mode) {
    if (m <= 0) return DBL_MAX;
    nn_ctx nn;
    if (nn_init(&nn, nn_mode, tgt, m, tgt_stride) != ST_OK) return DBL_MAX;
    double f = fitness_with(&nn, src, n, src_stride, T, max_range);
    nn_free(&nn);
    return f;
}

/* DefaultConvergenceCriteria<float>::hasConverged, including its early
 * returns: correspondences_prev_mse_ is only updated when no criterion fired. */
static int has_converged(const oracle_params* p, int32_t iterations, const float Tinc[16], double mse,
                         double rot_thr, double trans_thr, double* prev_mse, int32_t* similar, int32_t* state) {
    *state = CONV_NOT_CONVERGED;
    if (iterations >= p->max_iterations) {
        *state = CONV_ITERATIONS;
        return 1;
    }
    /* transformation_ is the ICP's Matrix4 (= Matrix4f): both expressions are evaluated in float and
     * only their results widened to double */
    const float tr = Tinc[0] + Tinc[5] + Tinc[10] - 1;
    double cos_angle = 0.5 * tr;
    const float tsq = Tinc[12] * Tinc[12] + Tinc[13] * Tinc[13] + Tinc[14] * Tinc[14];
    double translation_sqr = tsq;
    if (cos_angle >= rot_thr && translation_sqr <= trans_thr) {
        if (*similar < p->max_iterations_similar_transforms) {
            ++*similar;
            return 0;
        }
        *similar = 0;
        *state = CONV_TRANSFORM;
        return 1;
    }
    if (fabs(mse - *prev_mse) < p->mse_threshold_absolute) {
        if (*similar < p->max_iterations_similar_transforms) {
            ++*similar;
            return 0;
        }
        *similar = 0;
        *state = CONV_ABS_MSE;
        return 1;
    }
    if (fabs(mse - *prev_mse) / *prev_mse < p->euclidean_fitness_epsilon) {
        if (*similar < p->max_iterations_similar_transforms) {
            ++*similar;
            return 0;
        }
        *similar = 0;
        *state = CONV_REL_MSE;
        return 1;
    }
    *prev_mse = mse;
    return 0;
}

/* IterativeClosestPoint::computeTransformation. */
int oracle_align(const float* src, int32_t n, int32_t src_stride, const float* tgt, int32_t m, int32_t tgt_stride,
                 const float* guess, const oracle_params* pin, oracle_result* r, float* aligned_out,
                 oracle_trace* tr) {
    oracle_params p;
    if (pin) p = *pin;
    else oracle_params_default(&p);
    memset(r, 0, sizeof(*r));
    mat4_identity(r->T);
    r->fitness = DBL_MAX;
    if (n < 0 || m < 0 || (n > 0 && !src) || (m > 0 && !tgt) || src_stride < 3 || tgt_stride < 3) {
        r->status = ST_E_INVALID;
        return r->status;
    }
    /* Registration::initCompute: "No input target dataset was given!" → align returns early. */
    if (m == 0) {
        r->status = ST_E_EMPTY;
        return r->status;
    }
    if (!cloud_finite(src, n, src_stride) || !cloud_finite(tgt, m, tgt_stride)) {
        r->status = ST_E_NONFINITE;
        return r->status;
    }
    float final_T[16], Tinc[16];
    mat4_identity(final_T);
    int guess_is_identity = 1;
    if (guess) {
        float I[16];
        mat4_identity(I);
        guess_is_identity = memcmp(guess, I, sizeof(I)) == 0; /* Matrix4::Identity() != guess */
        memcpy(final_T, guess, sizeof(final_T));
    }
    float* X = (float*)malloc((size_t)(n > 0 ? n : 1) * 3 * sizeof(float));
    int32_t* cq = (int32_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
    int32_t* cm = (int32_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
    float* cd = (float*)malloc((size_t)(n > 0 ? n : 1) * sizeof(float));
    nn_ctx nn;
    if (!X || !cq || !cm || !cd || nn_init(&nn, p.nn, tgt, m, tgt_stride) != ST_OK) {
        free(X); free(cq); free(cm); free(cd);
        r->status = ST_E_NOMEM;
        return r->status;
    }
    for (int32_t i = 0; i < n; ++i) {
        const float* s = src + (size_t)i * src_stride;
        if (guess_is_identity) {
            X[3 * i + 0] = s[0]; X[3 * i + 1] = s[1]; X[3 * i + 2] = s[2];
        } else {
            xform_pt(final_T, s, X + 3 * (size_t)i);
        }
    }
    mat4_identity(Tinc);
    const double max_dist_sqr = p.max_correspondence_distance * p.max_correspondence_distance;
    const double rot_thr = p.transformation_rotation_epsilon > 0 ? p.transformation_rotation_epsilon
                                                                 : 1.0 - p.transformation_epsilon;
    const double trans_thr = p.transformation_epsilon;
    double prev_mse = DBL_MAX;
    int32_t nr_iterations = 0, similar = 0, converged = 0, state = CONV_NOT_CONVERGED, status = ST_OK;
    int32_t cnt = 0;
    g_leaf_visits = 0;
    do {
        /* determineCorrespondences(correspondences, corr_dist_threshold_) */
        cnt = 0;
        for (int32_t i = 0; i < n; ++i) {
            int32_t j;
            float d2;
            nn_query(&nn, X + 3 * (size_t)i, &j, &d2);
            if ((double)d2 > max_dist_sqr) continue;
            cq[cnt] = i;
            cm[cnt] = j;
            cd[cnt] = d2;
            ++cnt;
        }
        if (cnt < p.min_correspondences) {
            /* PCL_ERROR "Not enough correspondences found. Relax your threshold parameters." */
            state = CONV_NO_CORRESPONDENCES;
            converged = 0;
            status = ST_E_TOO_FEW_CORR;
            break;
        }
        if (p.numerics == ORACLE_NUM_F64)
            umeyama_f64(X, tgt, tgt_stride, cq, cm, cd, cnt, p.huber_delta, Tinc, tr, nr_iterations);
        else
            umeyama_f32(X, tgt, tgt_stride, cq, cm, cd, cnt, p.huber_delta,
                        oracle_sigma_max_kc(p.eigen_l1_bytes, p.eigen_gebp_mr), Tinc, tr, nr_iterations);
        /* transformCloud(*input_transformed, *input_transformed, transformation_) */
        for (int32_t i = 0; i < n; ++i) {
            float o[3];
            xform_pt(Tinc, X + 3 * (size_t)i, o);
            X[3 * i + 0] = o[0]; X[3 * i + 1] = o[1]; X[3 * i + 2] = o[2];
        }
        /* final_transformation_ = transformation_ * final_transformation_ */
        mat4_mul_f(Tinc, final_T, final_T);
        ++nr_iterations;
        /* DefaultConvergenceCriteria::hasConverged */
        double mse = 0.0;
        for (int32_t i = 0; i < cnt; ++i) mse += cd[i];
        mse /= (double)cnt;
        if (tr) {
            if (tr->T_inc) memcpy(tr->T_inc + 16 * (nr_iterations - 1), Tinc, 16 * sizeof(float));
            if (tr->T_final) memcpy(tr->T_final + 16 * (nr_iterations - 1), final_T, 16 * sizeof(float));
            if (tr->mse) tr->mse[nr_iterations - 1] = mse;
            if (tr->ncorr) tr->ncorr[nr_iterations - 1] = cnt;
        }
        converged = has_converged(&p, nr_iterations, Tinc, mse, rot_thr, trans_thr, &prev_mse, &similar, &state);
    } while (!converged);

    memcpy(r->T, final_T, sizeof(final_T));
    r->iterations = nr_iterations;
    r->converged = converged;
    r->convergence_state = state;
    r->n_correspondences = cnt;
    r->status = status;
    if (p.compute_fitness) r->fitness = fitness_with(&nn, src, n, src_stride, final_T, p.fitness_max_range);
    if (aligned_out) {
        for (int32_t i = 0; i < n; ++i) {
            const float* s = src + (size_t)i * src_stride;
            xform_pt(final_T, s, aligned_out + 4 * (size_t)i);
            aligned_out[4 * i + 3] = src_stride > 3 ? s[3] : 0.0f; /* intensity copied through */
        }
    }
    nn_free(&nn);
    free(X); free(cq); free(cm); free(cd);
    return status;
}

/* test hook: the float Umeyama rotation of a 3x3 sigma (row-major) */
void oracle_rot_f32(const float* sigma, float* R) { rot_f32(sigma, R); }
