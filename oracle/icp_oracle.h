/*
 * icp_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of PCL 1.8.1 default rigid ICP as the reference node calls it
 * (src/iterative_closest_point.cpp:510-521 → pcl::IterativeClosestPoint<PointXYZI,PointXYZI>).
 * The arithmetic lives in third-party PCL 1.8.1 / FLANN 1.9.1 / Eigen 3.3.4, none of which are
 * vendored in /root/reference or present in this image; SURVEY.md Appendix A is the binding spec
 * restated here function by function (see the comments in icp_oracle.c).
 *
 * This library is the CHECKER and the CPU baseline ("kind": "port") — never the product.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Parity status: UNPINNED by the reference itself (the reference has no tests, no fixtures and its
 * ICP cannot be built here).  Pinned instead by analytic known-answer tests and by an independently
 * written numpy/scipy twin (tests/golden/make_golden.py) — see DESIGN.md §Oracle.
 */
#ifndef ICP_ORACLE_H
#define ICP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Umeyama arithmetic.  PCL runs TransformationEstimationSVD with Scalar = float
 * (icp.h default template arg); ORACLE_NUM_F32 restates that.  ORACLE_NUM_F64 accumulates the
 * same sums in double and solves the 3x3 SVD in double — the arithmetic the HIP product uses. */
enum { ORACLE_NUM_F32 = 0, ORACLE_NUM_F64 = 1 };
/* Correspondence search.  KDTREE follows FLANN KDTreeSingleIndex (leaf 15, middle split, exact
 * eps = 0) as used by pcl::KdTreeFLANN; BRUTE is the exhaustive scan.  Both return the exact NN
 * under FLANN's L2_Simple<float> distance; ties resolve to the lowest target index. */
enum { ORACLE_NN_KDTREE = 0, ORACLE_NN_BRUTE = 1 };

typedef struct oracle_params {
    int32_t max_iterations;                 /* Registration::max_iterations_            = 10       */
    int32_t min_correspondences;            /* Registration::min_number_correspondences_ = 3       */
    double  max_correspondence_distance;    /* Registration::corr_dist_threshold_ = sqrt(DBL_MAX)  */
    double  transformation_epsilon;         /* Registration::transformation_epsilon_    = 0        */
    double  transformation_rotation_epsilon;/* Registration::transformation_rotation_epsilon_ = 0 */
    double  euclidean_fitness_epsilon;      /* Registration::euclidean_fitness_epsilon_ = -DBL_MAX */
    double  mse_threshold_absolute;         /* DefaultConvergenceCriteria::mse_threshold_absolute_ = 1e-12 */
    int32_t max_iterations_similar_transforms; /* DefaultConvergenceCriteria = 0 */
    int32_t numerics;                       /* ORACLE_NUM_* */
    int32_t nn;                             /* ORACLE_NN_* */
    int32_t compute_fitness;                /* 1: run getFitnessScore(fitness_max_range) once */
    double  huber_delta;                    /* build-only extension; +inf == PCL                 */
    double  fitness_max_range;              /* getFitnessScore(max_range) default DBL_MAX         */
    /* The sigma GEMM's depth blocking (Eigen 3.3 evaluateProductBlockingSizesHeuristic, see
     * umeyama_f32): the L1 data cache size Eigen queried on the reference host (0: 32768, the x86
     * L1d of the ROS-melodic era; < 0: no blocking, one sequential chain) and gebp_traits<float>::mr
     * of its SIMD build (0: 8 = SSE without FMA). */
    int32_t eigen_l1_bytes;
    int32_t eigen_gebp_mr;
} oracle_params;

/* The sigma GEMM's depth blocking (umeyama_f32): Eigen's largest panel depth for these host
 * facts, and the panel depth kc it picks for a depth of k correspondences. */
int32_t oracle_sigma_max_kc(int32_t l1_bytes, int32_t gebp_mr);
int32_t oracle_sigma_kc(int32_t k, int32_t max_kc);

typedef struct oracle_result {
    float   T[16];              /* final_transformation_, column-major (Eigen storage order) */
    double  fitness;            /* getFitnessScore()                                         */
    int32_t iterations;         /* nr_iterations_                                            */
    int32_t converged;          /* converged_                                                */
    int32_t status;             /* 0 ok, <0 error (same codes as icp4r.h)                    */
    int32_t convergence_state;  /* DefaultConvergenceCriteria::ConvergenceState              */
    int32_t n_correspondences;  /* |C| of the last iteration                                 */
    int32_t reserved;
} oracle_result;

/* Optional per-iteration trace (arrays sized max_iterations; may be NULL). */
typedef struct oracle_trace {
    float*  T_inc;      /* [iters][16] column-major increment (transformation_) */
    float*  T_final;    /* [iters][16] column-major final_transformation_ after the iteration */
    double* mse;        /* [iters] mean of correspondence d^2 (pre-update) */
    int32_t* ncorr;     /* [iters] */
    double* sigma;      /* [iters][9] row-major cross-covariance (dst x src^T)/n, for golden checks */
    double* mu_src;     /* [iters][3] */
    double* mu_dst;     /* [iters][3] */
} oracle_trace;

void oracle_params_default(oracle_params* p);

/* Registration::align(output, guess) with IterativeClosestPoint::computeTransformation.
 * Clouds are float arrays with a stride in floats (PCL PointXYZI = 8 floats, float4 = 4,
 * the .bin record = 5).  guess: 16 floats column-major or NULL (identity).
 * aligned_out: optional n*4 floats (x,y,z,intensity) = transformCloud(input, final). */
int oracle_align(const float* src, int32_t n, int32_t src_stride,
                 const float* tgt, int32_t m, int32_t tgt_stride,
                 const float* guess, const oracle_params* p,
                 oracle_result* r, float* aligned_out, oracle_trace* trace);

/* CorrespondenceEstimation::determineCorrespondences at max_distance = +inf: exact 1-NN. */
int oracle_nearest(const float* q, int32_t n, int32_t q_stride,
                   const float* tgt, int32_t m, int32_t tgt_stride,
                   int32_t nn_mode, int32_t* idx_out, float* d2_out);

/* Registration::getFitnessScore(max_range) for a given final transformation. */
double oracle_fitness(const float* src, int32_t n, int32_t src_stride,
                      const float* tgt, int32_t m, int32_t tgt_stride,
                      const float* T_colmajor, double max_range, int32_t nn_mode);

/* Test hook: float Umeyama rotation R = U diag(1,1,s) V^T of a row-major 3x3 sigma. */
void oracle_rot_f32(const float* sigma, float* R);

/* Statistics of the last kd-tree search (for the CPU-baseline report). */
int64_t oracle_kdtree_leaf_visits(void);

#ifdef __cplusplus
}
#endif
#endif
