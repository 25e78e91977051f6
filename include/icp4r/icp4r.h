/*
 * icp4r.h — C ABI of the MI355X-native ICP registration core (drop-in boundary).
 *
 * Replaces the PCL 1.8.1 default rigid ICP the reference node instantiates at
 * /root/reference/src/iterative_closest_point.cpp:510-521:
 *
 *     pcl::IterativeClosestPoint<pcl::PointXYZI, pcl::PointXYZI> icp;     // :510
 *     icp.setInputSource(cloud_src_in);                                  // :511
 *     icp.setInputTarget(cloud_tar_in);                                  // :512
 *     icp.align(*Final);                                                 // :514
 *     icp.hasConverged(); icp.getFitnessScore();                         // :516, :520
 *     icp.getFinalTransformation().cast<double>();                       // :521
 *
 * and the same getter surface consumed at /root/reference/src/radar_odometry.cpp:399-412.
 * The C++ facade include/icp4r/pcl_compat.hpp maps those method names onto these entry points;
 * INTEGRATION.md shows the binding a maintainer adds.
 *
 * Conventions: plain pointers and sizes only; every entry returns int status (0 = OK, < 0 = error,
 * see icp4r_status) and records a message retrievable with icp4r_last_error() (thread-local).
 * Matrices are 4x4 float COLUMN-MAJOR (= Eigen::Matrix4f storage; Eigen::Map<Matrix4f>(T) works).
 * A context owns one HIP device's buffers and stream; calls on one context are serialized.
 */
#ifndef ICP4R_H
#define ICP4R_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ICP4R_ABI_VERSION 6

typedef enum icp4r_status {
    ICP4R_OK = 0,
    ICP4R_E_INVALID = -1,      /* bad argument / stride / size                                  */
    ICP4R_E_EMPTY = -2,        /* empty target: Registration::initCompute fails, align returns  */
    ICP4R_E_TOO_FEW_CORR = -3, /* |C| < min_correspondences: PCL_ERROR, converged = false       */
    ICP4R_E_NONFINITE = -4,    /* NaN/Inf coordinate in an input cloud (rejected up front)      */
    ICP4R_E_HIP = -5,          /* HIP runtime failure (message has the HIP error string)        */
    ICP4R_E_RCCL = -6,         /* RCCL failure in the multi-GPU entries (icp4r_multi.h), incl.
                                  asynchronous errors reported by ncclCommGetAsyncError        */
    ICP4R_E_NOMEM = -7,        /* device or host allocation failed                               */
    ICP4R_E_TOO_LARGE = -8     /* a size exceeds what the selected kernel supports               */
} icp4r_status;

/* pcl::registration::DefaultConvergenceCriteria<float>::ConvergenceState, same order. */
typedef enum icp4r_convergence_state {
    ICP4R_CONV_NOT_CONVERGED = 0,
    ICP4R_CONV_ITERATIONS = 1,
    ICP4R_CONV_TRANSFORM = 2,
    ICP4R_CONV_ABS_MSE = 3,
    ICP4R_CONV_REL_MSE = 4,
    ICP4R_CONV_NO_CORRESPONDENCES = 5
} icp4r_convergence_state;

/* Umeyama arithmetic.
 * PCL: PCL's Scalar = float Umeyama restated operation by operation: centroids as the sequential
 *      float folds Eigen 3.3 performs, the 3x3 cross-covariance as its depth-blocked GEMM (one
 *      sequential chain per panel of kc correspondences, panels added in order), float one-sided Jacobi
 *      SVD, R and t as Matrix4f, MSE and fitness as sequential double sums.  Bit-identical to the
 *      float restatement in oracle/ (tests assert equal bits); the default.
 * F64: every moment summed in double (more accurate than PCL; differs from it by PCL's own
 *      float-centroid noise, up to ~2e-4 m on 8k-point clouds). */
typedef enum icp4r_numerics { ICP4R_NUMERICS_PCL = 0, ICP4R_NUMERICS_F64 = 1 } icp4r_numerics;

/* Correspondence search.  All modes return the exact nearest neighbour under FLANN's
 * L2_Simple<float> distance ((dx*dx + dy*dy) + dz*dz, float, unfused); ties -> lowest index. */
typedef enum icp4r_nn_mode {
    ICP4R_NN_AUTO = 0,         /* PRUNED when the largest target has >= 512 points, else BRUTE      */
    ICP4R_NN_BRUTE = 1,        /* exhaustive scan, target streamed through the scalar cache, FP32    */
    ICP4R_NN_BRUTE_PACKED = 2, /* same scan, two queries per v_pk_{add,mul}_f32 (identical results) */
    ICP4R_NN_PRUNED = 3        /* Morton-ordered target blocks with bounding boxes, exact search     */
} icp4r_nn_mode;

typedef struct icp4r_params {
    int32_t max_iterations;                    /* setMaximumIterations;           PCL default 10        */
    int32_t min_correspondences;               /* min_number_correspondences_;    3                     */
    double max_correspondence_distance;        /* setMaxCorrespondenceDistance;   sqrt(DBL_MAX)         */
    double transformation_epsilon;             /* setTransformationEpsilon;       0                     */
    double transformation_rotation_epsilon;    /* setTransformationRotationEpsilon; 0 (-> 1 - eps)      */
    double euclidean_fitness_epsilon;          /* setEuclideanFitnessEpsilon;     -DBL_MAX              */
    double mse_threshold_absolute;             /* DefaultConvergenceCriteria;     1e-12 (< 0: disabled) */
    int32_t max_iterations_similar_transforms; /* DefaultConvergenceCriteria;     0                     */
    int32_t numerics;                          /* icp4r_numerics;                 ICP4R_NUMERICS_PCL    */
    int32_t nn_mode;                           /* icp4r_nn_mode;                  ICP4R_NN_AUTO         */
    int32_t compute_fitness;                   /* 1: getFitnessScore(fitness_max_range) computed once   */
    double huber_delta;                        /* build extension (no PCL counterpart); +inf == PCL     */
    double fitness_max_range;                  /* getFitnessScore(max_range);     DBL_MAX               */
    /* PCL numerics: Eigen 3.3 evaluates umeyama's sigma = one_over_n * dst_demean * src_demean^T as a
     * GEMM whose depth (the correspondences) is cut into panels of kc, each a sequential float chain
     * added into sigma in order.  kc follows from two facts of the reference's host:   */
    int32_t eigen_l1_bytes;                    /* L1d size Eigen queried: 0 = 32768; < 0 = no panels    */
    int32_t eigen_gebp_mr;                     /* gebp_traits<float>::mr: 0 = 8 (SSE, no FMA)           */
    /* Known deviation: with fewer than 14 correspondences Eigen evaluates sigma coefficient by
     * coefficient (lazyproduct, an alignment-dependent vectorised redux); the GEMM panel form above is
     * used for every |C|.  Both host facts are assumptions about the node's build: parity with PCL
     * itself is unpinned (the reference holds no fixtures).                            */
    int32_t reserved[6];
} icp4r_params;

typedef struct icp4r_result {
    float T[16];               /* getFinalTransformation(), column-major                     */
    double fitness;            /* getFitnessScore(fitness_max_range); DBL_MAX if no point    */
    int32_t iterations;        /* nr_iterations_                                              */
    int32_t converged;         /* hasConverged()                                              */
    int32_t status;            /* icp4r_status of this pair                                   */
    int32_t convergence_state; /* icp4r_convergence_state                                     */
    int32_t n_correspondences; /* |C| of the last iteration                                   */
    int32_t reserved;
} icp4r_result; /* 96 bytes */

/* Device-resident batch: every cloud is float4 (x, y, z, intensity) = 16 B/point in HBM. */
typedef struct icp4r_batch {
    const float* src;        /* device: concatenated source clouds, float4 per point          */
    const float* tgt;        /* device: concatenated target clouds, float4 per point          */
    const int64_t* src_off;  /* device[npairs]: first point of pair p's source                */
    const int32_t* src_n;    /* device[npairs]                                                */
    const int64_t* tgt_off;  /* device[npairs]                                                */
    const int32_t* tgt_n;    /* device[npairs]                                                */
    const float* guess;      /* device[npairs*16] column-major, or NULL (identity)            */
    float* aligned;          /* device: optional output clouds, same layout as src, or NULL   */
    int32_t npairs;
    int32_t max_src_n;       /* host-known upper bound of src_n[] (selects the kernel)        */
    int32_t max_tgt_n;       /* host-known upper bound of tgt_n[]                             */
    int32_t reserved;
} icp4r_batch;

typedef struct icp4r_ctx icp4r_ctx;

const char* icp4r_version(void);
int icp4r_abi_version(void);
const char* icp4r_last_error(void);
void icp4r_params_default(icp4r_params* p);
int icp4r_device_count(int* count);

/* A context on one HIP device (its stream, workspace and plan options).  device = ICP4R_NO_DEVICE
 * makes a context without a device, for icp4r_plan queries and plan options only: no HIP call, and
 * every device call on it fails. */
#define ICP4R_NO_DEVICE (-1)
int icp4r_create(icp4r_ctx** out, int device);
int icp4r_destroy(icp4r_ctx* ctx);

/* Registration::align(output, guess) — synchronous, host buffers.  src/tgt: n/m points with a
 * stride in bytes (PCL PointXYZI: 32, float4: 16, the .bin record: 20); x, y, z are the first
 * three floats of a point, intensity the fourth when stride >= 16.  guess: 16 floats
 * column-major or NULL.  aligned_out (optional): n points written with out_stride_bytes,
 * x, y, z = transformCloud(input, final), intensity copied when out_stride_bytes >= 16. */
int icp4r_align(icp4r_ctx* ctx, const float* src, int32_t n, int32_t src_stride_bytes, const float* tgt,
                int32_t m, int32_t tgt_stride_bytes, const float* guess, const icp4r_params* params,
                icp4r_result* out, float* aligned_out, int32_t out_stride_bytes);

/* Many pairs, device-resident (inputs already in HBM), asynchronous on `hip_stream`
 * (a hipStream_t; NULL = the context's stream).  results: device[npairs]. */
int icp4r_align_batch_device(icp4r_ctx* ctx, const icp4r_batch* batch, const icp4r_params* params,
                             icp4r_result* results, void* hip_stream);

/* Many pairs from host buffers (float4 per point, concatenated), synchronous. */
int icp4r_align_batch_host(icp4r_ctx* ctx, const float* src, const int64_t* src_off, const int32_t* src_n,
                           const float* tgt, const int64_t* tgt_off, const int32_t* tgt_n, int32_t npairs,
                           const float* guess, const icp4r_params* params, icp4r_result* results);

/* Registration::getFitnessScore(max_range) for a given transform (host buffers). */
int icp4r_fitness(icp4r_ctx* ctx, const float* src, int32_t n, int32_t src_stride_bytes, const float* tgt,
                  int32_t m, int32_t tgt_stride_bytes, const float* T, double max_range, double* fitness);

/* CorrespondenceEstimation::determineCorrespondences at infinite distance: exact 1-NN of every
 * query in the target (host buffers).  idx_out[n], d2_out[n]. */
int icp4r_nearest(icp4r_ctx* ctx, const float* query, int32_t n, int32_t query_stride_bytes, const float* tgt,
                  int32_t m, int32_t tgt_stride_bytes, int32_t* idx_out, float* d2_out);

/* Synchronize the context's stream (or `hip_stream` if non-NULL). */
int icp4r_synchronize(icp4r_ctx* ctx, void* hip_stream);

/* Device-time accounting with HIP events on the launch stream (used by bench.py for the roofline):
 * icp4r_kernel_time_ms: average duration of the NN kernel launches (the batched search
 *                       nn_lds_kernel, the tiled search nn_tile_kernel, or the whole NN launch of the
 *                       other plans) recorded since the last reset, and how many there were — the
 *                       update's launches are icp4r_stage_time_ms(ICP4R_STAGE_UPDATE); which of the
 *                       two dominates a step depends on the plan (at C3 it is the update);
 * icp4r_batch_time_ms:  average duration of whole registration calls (all launches of a batch). */
int icp4r_kernel_time_ms(icp4r_ctx* ctx, double* avg_ms, int32_t* launches);
int icp4r_batch_time_ms(icp4r_ctx* ctx, double* avg_ms, int32_t* calls);
int icp4r_kernel_time_reset(icp4r_ctx* ctx);
/* Per-kernel timing (the events behind icp4r_kernel_time_ms / icp4r_stage_time_ms for NN, NN_TEST and
 * UPDATE): off by default — each event record between two kernels costs device time (an 8k pair's
 * registration 1.89 ms without them, 2.19 ms with them; a 1024-pair batch 7.01 vs 7.31 ms).  The
 * whole-call events (icp4r_batch_time_ms) are always recorded. */
int icp4r_set_kernel_timing(icp4r_ctx* ctx, int32_t enable);

/* Average device time of one stage of the registrations since the last reset (HIP events on the
 * launch stream), and how many launches it averages.  ICP4R_STAGE_NN is what icp4r_kernel_time_ms
 * reports: the batched search kernel (nn_lds_kernel) of the LDS plan, nn_tile_kernel of the tiled
 * plan, the whole NN launch of the others; ICP4R_STAGE_NN_TEST the cached-neighbour test kernel; ICP4R_STAGE_UPDATE the Umeyama /
 * convergence update (generalized ICP: its Gauss-Newton / LM iteration kernel); ICP4R_STAGE_BATCH a
 * whole registration call; ICP4R_STAGE_GICP_COV the generalized ICP's covariance kernel. */
typedef enum icp4r_stage {
    ICP4R_STAGE_NN = 0,
    ICP4R_STAGE_NN_TEST = 1,
    ICP4R_STAGE_UPDATE = 2,
    ICP4R_STAGE_BATCH = 3,
    ICP4R_STAGE_GICP_COV = 4
} icp4r_stage;
int icp4r_stage_time_ms(icp4r_ctx* ctx, int32_t stage, double* avg_ms, int32_t* launches);

/* Work the NN kernels performed since the last icp4r_kernel_time_reset — the algorithmic work
 * behind the roofline's `achieved`: distance evaluations (query x target; brute force exactly n*m
 * per pair and pass, the pruned search a small fraction) and bounding-box tests (query x box, the
 * pruned search only; may be NULL).  Synchronises the context's device.  The counters are
 * diagnostics, counted only by registrations that ran with plan option "counters" = 1 or with
 * per-kernel timing on (icp4r_set_kernel_timing); otherwise they stay at zero. */
int icp4r_nn_counters(icp4r_ctx* ctx, uint64_t* evaluations, uint64_t* box_tests);

/* Queries whose nearest neighbour the cached-neighbour test proved unchanged without a search
 * (icp4r_plan_info.cache) since the last icp4r_kernel_time_reset; each counts as one evaluation
 * in icp4r_nn_counters.  Synchronises the context's device. */
int icp4r_nn_cache_hits(icp4r_ctx* ctx, uint64_t* hits);

/* All NN work counters since the last icp4r_kernel_time_reset (synchronises the device). */
typedef struct icp4r_nn_stats_t {
    uint64_t evaluations;             /* distance evaluations (a cache hit counts one)          */
    uint64_t box_tests;               /* point-to-box lower-bound tests of the pruned searches  */
    uint64_t cache_hits;              /* queries the cached-neighbour test resolved             */
    uint64_t cache_tested;            /* queries the cached-neighbour test examined             */
    uint64_t records_written_by_test; /* correspondence records the test kernel wrote (32 B)    */
    uint64_t tested_in_update;        /* of cache_tested: tested in the update kernel's tail    */
    uint64_t hits_in_update;          /* of cache_hits: resolved there                          */
    uint64_t second_chance_hits;      /* search-list queries resolved inside the cached NN's kd
                                         leaf (nn_lds_kernel, before any traversal)           */
} icp4r_nn_stats_t;
int icp4r_nn_stats(icp4r_ctx* ctx, icp4r_nn_stats_t* out);

/* Plan options (A/B experiments and diagnostics): how a registration is laid out on the device —
 * which search and update kernels run, grid shapes, pair groups on streams, debug stamps.  No option
 * changes a result (the parity tests assert bit-identical registrations across them), and an option
 * never set keeps its measured-best default (DESIGN.md §6 lists every name and default).  Options
 * belong to a context and apply to its later calls; the library reads no environment variable.
 * An unknown name, or a value outside the option's range (e.g. "groups" above 3: a fourth pair
 * group would share a hardware queue with the third), is ICP4R_E_INVALID.
 * icp4r_get_plan_option: the value in effect for the context's calls (the default when never set)
 * and *is_set (may be NULL). */
int icp4r_set_plan_option(icp4r_ctx* ctx, const char* name, int32_t value);
int icp4r_get_plan_option(const icp4r_ctx* ctx, const char* name, int32_t* value, int32_t* is_set);
int icp4r_reset_plan_options(icp4r_ctx* ctx);

/* Launch geometry the batch path picks for a shape — exposed for tests and the benchmark report. */
typedef struct icp4r_plan_info {
    int32_t pruned;     /* 1: ICP4R_NN_PRUNED kernel, 0: brute force                 */
    int32_t q;          /* queries per lane                                          */
    int32_t splits;     /* brute force: target splits per pair                       */
    int32_t leaf;       /* pruned: targets per block                                 */
    int32_t lds;        /* pruned batch kernel with the target set in LDS (per-query
                           work lists); used for >= 256 pairs with <= 8192 targets    */
    int32_t cache;      /* lds: cached-neighbour test (a query keeps its previous NN
                           without a search when a second-nearest bound proves it;
                           exact); off with plan option nn_cache = 0                  */
    int64_t nn_blocks;  /* workgroups of one NN launch                               */
    int32_t solo;       /* 1: a PCL-numerics registration of this shape runs whole in one
                           workgroup per pair (solo_kernel): targets <= 8192, sources <=
                           1024 by default (plan option solo = 1: up to 16384), and a
                           plan that does not take the batched LDS search (fewer than
                           256 pairs, or nn_lds = 0); solo = 0: never                 */
    int32_t wide_update; /* 1: the PCL-numerics update runs one 1024-thread workgroup per pair
                           (fold_update_wide_kernel: at most one pair per CU, no fused cache
                           test, PCL numerics); off with plan option wide_update = 0    */
    int32_t res_update; /* 1 (ABI 6): the batched plan's update holds each pair on chip
                           (fold_update_res_kernel: the fused cache test, sources <= 8192,
                           PCL numerics) for unweighted registrations without a distance
                           threshold (PCL's defaults; the others take fold_update_kernel);
                           off with plan option res_update = 0                        */
    int32_t held_update; /* 1 (ABI 6): the wide update keeps each correspondence record in a
                           register from pass A to pass B (fold_update_held_kernel: sources
                           <= 8960); off with plan option held_update = 0             */
} icp4r_plan_info;
/* ctx: whose plan options and CU count apply (NULL: the defaults and 256 CUs); numerics:
 * ICP4R_NUMERICS_PCL / _F64, as icp4r_params.numerics. */
int icp4r_plan(const icp4r_ctx* ctx, int32_t npairs, int32_t max_src_n, int32_t max_tgt_n, int32_t nn_mode,
               int32_t numerics, icp4r_plan_info* out);

#ifdef __cplusplus
}
#endif

#endif /* ICP4R_H */
