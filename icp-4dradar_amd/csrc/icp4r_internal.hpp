// icp4r_internal.hpp — types shared by the C-ABI host code and the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "icp4r/icp4r.h"
#include "icp4r_math.hpp"

namespace icp4r {

constexpr int kNNWG = 256;        // threads per NN workgroup (4 waves)
constexpr int kMaxQ = 16;         // register-resident queries per lane in nn_kernel (instantiated)
constexpr int kDefaultQ = 4;      // default cap (tools/tune_sweep.py)
constexpr int kFoldChunk = 1024;  // points per LDS chunk of the sequential centroid fold

constexpr int kNumericsPCL = ICP4R_NUMERICS_PCL;
constexpr int kNumericsF64 = ICP4R_NUMERICS_F64;
constexpr int kStatusEmpty = ICP4R_E_EMPTY;
constexpr int kStatusTooFewCorr = ICP4R_E_TOO_FEW_CORR;
constexpr int kStatusNonFinite = ICP4R_E_NONFINITE;

// per-pair loop phase
constexpr int kPhaseActive = 0;     // iterating
constexpr int kPhaseConverged = 1;  // hasConverged() fired
constexpr int kPhaseFailed = 2;     // |C| < min_correspondences (PCL: converged_ = false, break)
constexpr int kPhaseInvalid = 3;    // empty target / non-finite input: nothing computed

using Result = icp4r_result;

struct KParams {
    ConvParams conv;
    int32_t min_corr;
    int32_t numerics;
    int32_t compute_fitness;
    float max_d2;          // reject a correspondence iff d2 > max_d2 (float image of max_dist^2)
    double huber_delta;    // +inf: unweighted (PCL)
    double fit_max_range;  // getFitnessScore(max_range): keep d2 <= max_range
};

struct PairArgs {
    const float4* src;
    const float4* tgt;
    const int64_t* src_off;
    const int32_t* src_n;
    const int64_t* tgt_off;
    const int32_t* tgt_n;
    const float* guess;  // npairs*16 column-major or nullptr
    float4* aligned;     // optional
    Result* results;
    KParams kp;
};

// Device-resident per-pair loop state (ICP members of PCL: transformation_, final_transformation_,
// nr_iterations_, converged_, and DefaultConvergenceCriteria's prev MSE / similar counter).
struct PairState {
    float T_inc[16];
    float final_T[16];
    double prev_mse;
    int32_t similar;
    int32_t conv_state;
    int32_t iterations;
    int32_t phase;
    int32_t status;
    int32_t ncorr;
};

// Workspace: X (input_transformed) and the NN results, pair p at [p * x_stride, ...).
struct WorkArgs {
    float4* X;
    float* nn_d2;       // [splits][npairs * x_stride]
    int32_t* nn_idx;    // [splits][npairs * x_stride]
    PairState* state;   // [npairs]
    int64_t x_stride;   // >= max source points per pair
    int64_t slot_stride;  // npairs * x_stride
    int32_t splits;     // target splits per pair (1 for batches; >1 for single-pair latency)
};

hipError_t launch_init(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st);
hipError_t launch_nn(int q, bool packed, const PairArgs& a, const WorkArgs& w, int npairs, int max_n,
                     int fitness_pass, hipStream_t st);
hipError_t launch_update(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st);
hipError_t launch_fitness_prep(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st);
hipError_t launch_finish(const PairArgs& a, const WorkArgs& w, int npairs, hipStream_t st);
hipError_t launch_rot_f32(const float* sigma, float* R, int k, hipStream_t st);
hipError_t launch_nn_query(const float4* q, int n, const float4* tgt, int m, const float* T, int32_t* idx, float* d2,
                           hipStream_t st);

}  // namespace icp4r
