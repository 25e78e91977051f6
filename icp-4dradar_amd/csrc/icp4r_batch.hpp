// icp4r_batch.hpp — the batch registration pipeline's host helpers (icp4r_capi.cpp), shared with
// the other entry points that run the same device machinery (icp4r_gicp.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "icp4r_host.hpp"
#include "icp4r_internal.hpp"

namespace icp4r_pipe {

struct Plan {
    int q;
    bool packed;  // brute force: v_pk_* FP32 sweep (two queries per register pair)
    int splits;   // brute force: target splits
    bool pruned;  // Morton-block pruned exact search
    bool lds;     // pruned, batched: nn_lds_kernel (whole target set in LDS, per-query work lists)
    bool cache;   // lds: cached-neighbour test + second-nearest search (plan option nn_cache = 0 disables)
    int leaf;     // pruned: targets per block
    int chunk_sb; // pruned (streamed): superblocks per target chunk (<= 64)
    int chunks;   // pruned (streamed): target chunks searched by separate waves (merged by atomicMin)
    bool tile;    // pruned, not batched: nn_tile_kernel (LDS target tiles x query parts; plan option nn_tile = 0: the stream)
    int max_m;    // the plan's largest target (tile grid)
    int tile_run; // tile: queries per wave run (64, 32, 16): 16 runs per workgroup
    bool solo;    // run_pairs: the whole registration of each pair in one workgroup (solo_kernel; PCL
                  // numerics, one target tile, sources <= kCacheMaxN; plan option solo = 0 disables)
    int64_t blocks;
};

// Plan options (icp4r_set_plan_option): the A/B and diagnostic switches of the
// pipeline, set per context through the C ABI.  None changes a result (the parity tests assert
// bit-identical registrations across them); an option never set takes the call site's default, the
// measured best.  The library reads no environment variable.
enum PlanOpt : int {
    kOptNnQ, kOptLeaf, kOptChunkSb, kOptNnLds, kOptNnCache, kOptNnTile, kOptTileRun, kOptSolo, kOptXpad,
    kOptPhaseTicks, kOptKd, kOptMortonMwg, kOptPart, kOptSrcOrder, kOptFuseSeed, kOptTileOwn, kOptTileDefer,
    kOptGroups, kOptSearchCuDiv, kOptFuseTest, kOptFuseOrder, kOptSumsTail, kOptWideUpdate, kOptGatherPadded,
    kOptGicpCovBrute, kOptFoldKeys, kOptGicpSpec, kOptGicpGrid, kOptGicpKnnLanes, kOptResUpdate, kOptHeldUpdate,
    kOptFitXform, kOptCounters, kOptStageSel, kNumPlanOpts
};
static_assert(kNumPlanOpts <= 64, "icp4r_ctx::plan_set is a 64-bit mask");
extern const char* const kPlanOptNames[kNumPlanOpts];
// The context's value of option k, or dflt when it was never set (ctx may be NULL: dflt).
int opt(const icp4r_ctx* ctx, PlanOpt k, int dflt);

// Geometry of the NN pass for a batch shape.  allow_lds = false keeps the batched LDS search out (a
// caller whose index strides exceed what it stages, icp4r_gicp.cpp), so every other field of the
// plan is the one of the plan that runs.
// registration = true: the plan of run_pairs for PCL numerics (solo_kernel where it applies).
Plan make_plan(const icp4r_ctx* ctx, int npairs, int max_n, int max_m, int nn_mode = ICP4R_NN_AUTO,
               bool allow_lds = true, bool registration = false);
// icp4r_params -> the kernels' KParams (validates).
int make_kparams(const icp4r_params* p, icp4r::KParams* kp);
// Size the context's workspace for a plan and fill WorkArgs.
int setup_work(icp4r_ctx* ctx, const Plan& pl, int npairs, int max_n, int max_m, bool corr, hipStream_t st,
               icp4r::WorkArgs& w);
// One NN pass over every pair the pass wants (timed with the context's NN events).
int nn_pass(icp4r_ctx* ctx, const Plan& pl, const icp4r::PairArgs& a, const icp4r::WorkArgs& w, int npairs, int max_n,
            int fitness_pass, int first, hipStream_t st, int ncu = 0, int test_fused = 0, int pass = -1,
            int ordered = 0);
int next_event(std::vector<icp4r_host::EventPair>& v, size_t& used, icp4r_host::EventPair** out);

}  // namespace icp4r_pipe
