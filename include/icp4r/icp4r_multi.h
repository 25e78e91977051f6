/*
 * icp4r_multi.h — the batched multi-GPU mode of the ICP core (BASELINE.json
 * configs[3]: 8192 independent scan pairs over 8 GPUs with a final RCCL gather over xGMI).
 *
 * The reference registers one pair per frame (/root/reference/src/iterative_closest_point.cpp:510-521)
 * and has no multi-GPU path of its own; a replay host that registers a whole sequence at once
 * (icp4radar_replay --batch, the host of :510-521) shards the independent pairs over devices.
 * Pairs are independent, so the data path has no collective: shard r owns the contiguous, balanced
 * block of global pairs [first, first + count) given by icp4r_shard, and the only exchange is the
 * gather of the 96-byte result rows.
 *
 * Two forms:
 *  - one process driving several devices (icp4r_align_batch_multi): one context per device, one
 *    host thread per context, results copied back into the caller's host array in global order;
 *  - one process per GPU (the torch.distributed / MPI layout): an RCCL communicator per rank
 *    (icp4r_comm_*), the ranks' device-written rows all-gathered into every rank's device buffer
 *    (ncclAllGather), so each rank holds every pose in global order.
 * Every entry returns an icp4r_status; RCCL failures, including asynchronous ones reported by
 * ncclCommGetAsyncError, return ICP4R_E_RCCL with RCCL's message in icp4r_last_error().
 */
#ifndef ICP4R_MULTI_H
#define ICP4R_MULTI_H

#include "icp4r/icp4r.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ICP4R_COMM_ID_BYTES 128 /* = NCCL_UNIQUE_ID_BYTES */

typedef struct icp4r_comm icp4r_comm;

/* Shard `rank` of `nranks` over `npairs` global pairs: first = rank * (npairs / nranks) +
 * min(rank, npairs % nranks), count = npairs / nranks + (rank < npairs % nranks). */
int icp4r_shard(int32_t npairs, int32_t nranks, int32_t rank, int32_t* first, int32_t* count);

/* One process, `nctx` distinct contexts (normally one per device; two contexts may share a device,
 * but one context listed twice is ICP4R_E_INVALID: each context's workspace and stream serve one
 * host thread at a time): context k
 * registers shard k of the batch (icp4r_align_batch_host's arguments, float4 points) on its own
 * device and stream, all shards concurrently (one host thread each); results[npairs] on the host in
 * global pair order, bit-identical to one icp4r_align_batch_host call over the whole batch.
 * Each context uploads only the point range its shard's offsets cover. */
int icp4r_align_batch_multi(icp4r_ctx* const* ctxs, int32_t nctx, const float* src, const int64_t* src_off,
                            const int32_t* src_n, const float* tgt, const int64_t* tgt_off, const int32_t* tgt_n,
                            int32_t npairs, const float* guess, const icp4r_params* params, icp4r_result* results);

/* RCCL unique id for a new communicator (ncclGetUniqueId); rank 0 makes it and hands it to the others. */
int icp4r_comm_unique_id(unsigned char id[ICP4R_COMM_ID_BYTES]);

/* This process' rank of an nranks-rank communicator on ctx's device (ncclCommInitRank; every rank
 * calls it with the same id; blocks until all have joined).  The communicator uses ctx's stream
 * unless a call passes another. */
int icp4r_comm_create(icp4r_comm** out, icp4r_ctx* ctx, int32_t nranks, int32_t rank,
                      const unsigned char id[ICP4R_COMM_ID_BYTES]);
/* Waits for the communicator's last gather, then frees it.  It does not touch the context it was
 * created on, so it may run before or after icp4r_destroy of that context. */
int icp4r_comm_destroy(icp4r_comm* comm);
int icp4r_comm_rank(const icp4r_comm* comm, int32_t* rank, int32_t* nranks);

/* ICP4R_E_RCCL (with RCCL's message) if the communicator has an asynchronous error, else ICP4R_OK.
 * Non-blocking (ncclCommGetAsyncError). */
int icp4r_comm_check(icp4r_comm* comm);

/* All-gather of result rows: this rank's icp4r_shard(npairs, nranks, rank) rows, `shard_rows`
 * (device), land at gathered[first, first + count) on every rank (`gathered`: device, npairs rows).
 * Asynchronous on hip_stream (NULL: the context's stream); equal shards gather in place, unequal
 * ones through a padded staging buffer and one copy per rank.  Gathers of one communicator may run
 * on different streams: a gather waits for the previous one (an event on its stream) before it
 * reuses the staging buffers.  The context's plan option "gather_padded" = 1 at icp4r_comm_create
 * (a test switch) sends every gather through the padded branch.  A communicator may outlive its
 * context: after icp4r_destroy(ctx) a gather needs an explicit hip_stream (NULL is
 * ICP4R_E_INVALID), and icp4r_align_batch_sharded is ICP4R_E_INVALID. */
int icp4r_gather_results(icp4r_comm* comm, const icp4r_result* shard_rows, int32_t npairs, icp4r_result* gathered,
                         void* hip_stream);

/* The C4 step on one rank: register this rank's shard (a device batch whose npairs is its
 * icp4r_shard count of npairs_total) into shard_results (device), then gather every rank's rows into
 * gathered (device, npairs_total rows).  Asynchronous on hip_stream. */
int icp4r_align_batch_sharded(icp4r_comm* comm, const icp4r_batch* shard, int32_t npairs_total,
                              const icp4r_params* params, icp4r_result* shard_results, icp4r_result* gathered,
                              void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* ICP4R_MULTI_H */
