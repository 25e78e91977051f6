// icp4r_multi.cpp — the batched multi-GPU mode (include/icp4r/icp4r_multi.h).
//
// Pairs are independent: shards are contiguous blocks of global pairs, registered with the
// single-device pipeline, and the only exchange is the gather of the 96-B result rows — host copies
// when one process drives every device, an RCCL all-gather (xGMI) when each GPU has its own process.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <thread>
#include <vector>

#include "icp4r/icp4r.h"
#include "icp4r/icp4r_multi.h"
#include "icp4r_batch.hpp"
#include "icp4r_host.hpp"

using icp4r_host::DevBuf;
using icp4r_host::fail;

struct icp4r_comm {
    icp4r_ctx* ctx = nullptr;  // NULL once icp4r_destroy(ctx) ran (icp4r_host::comm_detach)
    int device = 0;
    ncclComm_t nccl = nullptr;
    int32_t rank = 0, nranks = 1;
    DevBuf send, recv;  // padded staging for unequal shards
    // The last gather's completion on the stream it ran on: a gather on another stream waits for it
    // before it reuses the staging buffers, and icp4r_comm_destroy waits for it before freeing them.
    hipEvent_t done = nullptr;
    bool done_recorded = false;
    hipStream_t last = nullptr;
    // Test switch (the context's plan option gather_padded at creation): every gather takes the padded
    // branch, so a one-rank communicator exercises the staging path that only unequal multi-rank
    // shards reach.
    bool force_padded = false;
};

#define RCCL_TRY(expr)                                                                                     \
    do {                                                                                                   \
        ncclResult_t _r = (expr);                                                                          \
        if (_r != ncclSuccess)                                                                             \
            return fail(ICP4R_E_RCCL, "%s: %s (%s:%d)", #expr, ncclGetErrorString(_r), __FILE__, __LINE__); \
    } while (0)

namespace icp4r_host {
void comm_detach(icp4r_comm* c) { c->ctx = nullptr; }
}  // namespace icp4r_host

namespace {

void shard_of(int32_t npairs, int32_t nranks, int32_t rank, int32_t* first, int32_t* count) {
    const int32_t base = npairs / nranks, extra = npairs % nranks;
    *first = rank * base + (rank < extra ? rank : extra);
    *count = base + (rank < extra ? 1 : 0);
}

}  // namespace

extern "C" {

int icp4r_shard(int32_t npairs, int32_t nranks, int32_t rank, int32_t* first, int32_t* count) {
    if (npairs < 0 || nranks <= 0 || rank < 0 || rank >= nranks || !first || !count)
        return fail(ICP4R_E_INVALID, "icp4r_shard: npairs %d, rank %d of %d", npairs, rank, nranks);
    shard_of(npairs, nranks, rank, first, count);
    return ICP4R_OK;
}

int icp4r_align_batch_multi(icp4r_ctx* const* ctxs, int32_t nctx, const float* src, const int64_t* src_off,
                            const int32_t* src_n, const float* tgt, const int64_t* tgt_off, const int32_t* tgt_n,
                            int32_t npairs, const float* guess, const icp4r_params* params, icp4r_result* results) {
    if (!ctxs || nctx <= 0 || npairs < 0 || !results) return fail(ICP4R_E_INVALID, "icp4r_align_batch_multi: bad arguments");
    for (int32_t k = 0; k < nctx; ++k) {
        if (!ctxs[k]) return fail(ICP4R_E_INVALID, "icp4r_align_batch_multi: context %d is NULL", k);
        // one host thread per context: a context listed twice would share its workspace and stream
        for (int32_t j = 0; j < k; ++j)
            if (ctxs[j] == ctxs[k])
                return fail(ICP4R_E_INVALID, "icp4r_align_batch_multi: contexts %d and %d are the same context", j, k);
    }
    if (npairs == 0) return ICP4R_OK;
    if (!src_off || !src_n || !tgt_off || !tgt_n) return fail(ICP4R_E_INVALID, "NULL offset/count array");
    icp4r_host::Range range("icp4r_align_batch_multi");
    // one host thread per context: each sets its device and runs its shard on its own stream
    std::vector<int> rc((size_t)nctx, ICP4R_OK);
    std::vector<std::string> msg((size_t)nctx);
    auto work = [&](int32_t k) {
        int32_t f, c;
        shard_of(npairs, nctx, k, &f, &c);
        if (c == 0) return;
        rc[k] = icp4r_align_batch_host(ctxs[k], src, src_off + f, src_n + f, tgt, tgt_off + f, tgt_n + f, c,
                                       guess ? guess + 16 * (size_t)f : nullptr, params, results + f);
        if (rc[k] != ICP4R_OK) msg[k] = icp4r_last_error();  // (thread-local: carried to the caller)
    };
    std::vector<std::thread> th;
    th.reserve((size_t)nctx);
    for (int32_t k = 1; k < nctx; ++k) th.emplace_back(work, k);
    work(0);
    for (auto& t : th) t.join();
    for (int32_t k = 0; k < nctx; ++k)
        if (rc[k] != ICP4R_OK) return fail(rc[k], "shard %d (device %d): %s", k, ctxs[k]->device, msg[k].c_str());
    return ICP4R_OK;
}

int icp4r_comm_unique_id(unsigned char id[ICP4R_COMM_ID_BYTES]) {
    if (!id) return fail(ICP4R_E_INVALID, "id is NULL");
    static_assert(sizeof(ncclUniqueId) == ICP4R_COMM_ID_BYTES, "RCCL unique id size");
    ncclUniqueId u;
    RCCL_TRY(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof(u));
    return ICP4R_OK;
}

int icp4r_comm_create(icp4r_comm** out, icp4r_ctx* ctx, int32_t nranks, int32_t rank,
                      const unsigned char id[ICP4R_COMM_ID_BYTES]) {
    if (!out || !ctx || !id || nranks <= 0 || rank < 0 || rank >= nranks)
        return fail(ICP4R_E_INVALID, "icp4r_comm_create: bad arguments (rank %d of %d)", rank, nranks);
    *out = nullptr;
    HIP_TRY(hipSetDevice(ctx->device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    icp4r_comm* c = new icp4r_comm();
    c->ctx = ctx;
    c->device = ctx->device;
    c->rank = rank;
    c->nranks = nranks;
    // (plan option gather_padded, copied from the context at creation: the padded all-gather branch on
    // any communicator, so one GPU can test it)
    c->force_padded = icp4r_pipe::opt(ctx, icp4r_pipe::kOptGatherPadded, 0) != 0;
    if (hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return fail(ICP4R_E_HIP, "icp4r_comm_create: hipEventCreate failed");
    }
    const ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, u, rank);
    if (r != ncclSuccess) {
        (void)hipEventDestroy(c->done);
        delete c;
        return fail(ICP4R_E_RCCL, "ncclCommInitRank (rank %d of %d, device %d): %s", rank, nranks, ctx->device,
                    ncclGetErrorString(r));
    }
    ctx->comms.push_back(c);
    *out = c;
    return ICP4R_OK;
}

int icp4r_comm_destroy(icp4r_comm* comm) {
    if (!comm) return ICP4R_OK;
    if (comm->ctx) {
        auto& v = comm->ctx->comms;
        for (size_t k = 0; k < v.size(); ++k)
            if (v[k] == comm) {
                v.erase(v.begin() + (long)k);
                break;
            }
    }
    (void)hipSetDevice(comm->device);
    // the last gather (and with it every earlier one on its stream) done before the staging is freed
    if (comm->done_recorded) (void)hipEventSynchronize(comm->done);
    const ncclResult_t r = comm->nccl ? ncclCommDestroy(comm->nccl) : ncclSuccess;
    comm->send.release();
    comm->recv.release();
    if (comm->done) (void)hipEventDestroy(comm->done);
    delete comm;
    if (r != ncclSuccess) return fail(ICP4R_E_RCCL, "ncclCommDestroy: %s", ncclGetErrorString(r));
    return ICP4R_OK;
}

int icp4r_comm_rank(const icp4r_comm* comm, int32_t* rank, int32_t* nranks) {
    if (!comm) return fail(ICP4R_E_INVALID, "comm is NULL");
    if (rank) *rank = comm->rank;
    if (nranks) *nranks = comm->nranks;
    return ICP4R_OK;
}

int icp4r_comm_check(icp4r_comm* comm) {
    if (!comm) return fail(ICP4R_E_INVALID, "comm is NULL");
    ncclResult_t async = ncclSuccess;
    RCCL_TRY(ncclCommGetAsyncError(comm->nccl, &async));
    if (async != ncclSuccess && async != ncclInProgress)
        return fail(ICP4R_E_RCCL, "RCCL asynchronous error on rank %d: %s", comm->rank, ncclGetErrorString(async));
    return ICP4R_OK;
}

int icp4r_gather_results(icp4r_comm* comm, const icp4r_result* shard_rows, int32_t npairs, icp4r_result* gathered,
                         void* hip_stream) {
    if (!comm || npairs < 0 || (npairs > 0 && !gathered)) return fail(ICP4R_E_INVALID, "icp4r_gather_results: bad arguments");
    int32_t first, count;
    shard_of(npairs, comm->nranks, comm->rank, &first, &count);
    if (count > 0 && !shard_rows) return fail(ICP4R_E_INVALID, "icp4r_gather_results: shard_rows is NULL");
    if (npairs == 0) return ICP4R_OK;
    icp4r_host::Range range("icp4r_gather_results");
    HIP_TRY(hipSetDevice(comm->device));
    if (!hip_stream && !comm->ctx)
        return fail(ICP4R_E_INVALID, "icp4r_gather_results: the communicator's context was destroyed; pass a stream");
    hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : comm->ctx->stream;
    constexpr size_t R = sizeof(icp4r_result);
    const int32_t maxc = (npairs + comm->nranks - 1) / comm->nranks;
    // a gather on another stream than the previous one must not overwrite staging that is still read
    if (comm->done_recorded && st != comm->last) HIP_TRY(hipStreamWaitEvent(st, comm->done, 0));
    if (npairs % comm->nranks == 0 && !comm->force_padded) {
        // equal shards: rank r's rows are exactly gathered[r * count, ...) — in place
        RCCL_TRY(ncclAllGather(shard_rows, gathered, (size_t)count * R, ncclUint8, comm->nccl, st));
    } else {
        HIP_TRY(comm->send.ensure((size_t)maxc * R));
        HIP_TRY(comm->recv.ensure((size_t)maxc * comm->nranks * R));
        if (count > 0) HIP_TRY(hipMemcpyAsync(comm->send.p, shard_rows, (size_t)count * R, hipMemcpyDeviceToDevice, st));
        RCCL_TRY(ncclAllGather(comm->send.p, comm->recv.p, (size_t)maxc * R, ncclUint8, comm->nccl, st));
        for (int32_t r = 0; r < comm->nranks; ++r) {
            int32_t f, c;
            shard_of(npairs, comm->nranks, r, &f, &c);
            if (c > 0)
                HIP_TRY(hipMemcpyAsync(gathered + f, static_cast<const char*>(comm->recv.p) + (size_t)r * maxc * R,
                                       (size_t)c * R, hipMemcpyDeviceToDevice, st));
        }
    }
    HIP_TRY(hipEventRecord(comm->done, st));
    comm->done_recorded = true;
    comm->last = st;
    return icp4r_comm_check(comm);
}

int icp4r_align_batch_sharded(icp4r_comm* comm, const icp4r_batch* shard, int32_t npairs_total,
                              const icp4r_params* params, icp4r_result* shard_results, icp4r_result* gathered,
                              void* hip_stream) {
    if (!comm || !shard) return fail(ICP4R_E_INVALID, "icp4r_align_batch_sharded: NULL argument");
    if (!comm->ctx) return fail(ICP4R_E_INVALID, "icp4r_align_batch_sharded: the communicator's context was destroyed");
    int32_t first, count;
    if (npairs_total < 0) return fail(ICP4R_E_INVALID, "npairs_total < 0");
    shard_of(npairs_total, comm->nranks, comm->rank, &first, &count);
    if (shard->npairs != count)
        return fail(ICP4R_E_INVALID, "rank %d of %d owns %d of %d pairs, the shard holds %d", comm->rank, comm->nranks,
                    count, npairs_total, shard->npairs);
    int rc;
    if (count > 0 && (rc = icp4r_align_batch_device(comm->ctx, shard, params, shard_results, hip_stream))) return rc;
    return icp4r_gather_results(comm, shard_results, npairs_total, gathered, hip_stream);
}

}  // extern "C"
