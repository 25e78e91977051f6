"""The batched multi-GPU mode (include/icp4r/icp4r_multi.h; SURVEY.md §8e, BASELINE.json configs[3]).

On the one-GPU box: several contexts on device 0 stand in for several devices (separate streams,
workspaces and host threads — the same code path), an RCCL communicator of one rank exercises the
device-side gather entry points, and two processes on cuda:0 register their shards through the
library and gather the DEVICE-written result rows over gloo.  Every gathered batch must be
bit-identical to one single-process batch over all pairs.  RCCL refuses two ranks on one GPU, so the
multi-rank RCCL all-gather itself runs where bench.py --gpus N runs (the driver's 8-GPU node).
"""
import os
import socket
import sys

import numpy as np
import pytest

from test_gpu_parity import _batch, _pair

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _pairs(k0=2000, shapes=None):
    shapes = shapes or [(2048, 2048), (1500, 1800), (2048, 700), (900, 2048), (2048, 2048), (37, 500), (2000, 1990)]
    return [_pair(k0 + k, n, m) for k, (n, m) in enumerate(shapes)]


@pytest.mark.parametrize("nctx", [1, 2, 3, 9])
def test_align_batch_multi_equals_single_batch(gpu_ctx, nctx):
    """icp4r_align_batch_multi over nctx contexts (uneven contiguous shards; more contexts than pairs
    leaves some idle) returns the single batch's rows byte for byte, in global order."""
    import icp4r

    pairs = _pairs()
    args = _batch(pairs)
    p = icp4r.default_params(max_iterations=12)
    ref = gpu_ctx.align_batch_host(*args, params=p)
    ctxs = [icp4r.Context(0) for _ in range(nctx)]
    try:
        got = icp4r.align_batch_multi(ctxs, *args, params=p)
    finally:
        for c in ctxs:
            c.close()
    assert got.tobytes() == ref.tobytes()
    assert (got["status"] == 0).all()


def test_align_batch_multi_errors(gpu_ctx):
    import icp4r

    s, t = _pair(2100, 500)
    bad = s.copy()
    bad[7, 0] = np.nan
    args = _batch([(s, t), (bad, t)])
    ctxs = [icp4r.Context(0) for _ in range(2)]
    try:
        res = icp4r.align_batch_multi(ctxs, *args)  # per-pair statuses, as the single batch reports them
        assert res[0]["status"] == 0 and res[1]["status"] == icp4r.E_NONFINITE
        with pytest.raises(icp4r.ICP4RError):
            icp4r.align_batch_multi([], *args)
    finally:
        for c in ctxs:
            c.close()


def test_rccl_single_rank_sharded_batch(gpu_ctx):
    """A one-rank RCCL communicator: icp4r_align_batch_sharded (register + ncclAllGather) equals the
    plain device batch, and icp4r_gather_results moves the rows exactly."""
    import torch

    import icp4r

    pairs = _pairs(2200, [(2048, 2048)] * 5)
    src_h = np.concatenate([s for s, _ in pairs])
    tgt_h = np.concatenate([t for _, t in pairs])
    dev = torch.device("cuda", 0)
    n = 2048
    P = len(pairs)
    src = torch.from_numpy(src_h).to(dev)
    tgt = torch.from_numpy(tgt_h).to(dev)
    off = torch.arange(P, dtype=torch.int64, device=dev) * n
    cnt = torch.full((P,), n, dtype=torch.int32, device=dev)
    batch = icp4r.Batch(src=src.data_ptr(), tgt=tgt.data_ptr(), src_off=off.data_ptr(), src_n=cnt.data_ptr(),
                        tgt_off=off.data_ptr(), tgt_n=cnt.data_ptr(), guess=None, aligned=None, npairs=P,
                        max_src_n=n, max_tgt_n=n)
    params = icp4r.default_params(max_iterations=10)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ref = torch.zeros((P, 96), dtype=torch.uint8, device=dev)
    gpu_ctx.align_batch_device(batch, params, ref.data_ptr(), stream)
    comm = icp4r.Comm(gpu_ctx, 1, 0, icp4r.Comm.unique_id())
    try:
        rows = torch.zeros((P, 96), dtype=torch.uint8, device=dev)
        gathered = torch.full((P, 96), 255, dtype=torch.uint8, device=dev)
        comm.align_batch_sharded(batch, P, params, rows.data_ptr(), gathered.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        assert torch.equal(rows, ref) and torch.equal(gathered, ref)
        again = torch.zeros_like(gathered)
        comm.gather(rows.data_ptr(), P, again.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        assert torch.equal(again, ref)
        comm.check()
        with pytest.raises(icp4r.ICP4RError):  # the shard must be this rank's icp4r_shard of the total
            comm.align_batch_sharded(batch, P + 1, params, rows.data_ptr(), gathered.data_ptr(), stream)
    finally:
        comm.close()


def test_rccl_gather_padded_branch(gpu_ctx, plan):
    """icp4r_gather_results' unequal-shard branch (padded send / recv staging, one copy per rank),
    forced on a one-rank communicator by the gather_padded plan option (a test switch): the rows of a batch
    whose size no rank count divides evenly (7 pairs) land byte for byte in global order, also when
    consecutive gathers run on different streams (the staging is reused behind an event)."""
    import torch

    import icp4r

    pairs = _pairs(2300, [(2048, 2048), (1500, 1800), (2048, 700), (900, 2048), (37, 500), (2000, 1990),
                          (1024, 1024)])
    P = len(pairs)
    args = _batch(pairs)
    params = icp4r.default_params(max_iterations=8)
    ref_h = gpu_ctx.align_batch_host(*args, params=params)
    dev = torch.device("cuda", 0)
    rows = torch.from_numpy(np.frombuffer(ref_h.tobytes(), dtype=np.uint8).reshape(P, 96).copy()).to(dev)
    plan(gather_padded=1)
    comm = icp4r.Comm(gpu_ctx, 1, 0, icp4r.Comm.unique_id())
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    try:
        outs = []
        for k, s in enumerate([s1, s2, s1, None]):
            g = torch.full((P, 96), 255, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(dev)
            comm.gather(rows.data_ptr(), P, g.data_ptr(), s.cuda_stream if s is not None else None)
            outs.append(g)
        torch.cuda.synchronize(dev)
        comm.check()
        for g in outs:
            assert g.cpu().numpy().tobytes() == ref_h.tobytes()
    finally:
        comm.close()


def test_align_batch_multi_rejects_duplicate_context(gpu_ctx):
    import icp4r

    args = _batch(_pairs(2400, [(1024, 1024)] * 3))
    with pytest.raises(icp4r.ICP4RError):
        icp4r.align_batch_multi([gpu_ctx, gpu_ctx], *args)


def test_comm_destroy_after_context(gpu_ctx):
    """A communicator may outlive its context: icp4r_comm_destroy does not touch the context."""
    import icp4r

    ctx = icp4r.Context(0)
    comm = icp4r.Comm(ctx, 1, 0, icp4r.Comm.unique_id())
    ctx.close()
    comm.close()


def _rank_worker(rank, world, port, P, n, q):
    """One rank on cuda:0: its shard of the pairs through the library (device tensors), the device rows
    gathered over gloo."""
    try:
        sys.path[:0] = [os.path.join(ROOT, "icp-4dradar_amd"), os.path.join(ROOT, "tests")]
        import torch
        import torch.distributed as dist

        import icp4r
        from icp4r import dist as idist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.zeros(1, device=dev)
        mine = icp4r.shard(world * P, world, rank)
        from test_gpu_parity import _pair as pair

        sp = [pair(3000 + g, n) for g in mine]
        src = torch.from_numpy(np.concatenate([s for s, _ in sp])).to(dev)
        tgt = torch.from_numpy(np.concatenate([t for _, t in sp])).to(dev)
        off = torch.arange(P, dtype=torch.int64, device=dev) * n
        cnt = torch.full((P,), n, dtype=torch.int32, device=dev)
        batch = icp4r.Batch(src=src.data_ptr(), tgt=tgt.data_ptr(), src_off=off.data_ptr(), src_n=cnt.data_ptr(),
                            tgt_off=off.data_ptr(), tgt_n=cnt.data_ptr(), guess=None, aligned=None, npairs=P,
                            max_src_n=n, max_tgt_n=n)
        ctx = icp4r.Context(0)
        rows = torch.zeros((P, 96), dtype=torch.uint8, device=dev)
        ctx.align_batch_device(batch, icp4r.default_params(max_iterations=15), rows.data_ptr(),
                               torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        allr = idist.gather_results(rows.cpu(), world)  # the device-written rows, over gloo
        ctx.close()
        q.put((rank, allr.numpy().tobytes()))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        q.put((rank, repr(e)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_two_ranks_on_one_gpu_gather_device_rows(gpu_ctx):
    """Two processes on cuda:0, each registering its contiguous shard through the library; the rows the
    device wrote, gathered over gloo, are bit-identical to one single-process batch of all pairs."""
    import torch.multiprocessing as mp

    import icp4r

    world, P, n = 2, 6, 2048
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, P, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    ref = gpu_ctx.align_batch_host(*_batch([_pair(3000 + g, n) for g in range(world * P)]),
                                   params=icp4r.default_params(max_iterations=15))
    for r in range(world):
        assert isinstance(got[r], bytes), got[r]
        assert got[r] == ref.tobytes(), r
