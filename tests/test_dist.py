"""Multi-rank batched mode on CPU (gloo, world_size 2): sharding + result all-gather.

Each rank registers its own shard of pairs (here with the CPU oracle standing in for the device call,
since this runs without a GPU) and the gathered results must equal a single-process run over all
pairs, in global pair order — the same sharding/gather code path bench.py uses with RCCL.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _register(indices, n=300):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    from icp4r import RESULT_DTYPE, synth

    out = np.zeros(len(indices), RESULT_DTYPE)
    for k, i in enumerate(indices):
        p = synth.make_pair(i, n)
        r = oracle.align(p.src_xyzi(), p.tgt_xyzi(), max_iterations=5)
        out[k]["T"] = r["T"].T.reshape(16)
        out[k]["fitness"] = r["fitness"]
        out[k]["iterations"] = r["iterations"]
        out[k]["converged"] = r["converged"]
    return out


def _worker(rank, world, port, P, q):
    try:
        import torch
        import torch.distributed as dist

        sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))
        from icp4r import dist as idist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        mine = idist.shard(rank, world, P)
        local = torch.from_numpy(_register(list(mine)).view(np.uint8).reshape(P, 96).copy())
        allr = idist.gather_results(local, world)
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


def test_shard_ranges():
    from icp4r import dist as idist

    assert list(idist.shard(1, 4, 3)) == [3, 4, 5]
    blocks = [idist.split_even(10, r, 3) for r in range(3)]
    assert [len(b) for b in blocks] == [4, 3, 3]
    assert sorted(i for b in blocks for i in b) == list(range(10))
    with pytest.raises(ValueError):
        idist.shard(4, 4, 1)


def test_gloo_world2_gather_equals_single_process():
    import torch.multiprocessing as mp

    from icp4r import RESULT_DTYPE

    world, P = 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert isinstance(got[r], bytes), got[r]
    ref = _register(list(range(world * P)))
    for r in range(world):
        res = np.frombuffer(got[r], dtype=RESULT_DTYPE)
        assert len(res) == world * P
        assert (res["T"] == ref["T"]).all()
        assert (res["fitness"] == ref["fitness"]).all()
