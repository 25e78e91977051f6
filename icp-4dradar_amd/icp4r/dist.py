"""Multi-GPU batched mode: shard independent scan pairs over ranks, gather the result structs.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm; "gloo" for CPU tests).  The
pairs are independent, so the data path has no collective: rank r owns the contiguous block of
global pair indices [r * P, (r + 1) * P) and generates/loads its own inputs.  The
only exchange is the final all-gather of the 96-byte result structs (C4: 8192 x 96 B = 768 KiB over
xGMI), which leaves every rank holding all results in global pair order.
"""
from __future__ import annotations

import numpy as np

RESULT_BYTES = 96


def shard(rank: int, world: int, pairs_per_rank: int) -> range:
    """Global pair indices owned by `rank` (weak scaling: fixed pairs per rank)."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    return range(rank * pairs_per_rank, (rank + 1) * pairs_per_rank)


def split_even(total: int, rank: int, world: int) -> range:
    """Strong-scaling split of `total` pairs into contiguous, balanced blocks."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def gather_results(local, world: int, out=None):
    """All-gather equal-sized per-rank result blocks ((P, 96) uint8 tensors) in rank order.

    Works on any backend: NCCL/RCCL device tensors use all_gather_into_tensor (into `out` when
    given, so a timed loop allocates nothing), others all_gather.
    """
    import torch
    import torch.distributed as dist

    if world == 1:
        return local
    if local.is_cuda:
        if out is None:
            out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                              device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous())
        return out
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local.contiguous())
    return torch.cat(parts)


def results_to_numpy(t) -> np.ndarray:
    from . import RESULT_DTYPE

    return np.frombuffer(t.detach().cpu().numpy().tobytes(), dtype=RESULT_DTYPE)
