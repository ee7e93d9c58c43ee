"""Multi-GPU sharding of slot batches: one process per GPU, slots split by contiguous ranges, one
all-gather of the fixed-size result records (ft8_result, 40 B) per batch.

Slots are independent: no data-path collective is needed to decode.  The only
exchange is gathering every rank's decodes, e.g. to rank 0 for reporting; over RCCL ("nccl" backend)
the records stay on the GPU and travel over xGMI.
"""
from __future__ import annotations


def shard_range(n_slots: int, rank: int, world: int):
    """Contiguous slot range [lo, hi) of `rank` (sizes differ by at most one)."""
    base, rem = divmod(n_slots, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def gather_records(records, counts, group=None):
    """All-gather equal-shape record buffers (uint8 [S*cap*40]) and counts (int32 [S]) from every rank.

    Returns (records [world, ...], counts [world, S]) on every rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rec_all = torch.empty(world * records.numel(), dtype=records.dtype, device=records.device)
    cnt_all = torch.empty(world * counts.numel(), dtype=counts.dtype, device=counts.device)
    dist.all_gather_into_tensor(rec_all, records.contiguous().view(-1), group=group)
    dist.all_gather_into_tensor(cnt_all, counts.contiguous().view(-1), group=group)
    return rec_all.view((world,) + tuple(records.shape)), cnt_all.view((world,) + tuple(counts.shape))
