"""Multi-GPU sharding of slot batches: one process per GPU, slots split by contiguous ranges, one
all-gather of the result records (ft8_result, 40 B) per batch -- either the fixed per-slot buffers
(gather_records) or, far smaller, the decodes compacted on the device (gather_decodes).

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


REC_BYTES = 40  # sizeof(ft8_result)


def compact_records(records, counts, cap, capacity):
    """Pack the per-slot record buffer (uint8 [S*cap*40], slot s's decodes in rows [s*cap, s*cap +
    counts[s])) into `capacity` dense rows in slot order, on the records' device and without a host
    sync.  Returns (dense uint8 [capacity, 40], total int64 0-d tensor = sum of min(counts, cap));
    total > capacity means rows beyond `capacity` were dropped (every record keeps its own `slot`)."""
    import torch
    dev = records.device
    S = counts.numel()
    c = counts.to(torch.int64).clamp(0, cap)
    off = torch.cumsum(c, 0) - c
    j = torch.arange(cap, device=dev, dtype=torch.int64)
    dest = off[:, None] + j[None, :]
    keep = (j[None, :] < c[:, None]) & (dest < capacity)
    dest = torch.where(keep, dest, torch.full_like(dest, capacity))  # row `capacity` is a dump row
    dense = torch.zeros((capacity + 1, REC_BYTES), dtype=torch.uint8, device=dev)
    dense.index_copy_(0, dest.view(-1), records[: S * cap * REC_BYTES].view(S * cap, REC_BYTES))
    return dense[:capacity], c.sum()


def gather_decodes(records, counts, cap, capacity=None, group=None, slot_offset=0):
    """One all-gather of every rank's decodes, compacted: each rank packs its records into dense
    rows (compact_records) plus its per-slot counts and total into one byte buffer, so the exchange
    moves rows*40 + 4*S + 8 bytes per rank instead of S*cap*40.

    capacity=None (default) sizes the exchange from the data in two phases: an all-gather of the
    per-rank totals (8 bytes each; one host sync), then exactly max(totals) rows per rank, so no
    rank is ever truncated whatever the decodes per slot (top-k / subtract-and-redecode batches
    decode ~28 per slot).  An int capacity keeps a fixed row count (no extra sync); a rank whose
    total exceeds it is flagged by totals[r] > capacity.

    Returns (records uint8 [world, rows, 40], counts int32 [world, S], totals int64 [world]) on
    every rank; rank r's first min(totals[r], rows) rows are its decodes in slot order.
    slot_offset (this rank's first global slot, e.g. shard_range's lo) is added to every record's
    `slot` field, so gathered records carry global slot indices."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    S = counts.numel()
    dev = records.device
    if capacity is None:
        mine = counts.to(torch.int64).clamp(0, cap).sum().reshape(1)
        tot_all = torch.empty(world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(tot_all, mine, group=group)
        capacity = int(tot_all.max().item())
    dense, total = compact_records(records, counts, cap, capacity)
    if slot_offset:
        ids = dense.view(torch.int32)[:, 2]  # ft8_result.slot (bytes 8..11), rows < total only
        ids.add_((torch.arange(capacity, device=dev) < total).to(torch.int32) * int(slot_offset))
    nrec = capacity * REC_BYTES
    buf = torch.empty(nrec + 4 * S + 8, dtype=torch.uint8, device=dev)
    buf[:nrec] = dense.reshape(-1)
    buf[nrec:nrec + 4 * S] = counts.to(torch.int32).contiguous().view(torch.uint8)
    buf[nrec + 4 * S:] = total.reshape(1).view(torch.uint8)
    out = torch.empty(world * buf.numel(), dtype=torch.uint8, device=dev).view(world, -1)
    dist.all_gather_into_tensor(out.view(-1), buf, group=group)
    recs = out[:, :nrec].reshape(world, capacity, REC_BYTES)
    cnts = out[:, nrec:nrec + 4 * S].contiguous().view(torch.int32)
    totals = out[:, nrec + 4 * S:].contiguous().view(torch.int64).reshape(world)
    return recs, cnts, totals


def gathered_records(recs, totals):
    """(records [world, rows, 40], totals [world]) of gather_decodes -> one structured ft8_result
    array (host) of every rank's decodes, rank-major (i.e. in global slot order when ranks hold
    contiguous shards); raises if a rank was truncated."""
    import numpy as np
    from ._lib import RESULT_DTYPE
    rows = recs.shape[1]
    tot = [int(t) for t in totals.cpu().tolist()]
    if any(t > rows for t in tot):
        raise RuntimeError(f"gather_decodes truncated: totals {tot} > {rows} rows per rank")
    r = recs.cpu().numpy()
    parts = [r[k, :tot[k]].reshape(-1).view(RESULT_DTYPE) for k in range(len(tot))]
    return np.concatenate(parts) if parts else np.zeros(0, RESULT_DTYPE)
