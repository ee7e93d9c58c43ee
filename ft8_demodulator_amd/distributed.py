"""Multi-GPU sharding of slot batches: one process per GPU, slots split by contiguous ranges, one
all-gather of the decodes per batch.

Slots are independent: no data-path collective is needed to decode.  The only exchange is gathering
every rank's decodes (ft8_result records, 40 B).  A batch decodes ~1 message per slot, while its
record buffer holds max_candidates per slot, so the decodes are first packed on the device --
ft8_pack_decodes, one HIP kernel: [int64 total][int32 counts[S]][capacity x ft8_result] in one byte
buffer, records carrying global slot ids -- and that buffer is the all-gather's payload.  Over RCCL
("nccl" backend) it stays on the GPU and travels over xGMI; nothing waits on the host.

The capacity (rows per rank) is fixed when the exchange is issued, so the host never has to learn
the totals first: rows past it go to a per-call overflow buffer on the device, every rank sees the
true totals in the gathered headers, and resolving the exchange (GatherHandle.resolve, collective)
moves the overflow rows in a second all-gather only when some rank exceeded the capacity.
DecodeGatherer keeps a capacity per stream of batches and grows it after such a step.

gather_records (the fixed per-slot buffers, unpacked) remains for callers that want them.
"""
from __future__ import annotations

REC_BYTES = 40  # sizeof(ft8_result)


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


def header_bytes(n_slots: int) -> int:
    """Bytes before the records in a packed buffer: int64 total + int32 counts padded to 8 B."""
    return 8 + ((4 * n_slots + 7) & ~7)


def pack_bytes(n_slots: int, capacity: int) -> int:
    return header_bytes(n_slots) + capacity * REC_BYTES


def pack_decodes_reference(records, counts, cap, capacity, slot_offset=0):
    """The packed layout of ft8_pack_decodes computed with torch ops, for records that live in host
    memory (gloo runs on the CPU) and as the checker of the HIP kernel in tests.
    -> (send uint8 [pack_bytes], overflow uint8 [S*cap - capacity, 40] or None)."""
    import torch
    dev = records.device
    S = counts.numel()
    c = counts.to(torch.int64).clamp(0, cap)
    total = int(c.sum())
    # a gatherer's padded slots (zero counts past this rank's records) hold no rows
    S_rec = min(S, records.numel() // (cap * REC_BYTES)) if cap else 0
    if int(c[S_rec:].sum()):
        raise ValueError("counts name slots past the record buffer")
    rows = records[: S_rec * cap * REC_BYTES].view(S_rec, cap, REC_BYTES)
    keep = torch.arange(cap, device=dev)[None, :] < c[:S_rec, None]
    dense = rows[keep].clone()                                   # slot order, then candidate order
    if slot_offset and total:
        dense.view(torch.int32)[:, 2] += int(slot_offset)       # ft8_result.slot (bytes 8..11)
    send = torch.zeros(pack_bytes(S, capacity), dtype=torch.uint8, device=dev)
    send[:8] = torch.tensor([total], dtype=torch.int64).view(torch.uint8).to(dev)
    send[8:8 + 4 * S] = counts.to(torch.int32).contiguous().view(torch.uint8)
    h = header_bytes(S)
    k = min(total, capacity)
    send[h:h + k * REC_BYTES] = dense[:k].reshape(-1)
    over = None
    if S * cap > capacity:
        over = torch.zeros((S * cap - capacity, REC_BYTES), dtype=torch.uint8, device=dev)
        if total > capacity:
            over[: total - capacity] = dense[capacity:]
    return send, over


def pack_decodes(records, counts, cap, capacity, slot_offset=0):
    """Pack one batch's decodes (SlotDecoder.run's outputs) for the all-gather -> (send, overflow).
    GPU tensors: the HIP kernel ft8_pack_decodes on the current stream (no host sync); host tensors:
    pack_decodes_reference."""
    import torch
    if records.device.type != "cuda":
        return pack_decodes_reference(records, counts, cap, capacity, slot_offset)
    from . import _lib
    S = counts.numel()
    dev = records.device
    send = torch.empty(pack_bytes(S, capacity), dtype=torch.uint8, device=dev)
    n_over = S * cap - capacity
    over = torch.empty((n_over, REC_BYTES), dtype=torch.uint8, device=dev) if n_over > 0 else None
    cnt = counts if counts.dtype == torch.int32 and counts.is_contiguous() else counts.to(torch.int32).contiguous()
    ctx = _lib.context(dev)
    ctx.check(_lib.lib().ft8_pack_decodes(ctx.handle, _lib.ptr(records), _lib.ptr(cnt), S, int(cap), int(capacity),
                                          int(slot_offset), _lib.ptr(send), _lib.ptr(over) if over is not None else None,
                                          _lib.stream_handle(dev)),
              "ft8_pack_decodes")
    return send, over


class GatherHandle:
    """An issued exchange: the gathered packed buffers of every rank, not yet looked at."""

    def __init__(self, out, over, n_slots, capacity, group, on_resolve=None):
        self.out, self.over, self.S, self.capacity, self.group = out, over, n_slots, capacity, group
        self._on_resolve = on_resolve

    def resolve(self):
        """-> (records uint8 [world, rows, 40], counts int32 [world, S], totals int64 [world]) with
        rows = max(totals): rank r's decodes are rows [0, totals[r]) in slot order.  Reads the
        totals on the host (a sync); when a rank's total exceeded the capacity, moves the overflow
        rows with a second all-gather -- a collective, so every rank resolves its exchanges in the
        same order."""
        import torch
        import torch.distributed as dist
        S, cap_rows = self.S, self.capacity
        h = header_bytes(S)
        world = self.out.shape[0]
        totals = self.out[:, :8].contiguous().view(torch.int64).reshape(world)
        counts = self.out[:, 8:8 + 4 * S].contiguous().view(torch.int32).reshape(world, S)
        rows = int(totals.max().item()) if world else 0
        recs = self.out[:, h:].reshape(world, cap_rows, REC_BYTES)
        if rows > cap_rows:
            extra = rows - cap_rows
            if self.over is None or self.over.shape[0] < extra:
                raise RuntimeError(f"decode exchange: {rows} rows exceed this rank's record buffer")
            mine = self.over[:extra].contiguous().view(-1)
            got = torch.empty(world * mine.numel(), dtype=torch.uint8, device=mine.device)
            dist.all_gather_into_tensor(got, mine, group=self.group)
            recs = torch.cat([recs, got.view(world, extra, REC_BYTES)], dim=1)
        else:
            recs = recs[:, :rows]
        if self._on_resolve is not None:
            self._on_resolve(rows)
        return recs, counts, totals


class DecodeGatherer:
    """All-gathers of a stream of batches (S slots per rank, `cap` records per slot): start() packs
    and issues the exchange without a host sync and returns a GatherHandle.  The capacity (rows per
    rank) starts at `capacity` (default: 4 per slot, at least 64, at most S_pad * cap) and grows to
    1.25 x the largest total a resolved exchange reported beyond it.

    all_gather_into_tensor needs the same buffer size on every rank, so the packed header is sized
    for S_pad = the largest slot count of any rank (shard_range's shards differ by one): `max_slots`
    when the caller knows it (ceil(n / world) for shard_range), else one all-reduce(MAX) of S at the
    first start() (a host sync, once per gatherer).  A rank with fewer slots sends zero counts for
    the missing ones; resolve() returns counts [world, S_pad], rank r's real slots first."""

    def __init__(self, n_slots, cap, slot_offset=0, group=None, capacity=None, max_slots=None):
        self.S, self.cap, self.slot_offset, self.group = int(n_slots), int(cap), int(slot_offset), group
        if max_slots is not None and int(max_slots) < self.S:
            raise ValueError(f"max_slots {max_slots} < this rank's {self.S} slots")
        self.S_pad = None if max_slots is None else int(max_slots)
        self._capacity_arg = capacity
        self.capacity = None
        if self.S_pad is not None:
            self._set_capacity()
        self.grown = 0

    def _set_capacity(self):
        full = self.S_pad * self.cap
        c = self._capacity_arg
        self.capacity = min(full, int(c) if c is not None else max(64, 4 * self.S_pad))

    def _agree_slots(self, device):
        """S_pad = max over ranks of S (one all-reduce; gloo on the host, RCCL on the device)."""
        import torch
        import torch.distributed as dist
        dev = device if dist.get_backend(self.group) != "gloo" else torch.device("cpu")
        t = torch.tensor([self.S], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        self.S_pad = int(t.item())
        self._set_capacity()

    def _grow(self, rows):
        if rows > self.capacity:
            self.capacity = min(self.S_pad * self.cap, (rows * 5 // 4 + 63) // 64 * 64)
            self.grown += 1

    def start(self, records, counts) -> GatherHandle:
        import torch
        import torch.distributed as dist
        if counts.numel() != self.S:
            raise ValueError(f"batch has {counts.numel()} slots, the gatherer {self.S}")
        if self.S_pad is None:
            self._agree_slots(records.device)
        if self.S_pad > self.S:
            pad = torch.zeros(self.S_pad, dtype=torch.int32, device=counts.device)
            pad[: self.S] = counts.view(-1)
            counts = pad
        send, over = pack_decodes(records, counts, self.cap, self.capacity, self.slot_offset)
        world = dist.get_world_size(self.group)
        out = torch.empty(world * send.numel(), dtype=torch.uint8, device=send.device)
        dist.all_gather_into_tensor(out, send, group=self.group)
        return GatherHandle(out.view(world, -1), over, self.S_pad, self.capacity, self.group, self._grow)


def gather_decodes(records, counts, cap, capacity=None, group=None, slot_offset=0, max_slots=None):
    """One exchange of every rank's decodes, resolved at once (a host sync): packs this rank's
    records (capacity rows: the given number, or DecodeGatherer's default), all-gathers, and moves
    overflow rows in a second exchange if any rank exceeded the capacity -- so nothing is ever
    truncated.  slot_offset (this rank's first global slot, e.g. shard_range's lo) is added to every
    record's slot.  Ranks may hold different slot counts (max_slots: the largest, or None to agree
    on it by an all-reduce).  -> (records uint8 [world, max(totals), 40], counts int32 [world,
    S_pad], totals int64 [world]); rank r's decodes are rows [0, totals[r])."""
    g = DecodeGatherer(counts.numel(), cap, slot_offset, group, capacity, max_slots)
    return g.start(records, counts).resolve()


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
