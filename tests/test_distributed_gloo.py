"""N>1 path on CPU: world_size 2 over gloo -- slot sharding and the record all-gathers (fixed
buffers; the packed exchange with a capacity below the total, whose overflow rows take the second
exchange; a larger batch that grows the capacity; a step with no decodes)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _records(lo, hi, cap, counts):
    """Fake ft8_result rows: byte 0 = global slot, bytes 8..11 (slot field) = local slot, byte 28
    (payload[0]) = row within the slot."""
    n = hi - lo
    rec = torch.zeros(n * cap * 40, dtype=torch.uint8)
    v = rec.view(n, cap, 40)
    v[:, :, 0] = torch.arange(lo, hi, dtype=torch.uint8)[:, None]
    v[:, :, 28] = torch.arange(cap, dtype=torch.uint8)[None, :]
    v.view(n, cap, 10, 4)[:, :, 2, :] = torch.arange(n, dtype=torch.int32)[:, None].view(torch.uint8)[:, None, :]
    return rec, counts


def _worker(rank, world, port, n_slots, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
      try:
        from ft8_demodulator_amd.distributed import (gather_decodes, gather_records, gathered_records,
                                                      shard_range)
        lo, hi = shard_range(n_slots, rank, world)
        cap = 3
        rec, cnt = _records(lo, hi, cap, torch.arange(lo, hi, dtype=torch.int32) % 4)
        r_all, c_all = gather_records(rec, cnt)
        d_all, dc_all, tot = gather_decodes(rec, cnt, cap, 4)
        compact = [d_all[r, :int(tot[r]), 0].tolist() for r in range(world)]
        # data-sized exchange with many decodes per slot (rank 1: 10 + 11 + 12 + 12 rows > 8 per slot)
        cap2 = 12
        rec2, cnt2 = _records(lo, hi, cap2, torch.arange(lo, hi, dtype=torch.int32) + 6)
        s_all, sc_all, stot = gather_decodes(rec2, cnt2, cap2, slot_offset=lo)
        flat = gathered_records(s_all, stot)
        sized = (list(s_all.shape), stot.tolist(), flat["slot"].tolist(), flat["payload"][:, 0].tolist(),
                 [int(b) for b in flat.view(np.uint8).reshape(-1, 40)[:, 0]])
        # a step that decodes nothing anywhere: a zero-row exchange, an empty gathered array
        z_all, zc_all, ztot = gather_decodes(rec, torch.zeros_like(cnt), cap)
        zero = (list(z_all.shape), zc_all.tolist(), ztot.tolist(), len(gathered_records(z_all, ztot)))
        q.put((rank, lo, hi, r_all.view(world, hi - lo, cap, 40)[:, :, 0, 0].tolist(), c_all.tolist(),
               compact, dc_all.tolist(), tot.tolist(), (sized, zero)))
      except Exception as e:  # noqa: BLE001
        q.put((rank, "error", repr(e), None, None, None, None, None, (None, None)))
        raise
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    from ft8_demodulator_amd.distributed import shard_range
    for n in (0, 1, 7, 256, 2048):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_gloo_world2_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 2000)
    ps = [ctx.Process(target=_worker, args=(r, 2, port, 8, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    assert all(o[1] != "error" for o in out), out
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, lo, hi, recs, cnts, compact, dcnts, tot, (sized, zero) in out:
        assert zero == ([2, 0, 40], [[0, 0, 0, 0], [0, 0, 0, 0]], [0, 0], 0)
        assert recs == [[0, 1, 2, 3], [4, 5, 6, 7]]
        assert cnts == [[0, 1, 2, 3], [0, 1, 2, 3]]
        # packed: slot s contributes min(count, cap) rows tagged s, in slot order; each rank holds
        # 0 + 1 + 2 + 3 = 6 decodes for a capacity of 4, so rows 4 and 5 come by the overflow exchange
        assert dcnts == cnts
        assert tot == [0 + 1 + 2 + 3, 0 + 1 + 2 + 3]
        assert compact == [[1, 2, 2, 3, 3, 3], [5, 6, 6, 7, 7, 7]]
        # sized: counts 6..13 clamped to cap 12 -> rank 0 holds 6+7+8+9 = 30 rows, rank 1 10+11+12+12 = 45;
        # the exchange carries exactly 45 rows per rank, nothing is truncated, slots are global
        shape, stot, slots, rows, tags = sized
        assert shape == [2, 45, 40] and stot == [30, 45]
        want = [(s, j) for s in range(8) for j in range(min(6 + s, 12))]
        assert list(zip(slots, rows)) == want
        assert tags == slots  # the global slot written into byte 0 agrees with the offset slot field


def _uneven_worker(rank, world, port, n_slots, q):
    """Shards of different sizes (shard_range of 7 slots over 2 ranks: 4 and 3): the packed buffers
    must have one size on every rank, whether the gatherer learns the largest shard by an all-reduce
    or is told it."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        try:
            from ft8_demodulator_amd.distributed import (DecodeGatherer, gather_decodes, gathered_records,
                                                          shard_range)
            lo, hi = shard_range(n_slots, rank, world)
            cap = 5
            rec, cnt = _records(lo, hi, cap, torch.arange(lo, hi, dtype=torch.int32) % 4 + 1)
            out = []
            for kw in ({}, {"max_slots": -(-n_slots // world)}):
                recs, cnts, tot = gather_decodes(rec, cnt, cap, capacity=3, slot_offset=lo, **kw)
                flat = gathered_records(recs, tot)
                out.append((cnts.tolist(), tot.tolist(), flat["slot"].tolist(), flat["payload"][:, 0].tolist()))
            # a gatherer reused over steps: the agreement happens once
            g = DecodeGatherer(hi - lo, cap, slot_offset=lo)
            for _ in range(2):
                r2, c2, t2 = g.start(rec, cnt).resolve()
            out.append((g.S_pad, g.capacity, t2.tolist()))
            q.put((rank, out))
        except Exception as e:  # noqa: BLE001
            q.put((rank, "error " + repr(e)))
            raise
    finally:
        dist.destroy_process_group()


def test_gloo_world2_uneven_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + (os.getpid() % 2000)
    ps = [ctx.Process(target=_uneven_worker, args=(r, 2, port, 7, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    assert all(not isinstance(o[1], str) for o in out), out
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    # rank 0: slots 0..3 with counts 1,2,3,4 (10 rows); rank 1: slots 4..6 with counts 1,2,3 (+ a
    # zero pad slot): 6 rows; capacity 3 -> both take the overflow exchange
    want_slots = [s for s in range(7) for _ in range(s % 4 + 1)]
    want_rows = [j for s in range(7) for j in range(s % 4 + 1)]
    for rank, res in out:
        for cnts, tot, slots, rows in res[:2]:
            assert cnts == [[1, 2, 3, 4], [1, 2, 3, 0]]
            assert tot == [10, 6]
            assert slots == want_slots and rows == want_rows
        assert res[2] == (4, 20, [10, 6])  # capacity min(S_pad * cap, max(64, 4 S_pad))


class _FakeDecoder:
    """Stands in for SlotDecoder in bench.StepLoop on the CPU: every run() returns a fresh record
    buffer whose rows carry (rank, call number) in payload[0..1], and counts that vary per call, so
    a gathered step shows which step of which rank it came from."""

    def __init__(self, rank, lo, hi, cap, tag, log):
        self.rank, self.lo, self.hi, self.cap, self.tag, self.log = rank, lo, hi, cap, tag, log

    def run(self, x):
        k = len(self.log)
        self.log.append(self.tag)
        n = self.hi - self.lo
        counts = (torch.arange(n, dtype=torch.int32) + k + self.rank) % 3
        rec = torch.zeros(n * self.cap * 40, dtype=torch.uint8)
        v = rec.view(n, self.cap, 40)
        v[:, :, 28] = self.rank
        v[:, :, 29] = k
        v.view(n, self.cap, 10, 4)[:, :, 2, :] = torch.arange(n, dtype=torch.int32)[:, None].view(torch.uint8)[:, None, :]
        return rec, counts


def _steploop_worker(rank, world, port, S, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        try:
            import contextlib
            import importlib.util
            root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
            bench = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(bench)
            from ft8_demodulator_amd.distributed import DecodeGatherer, gathered_records
            cap, D, K = 4, 2, 6
            log = []
            decs = [_FakeDecoder(rank, rank * S, (rank + 1) * S, cap, d, log) for d in range(D)]
            # a small capacity so some steps overflow it and resolve() runs the second exchange
            g = DecodeGatherer(S, cap, slot_offset=rank * S, capacity=4)
            loop = bench.StepLoop(decs, [contextlib.nullcontext] * D, None, g)
            for k in range(3):              # warm-up steps: their exchanges are issued, not kept
                loop.step(k)
            for k in range(3, 3 + K):       # the timed steps, kept; the alternation continues
                loop.step(k, keep=True)
            res = loop.resolve()
            out = []
            for i, (recs, cnts, tot, capacity) in enumerate(res):
                flat = gathered_records(recs, tot)
                call = 3 + i                # every rank's call number of this timed step
                ok = bench.gather_check(flat, cnts.numpy(), tot.tolist(), S, world, int(tot.sum()), cap)
                tags = sorted(set(zip(flat["payload"][:, 0].tolist(), flat["payload"][:, 1].tolist())))
                out.append((ok["gather_ok"], tags, call, int(tot.max()) > capacity))
            q.put((rank, log, out, g.grown))
        except Exception as e:  # noqa: BLE001
            q.put((rank, "error " + repr(e), None, None))
            raise
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bench_step_loop_depth2():
    """bench.StepLoop at world size 2 over gloo, depth 2: the steps alternate over the two decoders,
    every warm-up and timed step issues its exchange without resolving it, the kept exchanges are
    resolved after the loop in issue order -- each gathered step holds exactly that step's records
    from both ranks (a rank resolving out of order would pair step k of one rank with another step
    of the other), gather_ok holds for every step, and overflowing steps take the second exchange."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33500 + (os.getpid() % 2000)
    ps = [ctx.Process(target=_steploop_worker, args=(r, 2, port, 5, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=180) for _ in ps], key=lambda o: o[0])
    for p in ps:
        p.join(timeout=60)
    assert all(not isinstance(o[1], str) for o in out), out
    for rank, log, steps, grown in out:
        assert log == [k % 2 for k in range(9)]                   # decoder k % D ran step k
        assert len(steps) == 6
        for ok, tags, call, over in steps:
            assert ok
            assert tags == [(r, call) for r in range(2)]            # both ranks' records of this very step
        assert any(over for *_, over in steps) and grown >= 1      # the overflow exchange ran
    assert out[0][2] == out[1][2]
