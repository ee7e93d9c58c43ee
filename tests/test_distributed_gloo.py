"""N>1 path on CPU: world_size 2 over gloo -- slot sharding and the record all-gather."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, n_slots, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
      try:
        from ft8_demodulator_amd.distributed import gather_records, shard_range
        lo, hi = shard_range(n_slots, rank, world)
        cap = 3
        rec = torch.zeros((hi - lo) * cap * 40, dtype=torch.uint8)
        rec.view(hi - lo, cap, 40)[:, :, 0] = torch.arange(lo, hi, dtype=torch.uint8)[:, None]
        cnt = torch.arange(lo, hi, dtype=torch.int32) % 4
        r_all, c_all = gather_records(rec, cnt)
        from ft8_demodulator_amd.distributed import gather_decodes
        d_all, dc_all, tot = gather_decodes(rec, cnt, cap, 4)
        compact = [d_all[r, :min(int(tot[r]), 4), 0].tolist() for r in range(world)]
        q.put((rank, lo, hi, r_all.view(world, hi - lo, cap, 40)[:, :, 0, 0].tolist(), c_all.tolist(),
               compact, dc_all.tolist(), tot.tolist()))
      except Exception as e:  # noqa: BLE001
        q.put((rank, "error", repr(e), None, None, None, None, None))
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
    for rank, lo, hi, recs, cnts, compact, dcnts, tot in out:
        assert recs == [[0, 1, 2, 3], [4, 5, 6, 7]]
        assert cnts == [[0, 1, 2, 3], [0, 1, 2, 3]]
        # compacted: slot s contributes min(count, cap) rows tagged s, in slot order; rank 1 holds
        # 0 + 1 + 2 + 3 = 6 decodes for a capacity of 4, so its total flags the truncation
        assert dcnts == cnts
        assert tot == [0 + 1 + 2 + 3, 0 + 1 + 2 + 3]
        assert compact == [[1, 2, 2, 3], [5, 6, 6, 7]]
