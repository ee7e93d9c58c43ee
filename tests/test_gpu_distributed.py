"""N>1 decode path on one GPU: two ranks (gloo, both on cuda:0) each decode their contiguous shard
of a 16-slot crowded batch, pack their decodes on the device (compact_records) and exchange them
with the data-sized gather_decodes; the gathered records must equal a single-process
SlotDecoder.records() of the whole batch byte for byte (slot ids are global after slot_offset).

RCCL cannot put two ranks on one device, so the exchange itself runs over gloo on host copies of
the device-packed buffers; the RCCL path is the same code with the nccl backend (bench.py)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_SLOTS, SIGNALS, SEED = 16, 50, 4100
KW = dict(max_candidates=300, min_score=2, max_iterations=20)


def _batch():
    from ft8_demodulator_amd import synth
    x, _ = synth.make_slots(N_SLOTS, SIGNALS, seed=SEED, device="cuda")
    return x


def _rank(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ft8_demodulator_amd import SlotDecoder
        from ft8_demodulator_amd.distributed import compact_records, gather_decodes, gathered_records, shard_range
        import numpy as np
        x = _batch()
        lo, hi = shard_range(N_SLOTS, rank, world)
        dec = SlotDecoder(12000, 2, 2, **KW)
        out, counts = dec.run(x[lo:hi])
        # device-side packing (what the RCCL path sends) == the host copy's packing
        total = int(counts.clamp(0, dec.cap).sum().item())
        dense, _ = compact_records(out, counts, dec.cap, max(total, 1))
        torch.cuda.synchronize()
        dense_bytes = dense[:total].cpu().numpy().tobytes()
        # the data-sized exchange of host copies over gloo, global slot ids
        recs2, cnts2, tots2 = gather_decodes(out.cpu(), counts.cpu(), dec.cap, slot_offset=lo)
        got = gathered_records(recs2, tots2)
        mine = recs2[rank, :total].numpy().copy()
        mine.view(np.int32)[:, 2] -= lo  # undo the offset: must equal the device packing
        q.put((rank, lo, hi, got.tobytes(), int(tots2.sum()), cnts2.numpy().tolist(),
               mine.tobytes() == dense_bytes))
    except Exception as e:  # noqa: BLE001
        q.put((rank, "error", repr(e), None, None, None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_two_rank_decode_gather_equals_single_process(gpu):
    import torch.multiprocessing as mp
    from ft8_demodulator_amd import SlotDecoder, _lib
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + (os.getpid() % 2000)
    ps = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=120)
    assert all(o[1] != "error" for o in out), out
    assert all(p.exitcode == 0 for p in ps)

    dec = SlotDecoder(12000, 2, 2, **KW)
    per_slot = dec.records(_batch())
    want = np.concatenate(per_slot)
    assert len(want) >= N_SLOTS // 2  # crowded slots decode about one message each
    for rank, lo, hi, got, n, cnts, dense_ok in out:
        assert n == len(want) and dense_ok
        assert got == want.tobytes(), rank       # byte for byte, global slot ids, slot order
        assert sum(cnts, []) == [len(r) for r in per_slot]
    assert {int(s) for s in want["slot"]} <= set(range(N_SLOTS))
    assert np.array_equal(want["slot"], np.sort(want["slot"], kind="stable"))
    _ = _lib
