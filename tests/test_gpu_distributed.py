"""N>1 decode path on one GPU.

* ft8_pack_decodes (the HIP kernel that packs a batch's decodes into the all-gather payload) equals
  the torch restatement of the layout, pack_decodes_reference, on synthetic records: empty slots,
  counts above cap, a capacity smaller than the total (overflow rows), > 1024 slots (several scan
  chunks), global slot offsets.
* RCCL: a world-size-1 "nccl" process group on cuda:0 runs the exchange the N > 1 bench runs --
  DecodeGatherer.start (device pack + all_gather_into_tensor, no host sync) then resolve -- on a
  real crowded 16-slot batch; the gathered records equal SlotDecoder.records() byte for byte, also
  when the capacity is forced below the total so the overflow rows take the second exchange.
* Two ranks (gloo, both on cuda:0) each decode their contiguous shard of the batch and exchange
  them; the gathered records equal a single-process decode of the whole batch.  RCCL cannot put
  two ranks on one device, so that exchange runs over gloo on host copies of the device-packed
  buffers."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_SLOTS, SIGNALS, SEED = 16, 50, 4100
KW = dict(max_candidates=300, min_score=2, max_iterations=20)


def _batch():
    from ft8_demodulator_amd import synth
    x, _ = synth.make_slots(N_SLOTS, SIGNALS, seed=SEED, device="cuda")
    return x


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _fake_records(S, cap, counts, torch):
    rec = torch.randint(0, 256, (S * cap * 40,), dtype=torch.uint8)
    v = rec.view(S, cap, 40)
    v.view(S, cap, 10, 4)[:, :, 2, :] = torch.arange(S, dtype=torch.int32)[:, None].view(torch.uint8)[:, None, :]
    return rec, torch.tensor(counts, dtype=torch.int32)


@pytest.mark.parametrize("S,cap,capacity,offset", [(5, 3, 16, 0), (5, 3, 4, 7), (3000, 4, 2000, 256),
                                                    (7, 2, 0, 0), (0, 3, 8, 0), (4, 300, 1200, 3)])
def test_pack_kernel_matches_reference(gpu, S, cap, capacity, offset):
    import torch
    from ft8_demodulator_amd.distributed import pack_decodes, pack_decodes_reference
    g = torch.Generator().manual_seed(S * 31 + cap)
    counts = torch.randint(-1, cap + 3, (S,), generator=g).tolist()  # negatives and counts > cap
    rec, cnt = _fake_records(S, cap, counts, torch)
    send_ref, over_ref = pack_decodes_reference(rec, cnt, cap, capacity, offset)
    send, over = pack_decodes(rec.cuda(), cnt.cuda(), cap, capacity, offset)
    torch.cuda.synchronize()
    assert send.cpu().numpy().tobytes() == send_ref.numpy().tobytes()
    total = int(send_ref[:8].view(torch.int64))
    if total > capacity:
        n = total - capacity
        assert over.cpu()[:n].numpy().tobytes() == over_ref[:n].numpy().tobytes()


def test_rccl_world1_gather_equals_records(gpu):
    """The nccl (RCCL) backend executes the decode exchange: device pack -> all_gather_into_tensor."""
    import torch
    import torch.distributed as dist
    from ft8_demodulator_amd import SlotDecoder
    from ft8_demodulator_amd.distributed import DecodeGatherer, gathered_records
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        x = _batch()
        dec = SlotDecoder(12000, 2, 2, **KW)
        want = np.concatenate(dec.records(x))
        assert len(want) >= N_SLOTS // 2
        for capacity in (None, 3):   # default capacity; 3 rows: the rest takes the overflow exchange
            g = DecodeGatherer(N_SLOTS, dec.cap, slot_offset=0, capacity=capacity)
            out, counts = dec.run(x)
            h = g.start(out, counts)                  # no host sync: pack + RCCL all-gather on the stream
            recs, cnts, tots = h.resolve()
            got = gathered_records(recs, tots)
            assert got.tobytes() == want.tobytes(), capacity
            assert int(tots[0]) == len(want) and recs.shape == (1, len(want), 40)
            assert cnts[0].cpu().tolist() == counts.cpu().tolist()
            if capacity == 3:
                assert g.capacity >= len(want) and g.grown == 1
    finally:
        dist.destroy_process_group()


def _rank(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ft8_demodulator_amd import SlotDecoder
        from ft8_demodulator_amd.distributed import (gather_decodes, gathered_records, pack_decodes,
                                                      pack_decodes_reference, shard_range)
        x = _batch()
        lo, hi = shard_range(N_SLOTS, rank, world)
        dec = SlotDecoder(12000, 2, 2, **KW)
        out, counts = dec.run(x[lo:hi])
        # device-side packing (the RCCL payload) == the packing of the host copies
        send, _ = pack_decodes(out, counts, dec.cap, 64, lo)
        ref, _ = pack_decodes_reference(out.cpu(), counts.cpu(), dec.cap, 64, lo)
        pack_ok = send.cpu().numpy().tobytes() == ref.numpy().tobytes()
        # the exchange of host copies over gloo, global slot ids
        recs2, cnts2, tots2 = gather_decodes(out.cpu(), counts.cpu(), dec.cap, slot_offset=lo)
        got = gathered_records(recs2, tots2)
        q.put((rank, lo, hi, got.tobytes(), int(tots2.sum()), cnts2.numpy().tolist(), pack_ok))
    except Exception as e:  # noqa: BLE001
        q.put((rank, "error", repr(e), None, None, None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_two_rank_decode_gather_equals_single_process(gpu):
    import torch.multiprocessing as mp
    from ft8_demodulator_amd import SlotDecoder
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
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
    for rank, lo, hi, got, n, cnts, pack_ok in out:
        assert n == len(want) and pack_ok
        assert got == want.tobytes(), rank       # byte for byte, global slot ids, slot order
        assert sum(cnts, []) == [len(r) for r in per_slot]
    assert {int(s) for s in want["slot"]} <= set(range(N_SLOTS))
    assert np.array_equal(want["slot"], np.sort(want["slot"], kind="stable"))
