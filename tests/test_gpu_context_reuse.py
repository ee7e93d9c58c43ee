"""One libft8hip context across entry points whose scratch needs differ.

The k_bp claim counters live in one context buffer: [0] for ft8_bp, [1 + k] for decode chunk k,
each with a host-side ticket base.  When a later call needs more counters the buffer is
reallocated and zeroed (possibly at the same address), so every base must restart at 0 and the
base vector must grow with it; otherwise k_bp retires every wave at once (no decodes, no error) or
writes past the base vector.  Sequence on a fresh context: ft8_bp -> a decode cut into one-slot
chunks (n_slots + 1 counters) -> ft8_bp -> a one-chain decode, each checked against the oracle or
the one-chain decode of a separate context."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KW = dict(max_candidates=300, min_score=2, max_iterations=20)


def _bp(ctx, llr, iters):
    import torch
    from ft8_demodulator_amd import _lib
    a = torch.from_numpy(np.ascontiguousarray(llr, dtype=np.float64)).cuda()
    n = a.shape[0]
    plain = torch.zeros(n, 174, dtype=torch.uint8, device="cuda")
    res = torch.zeros(n * _lib.RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    ctx.check(_lib.lib().ft8_bp(ctx.handle, _lib.ptr(a), n, int(iters), _lib.ptr(plain), _lib.ptr(res),
                                _lib.stream_handle()), "ft8_bp")
    return plain.cpu().numpy(), res.cpu().numpy().view(_lib.RESULT_DTYPE)


def test_counters_survive_reallocation(gpu, oracle):
    from ft8_demodulator_amd import _lib, synth
    from ft8_demodulator_amd._pipeline import SlotDecoder
    rng = np.random.default_rng(11)
    llr = rng.standard_normal((96, 174)) * 2.5
    want = [oracle.bp_decode(v, 20) for v in llr]

    def check_bp(ctx):
        plain, rec = _bp(ctx, llr, 20)
        for i, (p_ref, e_ref) in enumerate(want):
            assert int(rec[i]["ldpc_errors"]) == e_ref and np.array_equal(plain[i], p_ref), i

    x, _ = synth.make_slots(12, 50, seed=5150, device="cuda")
    ref = SlotDecoder(12000, 2, 2, **KW)
    ref.ctx = _lib.Context(0)
    want_recs = [r.tobytes() for r in ref.records(x)]
    assert sum(len(r) for r in want_recs) > 0

    ctx = _lib.Context(0)                       # fresh: one counter after the first ft8_bp
    check_bp(ctx)
    check_bp(ctx)                               # the base advanced: the second launch decodes too
    dec = SlotDecoder(12000, 2, 2, **KW)
    dec.ctx = ctx
    ctx.set_pipeline(chunk_slots=1, n_streams=2)  # 12 chunks: 13 counters, the buffer is reallocated
    try:
        got = [r.tobytes() for r in dec.records(x)]
        assert got == want_recs
        check_bp(ctx)
        got = [r.tobytes() for r in dec.records(x)]
        assert got == want_recs
    finally:
        ctx.set_pipeline()
    got = [r.tobytes() for r in dec.records(x)]   # one chain again, on the grown buffer
    assert got == want_recs
    check_bp(ctx)


def test_one_context_on_alternating_streams(gpu):
    """One context driven from two torch streams in turn with no host synchronisation: every call
    waits (device side) for the previous call's work when the stream changes (capi.hip
    StreamOrder), so each step's records equal a synchronous decode's.  Without that order two
    steps' kernels would share the scratch and the k_bp claim counter concurrently."""
    import torch
    from ft8_demodulator_amd import _lib, synth
    from ft8_demodulator_amd._pipeline import SlotDecoder
    x, _ = synth.make_slots(16, 50, seed=6262, device="cuda")
    ref = SlotDecoder(12000, 2, 2, **KW)
    ref.ctx = _lib.Context(0)
    out, counts = ref.run(x)
    want, want_counts = out.clone(), counts.clone()
    torch.cuda.synchronize()
    assert int(want_counts.sum()) > 0
    # two decoders (own output buffers, one per stream) on ONE context
    ctx = _lib.Context(0)
    decs = [SlotDecoder(12000, 2, 2, **KW), SlotDecoder(12000, 2, 2, **KW)]
    for d in decs:
        d.ctx = ctx
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for k in range(12):
        with torch.cuda.stream(streams[k % 2]):
            out, counts = decs[k % 2].run(x)
            outs.append((out.clone(), counts.clone()))  # before this stream's next step reuses them
    torch.cuda.synchronize()

    def valid(out, counts):  # each slot's written records (the rest of the buffer is never written)
        rec = out.cpu().numpy().view(_lib.RESULT_DTYPE).reshape(16, -1)
        return [rec[i, : int(c)].tobytes() for i, c in enumerate(counts.cpu().numpy())]
    want_recs = valid(want, want_counts)
    for k, (out, counts) in enumerate(outs):
        assert torch.equal(counts, want_counts), k
        assert valid(out, counts) == want_recs, k


def test_two_contexts_on_two_streams(gpu):
    """The bench's --depth 2 configuration: consecutive steps alternate over two decoders with their
    own contexts and streams, so steps overlap on the device; every step's records equal a
    synchronous decode's."""
    import torch
    from ft8_demodulator_amd import _lib, synth
    from ft8_demodulator_amd._pipeline import SlotDecoder
    x, _ = synth.make_slots(16, 50, seed=7373, device="cuda")
    ref = SlotDecoder(12000, 2, 2, **KW)
    want = ref.records(x)
    assert sum(len(r) for r in want) > 0
    want = [r.tobytes() for r in want]
    decs = [SlotDecoder(12000, 2, 2, context=_lib.Context(0), **KW) for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for k in range(10):
        with torch.cuda.stream(streams[k % 2]):
            out, counts = decs[k % 2].run(x)
            outs.append((out.clone(), counts.clone()))
    torch.cuda.synchronize()
    for k, (out, counts) in enumerate(outs):
        rec = out.cpu().numpy().view(_lib.RESULT_DTYPE).reshape(16, -1)
        got = [rec[i, : int(c)].tobytes() for i, c in enumerate(counts.cpu().numpy())]
        assert got == want, k
