"""End-to-end parity: WAV / synthetic slots through the whole GPU receive path vs the reference's
golden decodes (tests/golden, captured from the reference itself) and the oracle."""
import os

import numpy as np
import pytest

from conftest import DATA

pytestmark = pytest.mark.gpu


SCORE_ATOL = 1e-4  # end-to-end score tolerance of a decode on float32 input


def _same(got, gold, tag, atol=SCORE_ATOL):
    """Payload, CRC, status, time and frequency exact; score within `atol` (a scalar, or one value
    per decode).  The GPU FFT is a float32 FFT like scipy's but not pocketfft, so a score differs by
    its rounding; atol defaults to 1e-4 (float32 scores of strong candidates move by ~1e-6)."""
    assert [g[:7] + (g[8],) for g in got] == [r[:7] + (r[8],) for r in gold], tag
    d = np.abs(np.array([g[7] for g in got]) - np.array([r[7] for r in gold]))
    assert np.all(d <= np.broadcast_to(atol, d.shape)), (tag, d.tolist())


def _rows(results):
    return [(m.payload.hex(), m.hash, s.ldpc_errors, s.crc_extracted, s.crc_calculated, t, f, float(sc),
             type(sc).__name__) for (m, s, t, f, sc) in results]


def _gold_rows(case):
    return [(r["payload"], r["hash"], r["ldpc_errors"], r["crc_extracted"], r["crc_calculated"], r["time_sec"],
             r["freq_hz"], r["score"], r["score_dtype"]) for r in case["results"]]


def test_wav_cases_match_reference(golden, gpu):
    from ft8_demodulator_amd import decode_ft8_from_wave, decode_ft8_message, read_wave_file
    meta, _ = golden
    seen = 0
    for case in meta["e2e"]:
        if "wav" not in case or case.get("as_float64") or case.get("as_analytic") or case["error"]:
            continue
        path = os.path.join(DATA, case["wav"])
        got = decode_ft8_from_wave(path, **case["kwargs"])         # int16 path, on-device scaling
        x, fs = read_wave_file(path)
        gold = _gold_rows(case)
        print(case["name"], "score |diff|", [abs(g[7] - r[7]) for g, r in zip(_rows(got), gold)])
        _same(_rows(got), gold, case["name"])
        got2 = decode_ft8_message(x, fs, **case["kwargs"])         # float32 path
        assert _rows(got2) == _rows(got), case["name"]
        seen += 1
    assert seen >= 7


def test_float64_and_analytic_inputs(golden, gpu):
    import scipy.signal
    from ft8_demodulator_amd import decode_ft8_message, read_wave_file
    meta, _ = golden
    x, fs = read_wave_file(os.path.join(DATA, "synth_cfg1.wav"))
    cases = {c["name"]: c for c in meta["e2e"]}
    got = decode_ft8_message(x.astype(np.float64), fs)
    _same(_rows(got), _gold_rows(cases["cfg1_f64"]), "f64", atol=1e-9)
    z = scipy.signal.hilbert(x.astype(np.float64))
    got = decode_ft8_message(z, fs)
    _same(_rows(got), _gold_rows(cases["cfg1_c128"]), "c128", atol=1e-9)


def test_edge_cases_return_empty(gpu):
    from ft8_demodulator_amd import decode_ft8_message
    assert decode_ft8_message(np.zeros(1000), 12000) == []
    assert decode_ft8_message(np.zeros(10), 12000) == []
    assert decode_ft8_message(np.zeros(180000, dtype=np.float32), 12000) == []
    assert decode_ft8_message(np.random.default_rng(0).standard_normal(180000).astype(np.float32), 12000,
                              freq_min=5000.0, freq_max=4000.0) == []
    assert decode_ft8_message(np.zeros(180000, dtype=np.float32), 12000, max_candidates=0) == []


def test_batch_equals_single_and_oracle(gpu, oracle):
    """A batch of crowded synthetic slots: batched decode == per-slot decode == oracle (same input)."""
    import torch
    from ft8_demodulator_amd import SlotDecoder, decode_ft8_message, synth
    x, truth = synth.make_slots(6, 50, seed=900, device="cuda")
    kw = dict(max_candidates=300, min_score=2, max_iterations=20)
    dec = SlotDecoder(12000, **kw)
    batched = dec.decode(x)
    for s in range(x.shape[0]):
        single = decode_ft8_message(x[s].cpu().numpy(), 12000, **kw)
        assert _rows(batched[s]) == _rows(single)
        ref = oracle.decode_ft8_message(x[s].cpu().numpy(), 12000, **kw)
        got = sorted((m.payload.hex(), m.hash) for m, *_ in batched[s])
        exp = sorted((p.hex(), h) for (p, h, *_r) in ref)
        assert got == exp, s
        assert set(p for p, _ in got) <= set(q.hex() for q in truth[s].payloads)


def test_long_recording_and_large_batch(gpu, oracle):
    """Sizes beyond one slot: a 61-s recording (four slots' worth of frames, signals in each) decodes
    like the oracle; a 1024-slot batch (every grid dimension 4x the bench's) equals per-slot decodes
    on a sample of its slots."""
    import torch
    from ft8_demodulator_amd import SlotDecoder, decode_ft8_message, synth
    kw = dict(max_candidates=300, min_score=2, max_iterations=20)
    parts, _ = synth.make_slots(4, 12, seed=4100, device="cpu", snr_db=(-16.0, -8.0))
    x = np.concatenate([parts.numpy().reshape(-1), np.zeros(12000, np.float32)])   # 61 s
    got = decode_ft8_message(x, 12000, **kw)
    ref = oracle.decode_ft8_message(x, 12000, **kw)
    assert sorted((m.payload.hex(), m.hash, t, f) for m, _s, t, f, _sc in got) == \
        sorted((p.hex(), h, t, f) for (p, h, _e, _ce, _cc, t, f, _sc) in ref)
    assert len(got) >= 1   # the reference heap keeps the first K passing candidates in scan (time) order
    big, _ = synth.make_slots(1024, 20, seed=5000, device="cuda")
    dec = SlotDecoder(12000, **kw)
    per_slot = dec.decode(big)
    for s in (0, 1, 511, 777, 1023):
        assert _rows(per_slot[s]) == _rows(decode_ft8_message(big[s].cpu().numpy(), 12000, **kw)), s
    del big
    torch.cuda.empty_cache()


def test_cli_several_files_equals_one_at_a_time(gpu, capsys):
    """The WAV CLI with several files (equal-length 16-bit PCM ones batched through the stream path,
    the 20-kHz one on its own) returns, per file, what the one-file call returns."""
    from ft8_demodulator_amd import decode_ft8_from_wave
    from ft8_demodulator_amd.from_wave import main
    files = [os.path.join(DATA, f) for f in ("synth_cfg1.wav", "ft8_fs20k_f0_550_id_1.wav", "synth_few.wav",
                                             "synth_cfg2.wav")]
    per_file = main(files + ["--max-candidates", "300", "--min-score", "2"])
    assert len(per_file) == len(files)
    for path, got in zip(files, per_file):
        assert _rows(got) == _rows(decode_ft8_from_wave(path, max_candidates=300, min_score=2)), path
    assert sum(len(r) for r in per_file) >= 3
    out = capsys.readouterr().out
    assert all(f"== {p}" in out for p in files)


def test_stft_i16_equals_f32(gpu):
    import torch
    from ft8_demodulator_amd import _device, read_wave_file
    from ft8_demodulator_amd.from_wave import _read_raw
    path = os.path.join(DATA, "ft8_fs20k_f0_550_id_1.wav")
    raw, _, fs = _read_raw(path)
    x, _ = read_wave_file(path)
    a, _, _ = _device.stft(x, fs, 2, 2)
    # int16 PCM through the C-ABI: the device applies read_wave_file's float32 x/32767 scaling
    import ctypes
    from ft8_demodulator_amd import _lib
    from ft8_demodulator_amd._pipeline import make_plan
    plan = make_plan(len(raw), fs)
    p = _lib.Ft8Params()
    p.sample_rate, p.bins_per_tone, p.steps_per_symbol = fs, 2, 2
    p.f_lo, p.f_hi, p.t_lo, p.t_hi = 0, plan.nfft, 0, plan.frames
    xi = torch.from_numpy(raw.copy()).cuda()
    out = torch.empty(plan.frames, plan.nfft, dtype=torch.float32, device="cuda")
    ctx = _lib.context()
    ctx.check(_lib.lib().ft8_stft(ctx.handle, _lib.ptr(xi), _lib.FT8_I16, len(raw), 1, len(raw), ctypes.byref(p),
                                  _lib.ptr(out), _lib.stream_handle()), "stft")
    assert torch.equal(out, a)


def test_pipeline_settings_do_not_change_results(gpu):
    """ft8_decode_batch cut into slot chunks over internal streams returns the same records as one
    chain on the caller's stream."""
    from ft8_demodulator_amd import SlotDecoder, synth
    x, _ = synth.make_slots(40, 30, seed=4242, device="cuda")
    dec = SlotDecoder(12000, 2, 2, 100, 3, 20)
    got = {}
    for cfg in [(0, 0, 4), (0, 0, 2), (8, 2, 2), (16, 3, 1), (7, 2, 4)]:
        dec.ctx.set_pipeline(*cfg)
        out, cnt = dec.run(x)
        got[cfg] = (out.cpu().numpy().tobytes(), cnt.cpu().numpy().tobytes())
    dec.ctx.set_pipeline()
    base = got[(0, 0, 4)]
    assert sum(np.frombuffer(base[1], np.int32)) > 0
    for cfg, v in got.items():
        assert v == base, cfg


def test_stream_decoder_matches_resident_decode(gpu):
    """Host PCM batches through the triple-buffered upload path == decoding the same int16 slots
    already resident on the GPU (and the per-file WAV helper == decode_ft8_from_wave)."""
    import torch
    from ft8_demodulator_amd import SlotDecoder, synth
    from ft8_demodulator_amd.stream import StreamDecoder, decode_wave_files
    x, _ = synth.make_slots(24, 20, seed=99, device="cuda")
    pcm = torch.clamp(torch.round(x / x.abs().amax() * 30000.0), -32767, 32767).to(torch.int16).cpu().numpy()
    kw = dict(max_candidates=100, min_score=3, max_iterations=20)
    ref = SlotDecoder(12000, **kw).decode(torch.from_numpy(pcm).cuda())
    key = lambda rs: [[(m.payload.hex(), s.crc_calculated, t, f, float(sc)) for (m, s, t, f, sc) in r] for r in rs]
    # depth 1 (one decoder), 2 (the default: two contexts/streams) and 3; ragged last batches
    for depth in (1, 2, 3):
        sd = StreamDecoder(pcm.shape[1], max_batch=8, depth=depth, **kw)
        got = []
        for res in sd.decode_batches([pcm[0:8], pcm[8:16], pcm[16:21], pcm[21:24]]):
            got.extend(res)
        assert key(got) == key(ref), depth
        # a second pass over the same decoder (buffers and events reused), as pinned tensors
        got = []
        pinned = torch.from_numpy(pcm).pin_memory()
        for res in sd.decode_batches([pinned[0:8], pinned[8:16], pinned[16:24]]):
            got.extend(res)
        assert key(got) == key(ref), depth
        # lent pinned batches (no host wait on uploads)
        got = []
        for res in sd.decode_batches([pinned[0:8], pinned[8:16], pinned[16:21], pinned[21:24]], borrow=True):
            got.extend(res)
        assert key(got) == key(ref), depth
    assert sum(len(r) for r in got) > 0
    # buffer recycling: at least 2 (depth + 2) batches so every device, pinned-input and
    # pinned-output buffer is reused (and decode_batches' start-next-upload-before-waiting path
    # runs on reused buffers), ragged last batch; then borrow=True with the caller cycling through
    # depth + 3 pinned buffers and rewriting each right after its batch's results are yielded
    for depth in (2, 3):
        sd = StreamDecoder(pcm.shape[1], max_batch=2, depth=depth, **kw)
        nb = 2 * (depth + 2) + 1
        order = [(3 * j) % 24 for j in range(nb * 2)]          # slots in a permuted order
        chunks = [pcm[order[2 * j:2 * j + 2]] for j in range(nb - 1)] + [pcm[order[2 * nb - 2:2 * nb - 1]]]
        got = []
        for res in sd.decode_batches(chunks):
            got.extend(res)
        exp = [ref[s] for c in range(nb) for s in order[2 * c:2 * c + (2 if c < nb - 1 else 1)]]
        assert key(got) == key(exp), depth
        ring = [torch.empty((2, pcm.shape[1]), dtype=torch.int16).pin_memory() for _ in range(depth + 3)]

        def lent():
            for j, c in enumerate(chunks):
                buf = ring[j % len(ring)]
                buf[:c.shape[0]].copy_(torch.from_numpy(c))
                yield buf[:c.shape[0]]

        got = []
        for j, res in enumerate(sd.decode_batches(lent(), borrow=True)):
            got.extend(res)
            ring[j % len(ring)].fill_(0)     # the caller rewrites a buffer once its results are back
        assert key(got) == key(exp), ("borrow", depth)
    from ft8_demodulator_amd import decode_ft8_from_wave
    wavs = [os.path.join(DATA, n) for n in ("synth_cfg1.wav", "synth_cfg2.wav")]
    files = decode_wave_files(wavs, batch=2)
    for w, r in zip(wavs, files):
        assert key([r]) == key([decode_ft8_from_wave(w)])


def test_decode_batch_orders_equal_scores_like_the_reference(gpu, oracle):
    """ft8_decode_batch leaves equal scores in scan order through LLR/BP (warn bit 3), replays the
    reference heap in k_llr's first workgroups and lets k_compact apply the order: every record's
    cand_index, time, frequency and score follow the oracle's heapq order of the same score grid,
    and the tie flag (bit 0) matches.  Such slots are rare (about 1 in 100 of the bench workload's,
    depending on the waterfall's last bits), so batches of the bench workload are drawn until one
    holds them."""
    import torch
    from ft8_demodulator_amd import FT8Waterfall, SlotDecoder, _device, _lib, synth
    from ft8_demodulator_amd._pipeline import make_plan
    dec = SlotDecoder(12000, 2, 2, 300, 2, 20)
    for seed in (100000, 200000, 300000, 400000, 500000, 600000):
        x, _ = synth.make_slots(256, 50, seed=seed, device="cuda")
        recs = dec.records(x)
        w = torch.zeros(256, dtype=torch.int32, device="cuda")
        dec.ctx.check(_lib.lib().ft8_select_warnings(dec.ctx.handle, _lib.ptr(w), 256, _lib.stream_handle()),
                      "warn")
        w = w.cpu().numpy()
        slots = np.nonzero(w & 8)[0]
        if len(slots):
            break
    assert len(slots) >= 1 and np.all(w[slots] & 4)
    plan = make_plan(x.shape[1], 12000, 2, 2)
    checked = 0
    for s in slots:
        wf, _, _ = _device.stft(x[s], 12000, 2, 2, plan.f_lo, plan.f_hi, plan.t_lo, plan.t_hi)
        mag = np.ascontiguousarray(wf.cpu().numpy().T)
        grid = oracle.score_grid(mag, 2, 2)
        t0, _, NF = _device.grid_shape(mag.shape[1], mag.shape[0], 2, 2)
        idx, sc, tie = oracle.select(grid, 300, 2)
        exp = [(int(i // NF) + t0, int(i % NF)) for i in idx]
        cands, _, warn = _device.sync_select(FT8Waterfall(mag=mag, time_osr=2, freq_osr=2), 300, 2)
        assert [(c[0], c[1]) for c in cands] == exp, s
        assert bool(w[s] & 1) == tie == bool(warn & 1), s
        for r in recs[s]:
            c = int(r["cand_index"])
            assert (int(r["abs_time"]), int(r["abs_freq"])) == exp[c], (s, c)
            assert np.float32(r["score"]) == sc[c], (s, c)
            checked += 1
    assert checked > 0


@pytest.mark.gpu
def test_packed_records_on_device(gpu):
    """ft8_pack_decodes (the N > 1 exchange's device packing) on real decode output: the packed rows
    are every slot's decodes in slot order, identical to SlotDecoder.records(); with a capacity
    below the total, the rest lands in the overflow rows in order."""
    import numpy as np
    import torch
    from ft8_demodulator_amd import SlotDecoder, _lib, synth
    from ft8_demodulator_amd.distributed import header_bytes, pack_decodes
    x, _ = synth.make_slots(12, 30, seed=321, device="cuda")
    dec = SlotDecoder(12000, 2, 2, 300, 2, 20)
    out, counts = dec.run(x)
    send, _ = pack_decodes(out, counts, dec.cap, 64)
    torch.cuda.synchronize()
    per_slot = dec.records(x)
    want = np.concatenate([r for r in per_slot]) if per_slot else np.zeros(0, _lib.RESULT_DTYPE)
    h = header_bytes(12)
    total = int(send[:8].cpu().view(torch.int64))
    assert total == len(want) >= 3
    assert send[8:8 + 48].cpu().view(torch.int32).tolist() == counts.cpu().tolist()
    got = send[h:h + 40 * total].cpu().numpy().view(_lib.RESULT_DTYPE)
    assert got.tobytes() == want.tobytes()
    small, over = pack_decodes(out, counts, dec.cap, 3)
    rows = small[h:].cpu().numpy().view(_lib.RESULT_DTYPE)
    assert int(small[:8].cpu().view(torch.int64)) == len(want) and len(rows) == 3
    assert rows.tobytes() == want[:3].tobytes()
    assert over[: total - 3].cpu().numpy().tobytes() == want[3:].tobytes()


@pytest.mark.parametrize("band", [(800.0, 2300.0), (0.0, 1500.0), (2000.0, None)])
def test_band_limited_production_geometry_matches_oracle(gpu, oracle, band):
    """12 kHz slots decoded with freq_min / freq_max: the production STFT's band-limited epilogue
    (kept bins f_lo .. f_lo + nf_out of the 3840-point real FFT, post-twiddles by recurrence) and
    the narrowed candidate grid decode exactly what the oracle decodes with the same band; time
    limits too."""
    from ft8_demodulator_amd import decode_ft8_message, synth
    x, _ = synth.make_slots(3, 40, seed=4242, device="cpu")
    kw = dict(max_candidates=200, min_score=2, max_iterations=20, freq_min=band[0], freq_max=band[1])
    if band[1] is None:
        kw.update(time_min=1.0, time_max=12.0)
    n_dec = 0
    for s in range(x.shape[0]):
        xs = x[s].numpy()
        got = decode_ft8_message(xs, 12000, **kw)
        ref = oracle.decode_ft8_message(xs, 12000, **kw)
        n_dec += len(ref)
        assert sorted((m.payload.hex(), m.hash, t, f) for m, _s, t, f, _sc in got) == \
            sorted((p.hex(), h, t, f) for (p, h, _e, _ce, _cc, t, f, _sc) in ref), (band, s)
        for (m, _s, t, f, sc), r in zip(sorted(got, key=lambda g: (g[2], g[3])), sorted(ref, key=lambda r: (r[5], r[6]))):
            assert abs(float(sc) - float(r[7])) <= 1e-4
    assert n_dec >= 3
