"""Stage-by-stage parity of the HIP kernels against the reference's golden vectors and the oracle.

Waterfall injection: the reference's own waterfalls (tests/golden) are fed to the GPU sync /
selection / LLR / BP kernels, so every downstream stage is compared bit-for-bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _wf(mag, sps, bpt):
    from ft8_demodulator_amd import FT8Waterfall
    return FT8Waterfall(mag=mag, time_osr=sps, freq_osr=bpt)


def test_score_grid_bit_exact(golden, gpu):
    from ft8_demodulator_amd import ft8_score_grid
    meta, arr = golden
    for c in meta["sync"]:
        mag = arr[f"sync_{c['name']}_mag"]
        g = ft8_score_grid(_wf(mag, c["sps"], c["bpt"]))
        ref = arr[f"sync_{c['name']}_grid"]
        assert g.dtype == ref.dtype, c["name"]
        assert g.shape == ref.shape, c["name"]
        assert np.array_equal(g.view(np.uint8), ref.view(np.uint8)), c["name"]


def test_score_grid_bpt10_bit_exact(gpu, oracle):
    """k_score2 at bins_per_tone = steps_per_symbol = 10 (round 4; the reference decode test's
    geometry, test_spectrogram_analyse.py:128-163): full grid bit-exact against the oracle (which
    follows ft8_decode.py:47-100), and the compact-layout selections (reference heap and top-k)
    equal the full-grid ones, on a waterfall with strong tones over noise."""
    from ft8_demodulator_amd import _device, ft8_score_grid
    rng = np.random.default_rng(1010)
    F, T = 1200, 940   # 10x oversampled: 120 tones x 94 blocks
    mag = (rng.standard_normal((F, T)) * 3.0 - 70.0).astype(np.float32)
    mag[300:310, 100:890] += 25.0
    mag[700:705, 40:600] += 18.0
    wf = _wf(mag, 10, 10)
    g = ft8_score_grid(wf)
    ref = oracle.score_grid(mag, 10, 10)
    assert g.shape == ref.shape and g.dtype == ref.dtype
    assert np.array_equal(g.view(np.uint8), ref.view(np.uint8))
    for N, ms, flags in ((300, 2, 0), (1000, 0.5, 0), (300, 2, 1), (4096, -100, 1)):
        compact, _, w1 = _device.sync_select(wf, N, ms, flags=flags)
        full, _, w2 = _device.sync_select(wf, N, ms, want_grid=True, flags=flags)
        assert compact == full and w1 == w2, (N, ms, flags)
        if flags == 0:
            idx, sc, tie = oracle.select(ref, N, ms)
        else:
            idx, sc = oracle.select_topk(ref, N, ms)
        NF = ref.shape[1]
        assert [(a, b) for a, b, _ in compact] == [(int(i // NF) - 100, int(i % NF)) for i in idx], (N, ms, flags)


def test_candidates_exact(golden, gpu):
    from ft8_demodulator_amd import _device, ft8_find_candidates
    meta, arr = golden
    n = n_err = 0
    for c in meta["sync"]:
        mag = arr[f"sync_{c['name']}_mag"]
        wf = _wf(mag, c["sps"], c["bpt"])
        for s in c["sel"]:
            _, _, warn = _device.sync_select(wf, s["N"], s["min_score"])
            # bit 0 <=> the reference raised TypeError (an exact tie reached a heap comparison)
            assert bool(warn & 1) == (s["error"] is not None), (c["name"], s["N"], s["min_score"], warn)
            if s["error"] is not None:
                n_err += 1
                continue
            got = ft8_find_candidates(wf, s["N"], s["min_score"])
            assert [[x.abs_time, x.abs_freq] for x in got] == s["cands"], (c["name"], s["N"], s["min_score"])
            if s["cands"]:
                sc = arr[f"sync_{c['name']}_N{s['N']}_ms{s['min_score']}_scores"]
                gs = np.array([x.score for x in got], dtype=sc.dtype)
                assert np.array_equal(gs, sc)
                assert type(got[0].score) is type(sc[0])
            n += 1
    assert n >= 15 and n_err >= 1


def test_llr_bit_exact(golden, gpu):
    from ft8_demodulator_amd import ft8_extract_likelihood, ftx_normalize_logl
    from ft8_demodulator_amd import _device
    meta, arr = golden
    for c in meta["sync"]:
        mag = arr[f"sync_{c['name']}_mag"]
        wf = _wf(mag, c["sps"], c["bpt"])
        for s in c["sel"]:
            key = f"sync_{c['name']}_N{s['N']}_ms{s['min_score']}_llr"
            if s["error"] is not None or key not in arr.files:
                continue
            cands = s["cands"][: arr[key].shape[0]]
            raw = _device.llr(wf, cands, normalize=False)
            assert np.array_equal(raw, arr[key + "_raw"]), key
            with np.errstate(all="ignore"):
                nl = _device.llr(wf, cands, normalize=True)
            assert np.array_equal(nl.view(np.uint64), arr[key].view(np.uint64)), key
    # the mirror functions (in place)
    cands = meta["sync"][0]["sel"][1]["cands"]
    wf = _wf(arr["sync_rand32_mag"], 2, 2)
    from ft8_demodulator_amd import FT8Candidate
    x = np.zeros(174)
    ft8_extract_likelihood(wf, FT8Candidate(wf, *cands[0]), x)
    assert np.array_equal(x, arr["sync_rand32_N50_ms2_llr_raw"][0])
    ftx_normalize_logl(x)
    assert np.array_equal(x, arr["sync_rand32_N50_ms2_llr"][0])


def test_wav_waterfall_injection(golden, gpu, oracle):
    """Reference WAV waterfall (scipy, pinned by sha256) -> GPU grid / candidates / LLR / decode."""
    import hashlib
    from ft8_demodulator_amd import FT8Candidate, ft8_decode_candidate, ft8_find_candidates, ft8_score_grid
    from ft8_demodulator_amd import _device, read_wave_file
    meta, arr = golden
    x, fs = read_wave_file(f"{__import__('conftest').DATA}/ft8_fs20k_f0_550_id_1.wav")
    mag = oracle.waterfall(x, fs)
    assert hashlib.sha256(mag.tobytes()).hexdigest() == meta["wav_waterfall"]["sha256"]
    wf = _wf(mag, 2, 2)
    g = ft8_score_grid(wf)
    assert hashlib.sha256(g.tobytes()).hexdigest() == meta["wav_grid"]["sha256"]
    cands = ft8_find_candidates(wf, 20, 10)
    assert [[c.abs_time, c.abs_freq] for c in cands] == arr["wav_cands"].tolist()
    assert np.array_equal(np.array([c.score for c in cands], dtype=np.float32), arr["wav_scores"])
    l = _device.llr(wf, arr["wav_cands"].tolist(), normalize=True)
    assert np.array_equal(l, arr["wav_llr"])
    for c, st in zip(cands, arr["wav_cand_status"]):
        ok, m, s = ft8_decode_candidate(wf, c, 20)
        assert [int(ok), s.ldpc_errors, s.crc_extracted, s.crc_calculated] == st.tolist()


def test_bp_golden(golden, gpu):
    from ft8_demodulator_amd import _device
    meta, arr = golden
    llr, iters, plain, errs = arr["bp_llr"], arr["bp_iters"], arr["bp_plain"], arr["bp_errors"]
    for it in sorted(set(iters.tolist())):
        sel = np.nonzero(iters == it)[0]
        p, rec = _device.bp(llr[sel], int(it))
        assert np.array_equal(p, plain[sel]), it
        assert np.array_equal(rec["ldpc_errors"].astype(np.int32), errs[sel]), it
        for k, i in enumerate(sel):
            t = meta["bp_tail"][i]
            assert bool(rec[k]["ok"]) == t["ok"]
            if t["ok"]:
                assert bytes(rec[k]["payload"]).hex() == t["payload"]
            assert int(rec[k]["crc_extracted"]) == t["crc_extracted"]
            assert int(rec[k]["crc_calculated"]) == t["crc_calculated"]


def test_bp_random_vs_oracle(gpu, oracle):
    """2000 noisy codewords across the waterfall of convergence: plain bits and min errors bit-exact."""
    from ft8_demodulator_amd import _device, synth
    rng = np.random.default_rng(123)
    n = 2000
    llrs = np.empty((n, 174))
    for i in range(n):
        bits = synth.codeword_bits(synth.random_payload(rng)).astype(np.float64)
        sigma = 0.5 + 1.2 * (i % 20) / 19
        llrs[i] = oracle.normalize((2 * bits - 1) + sigma * rng.standard_normal(174))
    for it in (20, 50):
        p, rec = _device.bp(llrs, it)
        for i in range(0, n, 7 if it == 50 else 1):
            pr, er = oracle.bp_decode(llrs[i], it)
            assert er == int(rec[i]["ldpc_errors"]), (it, i)
            assert np.array_equal(pr, p[i]), (it, i)


def test_bp_short_iteration_counts_vs_oracle(gpu, oracle):
    """max_iterations 0..4: no sweep at all, the first sweep alone (k_bp evaluates fast_tanh once per
    variable there), and the last sweep that stops after the parity check -- all bit-exact."""
    from ft8_demodulator_amd import _device, synth
    rng = np.random.default_rng(321)
    n = 300
    llrs = np.empty((n, 174))
    for i in range(n):
        bits = synth.codeword_bits(synth.random_payload(rng)).astype(np.float64)
        llrs[i] = oracle.normalize((2 * bits - 1) + (0.4 + 1.0 * (i % 10) / 9) * rng.standard_normal(174))
    for it in (0, 1, 2, 3, 4):
        p, rec = _device.bp(llrs, it)
        for i in range(n):
            pr, er = oracle.bp_decode(llrs[i], it)
            assert er == int(rec[i]["ldpc_errors"]), (it, i)
            assert np.array_equal(pr, p[i]), (it, i)


def test_normalize_random_vs_oracle(gpu, oracle):
    from ft8_demodulator_amd import _device
    rng = np.random.default_rng(5)
    x = rng.standard_normal((500, 174)) * rng.uniform(0.1, 50, (500, 1)) + rng.uniform(-3, 3, (500, 1))
    got = _device.normalize(x)
    for i in range(500):
        assert np.array_equal(got[i].view(np.uint64), oracle.normalize(x[i]).view(np.uint64)), i


def test_crc_and_check(golden, gpu, oracle):
    from ft8_demodulator_amd import compute_crc, extract_crc, ldpc_check, pack_bits, add_crc, synth
    meta, _ = golden
    for r in meta["crc"]:
        d = bytearray.fromhex(r["data"])
        assert compute_crc(d, r["nbits"]) == r["crc"]
        assert extract_crc(d) == r["extract"]
        bits = np.array([int(ch) for ch in r["bits"]], dtype=np.uint8)
        assert bytes(pack_bits(bits, 91)).hex() == r["packed91"]
        assert ldpc_check(bits) == oracle.ldpc_check(bits)
    for t in meta["tx"]:
        a91 = bytearray(12)
        add_crc(bytearray.fromhex(t["payload"]), a91)
        assert bytes(a91).hex() == t["a91"]
        cw = np.unpackbits(np.frombuffer(bytes.fromhex(t["codeword"]), dtype=np.uint8))[:174]
        assert ldpc_check(cw) == 0


def test_bp_extreme_inputs_vs_oracle(gpu, oracle):
    """Inputs that drive messages to zero / subnormal / huge values exercise the full IEEE
    division path (the fast path needs 2^-960 <= |numerator| < 2^900), and NaN / infinite LLRs
    the NaN-preserving clip: still bit-exact."""
    from ft8_demodulator_amd import _device
    rng = np.random.default_rng(77)
    vecs = []
    for scale in (1e-300, 1e-200, 1e-100, 1e-12, 1.0, 1e12, 1e300):
        v = rng.standard_normal(174) * scale
        v[rng.random(174) < 0.3] = 0.0          # erasures: exact zeros
        vecs.append(v)
    v = np.zeros(174)
    v[::7] = 1e-310                             # subnormal inputs
    vecs.append(v)
    v = rng.standard_normal(174)
    v[:60] = 0.0
    vecs.append(v)
    # around k_bp's per-sweep short-division bound (|V->C argument| >= 2^-100, bp.hip sweep_fast):
    # whole vectors just above / below it, and normal vectors with one or a few arguments near it
    for scale in (2.0 ** -99, 2.0 ** -100, 2.0 ** -101, 1e-30, 1e-31):
        vecs.append(rng.standard_normal(174) * scale)
    for pos in ([0], [173], [5, 60, 120]):
        for tiny in (2.0 ** -100, 2.0 ** -100 * (1 - 2.0 ** -52), 2.0 ** -101, 5e-324):
            v = rng.standard_normal(174) * 3.0
            v[pos] = tiny * np.sign(rng.standard_normal(len(pos)))
            vecs.append(v)
    # NaN and infinite LLRs (bp_decode accepts any vector): np.clip keeps NaN, so it spreads
    for pos in ([3], [3, 50, 100, 171], list(range(0, 174, 5))):
        v = rng.standard_normal(174) * 2.0
        v[pos] = np.nan
        vecs.append(v)
    v = rng.standard_normal(174)
    v[[7, 8]] = np.inf
    v[[90]] = -np.inf
    vecs.append(v)
    vecs.append(np.full(174, np.nan))
    llrs = np.array(vecs)
    for it in (1, 5, 20, 50):
        p, rec = _device.bp(llrs, it)
        for i in range(len(vecs)):
            pr, er = oracle.bp_decode(llrs[i], it)
            assert er == int(rec[i]["ldpc_errors"]), (it, i)
            assert np.array_equal(pr, p[i]), (it, i)


def test_bp_stress_config4_vs_oracle(gpu, oracle):
    """BASELINE config 4 input (bench.py bp_stress): device-normalised LLRs, 50 iterations; hard
    decisions, min errors and CRC status bit-exact vs the oracle on 600 vectors."""
    from ft8_demodulator_amd import _device, synth
    llr, bits = synth.bp_stress_llrs(600, seed=11)
    x = _device.normalize(llr)
    p, rec = _device.bp(x, 50)
    conv = 0
    for i in range(600):
        xr = oracle.normalize(llr[i])
        assert np.array_equal(x[i].view(np.uint64), xr.view(np.uint64)), i
        pr, er = oracle.bp_decode(xr, 50)
        assert er == int(rec[i]["ldpc_errors"]) and np.array_equal(pr, p[i]), i
        ok, pay, ce, cc = oracle.decode_tail(pr, er)
        assert bool(rec[i]["ok"]) == ok and int(rec[i]["crc_calculated"]) == cc, i
        conv += er == 0
    assert 0.3 < conv / 600 < 0.7   # the ~50 % failure point the workload is defined at


def test_selection_with_ties_vs_oracle(gpu, oracle):
    """Quantised waterfalls give many exactly equal scores: the selected set, its order (heap-array
    order for equal scores, ties broken by scan index where the reference would raise) and the
    TypeError flag match the oracle's full heapq simulation, with and without records."""
    from ft8_demodulator_amd import _device
    rng = np.random.default_rng(2024)
    cases = 0
    for trial in range(12):
        F, T = 160 + 8 * trial, 186
        levels = (2, 3, 5, 8)[trial % 4]
        mag = rng.integers(0, levels, size=(F, T)).astype(np.float32) * 3.0
        if trial % 3 == 0:  # a ramp of strong late bins makes records beyond rank N
            mag[:, 150:] += np.linspace(0, 12, T - 150, dtype=np.float32)[None, :]
        wf = _wf(mag, 2, 2)
        grid = oracle.score_grid(mag, 2, 2)
        NF = grid.shape[1]
        for N, ms in ((5, 0), (50, 1), (300, 0), (1000, -100)):
            idx, sc, tie = oracle.select(grid, N, ms)
            cands, _, warn = _device.sync_select(wf, N, ms)
            exp = [(int(i // NF) - 20, int(i % NF)) for i in idx]
            assert [(c[0], c[1]) for c in cands] == exp, (trial, N, ms)
            assert np.array_equal(np.array([c[2] for c in cands]), sc), (trial, N, ms)
            assert bool(warn & 1) == tie, (trial, N, ms)
            cases += bool(warn & 4)
    assert cases >= 10   # the replay path ran


def test_sync_score_any_candidate_matches_reference(golden, gpu):
    """ft8_sync_score off the search grid (k_score_list): NumPy wrap-around of negative frequency
    indices, IndexError past the last bin, -inf when no block is comparable -- against the
    reference's own values (tests/golden/syncscore.json, tools/make_golden_syncscore.py)."""
    import json
    import os
    from conftest import GOLD
    from ft8_demodulator_amd import FT8Candidate, FT8Waterfall, ft8_sync_score
    _, arr = golden
    with open(os.path.join(GOLD, "syncscore.json")) as f:
        cases = json.load(f)
    for c in cases:
        mag = arr[f"sync_{c['case']}_mag"]
        wf = FT8Waterfall(mag=mag, time_osr=c["sps"], freq_osr=c["bpt"])
        cand = FT8Candidate(waterfall=wf, abs_time=c["abs_time"], abs_freq=c["abs_freq"])
        if c["error"]:
            with pytest.raises(IndexError):
                ft8_sync_score(wf, cand)
            continue
        v = ft8_sync_score(wf, cand)
        assert type(v).__name__ == c["dtype"], c
        assert float(v) == c["score"], c   # bit-exact (float32 widened exactly / float64)
    # on the grid it equals the grid kernel
    from ft8_demodulator_amd import ft8_score_grid
    from ft8_demodulator_amd.ft8_decode import ft8_sync_scores
    wf = FT8Waterfall(mag=arr["sync_rand32_mag"], time_osr=2, freq_osr=2)
    g = ft8_score_grid(wf)
    pts = [(-20 + i, j) for i in (0, 5, 37, g.shape[0] - 1) for j in (0, 1, 40, g.shape[1] - 1)]
    s = ft8_sync_scores(wf, pts)
    assert np.array_equal(s, np.array([g[t + 20, f] for t, f in pts], dtype=s.dtype))


def test_max_candidates_limit_is_an_error(gpu):
    """Deliberate deviation: the selection holds its candidates in LDS, so
    max_candidates above ft8_limits() (4096) is refused with FT8_E_RANGE (ValueError) rather than silently
    truncated; the reference has no cap (ft8_decode.py:102-149)."""
    from ft8_demodulator_amd import _lib, decode_ft8_message
    lim = _lib.limits()["max_candidates"]
    assert lim == 4096
    x = np.random.default_rng(1).standard_normal(180000).astype(np.float32)
    assert decode_ft8_message(x, 12000, max_candidates=lim, min_score=100) == []
    with pytest.raises(ValueError, match="max_candidates"):
        decode_ft8_message(x, 12000, max_candidates=lim + 1, min_score=100)


def test_compact_scores_select_like_the_full_grid(gpu, oracle):
    """Without a caller grid the score kernel writes only the passing scores of each 128-column
    segment plus its column mask, and k_select walks the masks; with a grid it reads the full grid.
    Both give the oracle's selection (ft8_decode.py:102-149) on dense, sparse and record-making
    waterfalls, ragged segment tails (NF not a multiple of 128) and N from 1 to the 4096 limit."""
    from ft8_demodulator_amd import _device
    rng = np.random.default_rng(77)
    n = 0
    for trial, (F, T) in enumerate(((135, 186), (520, 186), (1920, 186), (1000, 150), (300, 400))):
        mag = (rng.standard_normal((F, T)) * 6.0 - 60.0).astype(np.float32)
        if trial % 2 == 0:
            mag[:, -40:] += np.linspace(0, 20, 40, dtype=np.float32)[None, :]  # late records
        wf = _wf(mag, 2, 2)
        grid = oracle.score_grid(mag, 2, 2)
        NF = grid.shape[1]
        for N, ms in ((1, 0), (7, 2), (300, 2), (300, 6), (4096, -100), (2000, 1)):
            idx, sc, _ = oracle.select(grid, N, ms)
            exp = [(int(i // NF) - 20, int(i % NF)) for i in idx]
            compact, _, w1 = _device.sync_select(wf, N, ms)
            full, _, w2 = _device.sync_select(wf, N, ms, want_grid=True)
            assert compact == full and w1 == w2, (trial, N, ms)
            assert [(c[0], c[1]) for c in compact] == exp, (trial, N, ms)
            assert np.array_equal(np.array([c[2] for c in compact], dtype=np.float32).reshape(-1), sc), (trial, N, ms)
            n += 1
    assert n == 30
