"""CPU: the oracle's transmit-chain restatement (oracle/oracle.py) against the reference
generator's golden vectors, and the top-k selection oracle against a brute-force definition."""
import json
import os

import numpy as np

from conftest import GOLD


def test_oracle_encoder_known_answers(golden, oracle):
    meta, _ = golden
    for r in meta["tx"]:
        p = bytes.fromhex(r["payload"])
        a91 = oracle.crc_generator(p)
        assert a91.hex() == r["a91"]
        assert oracle.ldpc_encode(a91).hex() == r["codeword"]
        assert "".join(map(str, oracle.tx_itones(p))) == r["itones"]


def test_oracle_waveforms_vs_reference(oracle):
    meta = json.load(open(os.path.join(GOLD, "tx_wave.json")))
    arr = np.load(os.path.join(GOLD, "tx_wave.npz"), allow_pickle=False)
    for c in meta["cases"]:
        it = oracle.tx_itones(bytes.fromhex(c["payload"]))
        if c["kind"] == "freq":
            got = oracle.gfsk_freq_seq(it, c["fs"])
            assert np.array_equal(got, arr[c["name"]])
            continue
        bb = oracle.gfsk_waveform(it, c["fs"], c["f0"] + c["fc"], style=1)
        got = bb if c["kind"] == "baseband" else np.real(bb)
        assert got.shape[0] == c["length"]
        if c["segment"]:
            a0, a1, b0, b1 = c["segment"]
            got = np.concatenate([got[a0:a1], got[b0:b1]])
        # fc folded into f0: the reference rotates by exp(2j pi fc n / fs) separately
        tol = 0.0 if c["fc"] == 0 else 1e-10
        assert np.max(np.abs(got - arr[c["name"]])) <= tol, c["name"]


def test_select_topk_definition(oracle):
    rng = np.random.default_rng(2)
    for dt in (np.float32, np.float64):
        g = np.round(rng.normal(0, 3, size=(40, 57)), 1).astype(dt)  # many exact ties
        g[3, 4] = -np.inf
        g[5, 6] = np.nan
        for N, ms in ((1, 0), (25, 1.5), (5000, -100), (10, 100)):
            idx, sc = oracle.select_topk(g, N, ms)
            flat = g.reshape(-1)
            cand = [(-float(flat[i]), i) for i in range(flat.size)
                    if not np.isnan(flat[i]) and flat[i] != -np.inf and flat[i] >= dt(ms)]
            exp = [i for _, i in sorted(cand)[:N]]
            assert list(idx) == exp
            assert np.array_equal(sc, flat[exp].astype(np.float64))
