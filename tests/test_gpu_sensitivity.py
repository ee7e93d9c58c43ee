"""bench.sensitivity -- the reference's sensitivity harness (test_ft8_standard.py:43-123) on the GPU --
at a small size: two rates (one on the chirp-z STFT), a few SNR points and rounds.  The success rule
(first SNR with >= 50 % decodes), the table's shape and the oracle sample's parity (payload lists of
the same float64 bytes through oracle/ft8_oracle.c + scipy) are checked; the full sweep is the bench
leg's."""
import pytest

pytestmark = pytest.mark.gpu


def test_sensitivity_small(gpu):
    import bench
    import torch
    out = bench.sensitivity(torch.device("cuda", 0), rates=[4000, 5500], snr_lo=-20.0, snr_hi=-8.0, step=2.0,
                            rounds=4, oracle_per_rate=2, procs=4)
    assert [r["fs"] for r in out["table"]] == [4000, 5500]
    assert out["slots"] == 2 * 7 * 4
    for r in out["table"]:
        # clean-ish slots at -8 dB decode (the reference's harness decodes these rates well above
        # its thresholds), so every rate has a threshold inside the sweep
        assert r["min_snr_db"] is not None and -20.0 <= r["min_snr_db"] <= -8.0
        assert r["xlsx_min_snr_db"] is None or isinstance(r["xlsx_min_snr_db"], int)
    par = out["parity"]
    assert par["slots"] == 4 and par["equal"] == par["slots"], par["mismatches"]
    assert out["cpu_baseline"]["cores"] == 4 and out["cpu_baseline"]["value"] > 0
