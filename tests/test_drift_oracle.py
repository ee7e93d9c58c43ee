"""The drift-correction oracle (oracle/drift.py) against the reference's own outputs (CPU).

tests/golden/drift.{json,npz} were written by tools/make_golden_drift.py, which imported the
reference's frequency_correction.py (src/ft8_tools/ft8_beacon_receiver) in the build container and
ran it on beacon inputs regenerated here from their parameters.  Checked per case: the per-frame
argmax of both spectrograms (exact), the continuity segments (exact), the continuity metric, the
estimated rate and a strided subsample of the corrected waveform."""
import numpy as np
import pytest

from oracle import drift as OD


def _cases(drift_golden):
    return drift_golden[0]["cases"]


def test_beacon_input_shape(drift_golden, drift_inputs):
    for c in _cases(drift_golden):
        x = drift_inputs[c["name"]]
        assert x.dtype == np.complex128 and x.shape == (c["n_samples"],)


@pytest.mark.parametrize("idx", range(10))
def test_oracle_matches_reference(drift_golden, drift_inputs, idx):
    meta, arr = drift_golden
    if idx >= len(meta["cases"]):
        pytest.skip("fewer golden cases")
    c = meta["cases"][idx]
    nm = c["name"]
    tr = {}
    y, rate = OD.correct_frequency_drift(drift_inputs[nm], c["fs"], 6.25, 0.16, params=c["params"], trace=tr)
    assert tr["status"] == c["status"], nm
    assert np.array_equal(tr["argmax1"], arr[f"{nm}/argmax1"]), nm
    assert [tuple(s) for s in tr["segments"]] == [tuple(s) for s in arr[f"{nm}/segments"].tolist()], nm
    assert np.allclose(tr["metric"], arr[f"{nm}/metric"], rtol=1e-9, atol=1e-9), nm
    assert abs(float(rate) - c["rate_per_sample"]) <= 1e-12 * max(1.0, abs(c["rate_per_sample"])), nm
    if f"{nm}/argmax2" in arr:
        assert np.array_equal(tr["argmax2"], arr[f"{nm}/argmax2"]), nm
    stride = meta["subsample_stride"]
    assert np.max(np.abs(np.asarray(y)[::stride] - arr[f"{nm}/corrected_sub"])) < 1e-9, nm


def test_detect_signal_continuity_edge_cases():
    segs, m = OD.detect_signal_continuity(np.arange(5), window_size=8)
    assert segs == [] and m.shape == (5,)
    # a perfect line is one segment that runs to len - 1 (frequency_correction.py:111-112)
    segs, m = OD.detect_signal_continuity(np.arange(40) * 3, window_size=8, max_variance=1.0)
    assert segs == [(0, 39)] and np.allclose(m, 0.0, atol=1e-9)
