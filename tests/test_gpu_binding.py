"""The reference-side ctypes binding (examples/reference_binding.py): torch-free
hipMalloc + ft8_decode_batch reproduces the reference's golden decodes of the WAV cases."""
import importlib.util
import os

import numpy as np
import pytest

from conftest import DATA, ROOT

pytestmark = pytest.mark.gpu


def _load_binding():
    os.environ.setdefault("FT8HIP_LIB", os.path.join(ROOT, "ft8_demodulator_amd", "lib", "libft8hip.so"))
    spec = importlib.util.spec_from_file_location("reference_binding",
                                                  os.path.join(ROOT, "examples", "reference_binding.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_reference_binding_matches_golden(golden, gpu):
    from ft8_demodulator_amd import read_wave_file
    rb = _load_binding()
    meta, _ = golden
    seen = 0
    for case in meta["e2e"]:
        if "wav" not in case or case.get("as_float64") or case.get("as_analytic") or case["error"]:
            continue
        x, fs = read_wave_file(os.path.join(DATA, case["wav"]))
        got = rb.decode_ft8_message(x, fs, **case["kwargs"])
        exp = case["results"]
        assert [(m.payload.hex(), m.hash, s.ldpc_errors, s.crc_extracted, s.crc_calculated, t, f)
                for (m, s, t, f, _) in got] == \
               [(r["payload"], r["hash"], r["ldpc_errors"], r["crc_extracted"], r["crc_calculated"],
                 r["time_sec"], r["freq_hz"]) for r in exp], case["name"]
        assert np.allclose([float(g[4]) for g in got], [r["score"] for r in exp], rtol=0, atol=2e-3)
        assert all(isinstance(g[4], np.float32) for g in got)
        seen += 1
    assert seen >= 7
    assert rb.decode_ft8_message(np.zeros(1000, np.float32), 12000) == []
