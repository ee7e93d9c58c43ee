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


def test_c_example_matches_golden(golden, gpu):
    """examples/decode_wav.c: the C-ABI from plain C (WAV parsing, hipMalloc, ft8_decode_batch, the
    reference's time / frequency arithmetic) reproduces the reference's golden decodes of every WAV
    case it can express (the decode keywords without the band / time masks)."""
    import subprocess
    exe = os.path.join(ROOT, "examples", "decode_wav")
    if not os.path.exists(exe):
        pytest.fail("examples/decode_wav is not built (__graft_entry__.build() / make -C examples)")
    meta, _ = golden
    flag = {"max_candidates": "-k", "min_score": "-s", "max_iterations": "-i"}
    seen = 0
    for case in meta["e2e"]:
        if "wav" not in case or case.get("as_float64") or case.get("as_analytic") or case["error"]:
            continue
        if set(case["kwargs"]) - set(flag):
            continue
        args = [exe, os.path.join(DATA, case["wav"])]
        for k, v in case["kwargs"].items():
            args += [flag[k], str(v)]
        out = subprocess.run(args, capture_output=True, text=True, timeout=120, check=True).stdout.split("\n")
        got = [ln.split() for ln in out if ln.strip()]
        exp = case["results"]
        assert [(g[0], int(g[1]), int(g[2]), int(g[3]), float(g[4]), float(g[5])) for g in got] == \
               [(r["payload"], r["crc_calculated"], r["ldpc_errors"], r["crc_extracted"], r["time_sec"],
                 r["freq_hz"]) for r in exp], case["name"]
        assert np.allclose([float(g[6]) for g in got], [r["score"] for r in exp], rtol=0, atol=1e-4), case["name"]
        seen += 1
    assert seen >= 5
