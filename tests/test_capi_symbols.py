"""The C-ABI library loads and exports every entry point include/ft8hip.h declares (CPU only)."""
import ctypes
import os
import re

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "ft8hip.h")).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\*)\s+(ft8_\w+)\(", src, flags=re.M)))


def test_header_symbols_exported():
    from ft8_demodulator_amd import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    names = _declared()
    assert len(names) >= 17
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_lib.EXPORTED_SYMBOLS)


def test_host_entry_points_without_gpu():
    from ft8_demodulator_amd import _lib
    assert _lib.lib().ft8_abi_version() == 2
    # ABI 2: ft8_params ends with the double sample_rate_hz (64 bytes); the example binding agrees
    assert ctypes.sizeof(_lib.Ft8Params) == 64 and _lib.Ft8Params.sample_rate_hz.offset == 56
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("rb", os.path.join(root, "examples", "reference_binding.py"))
    rb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rb)
    assert [f[0] for f in rb.ft8_params._fields_] == [f[0] for f in _lib.Ft8Params._fields_]
    assert _lib.geometry(12000, 2, 2, 180000) == (1920, 960, 3840, 186)
    assert _lib.geometry(20000, 2, 2, 252800) == (3200, 1600, 6400, 157)
    assert _lib.geometry(12000, 2, 2, 1000)[3] == 0
    assert _lib.limits()["max_candidates"] == 4096


def test_c_example_compiles_against_the_header(tmp_path):
    """examples/decode_wav.c builds with gcc against include/ft8hip.h and links the in-tree
    libft8hip.so (the header is plain C; ft8_params is the 64-byte ABI-2 block there too)."""
    import shutil
    import subprocess
    gcc = shutil.which("gcc")
    if gcc is None:
        import pytest
        pytest.skip("no gcc")
    probe = tmp_path / "size.c"
    probe.write_text('#include "ft8hip.h"\n#include <stddef.h>\n'
                     '_Static_assert(sizeof(ft8_params) == 64, "ft8_params");\n'
                     '_Static_assert(offsetof(ft8_params, sample_rate_hz) == 56, "sample_rate_hz");\n'
                     '_Static_assert(sizeof(ft8_result) == 40, "ft8_result");\n'
                     'int main(void) { return 0; }\n')
    inc = os.path.join(ROOT, "include")
    subprocess.run([gcc, "-std=c11", "-Wall", "-Werror", "-I", inc, "-o", str(tmp_path / "size"), str(probe)],
                   check=True)
    lib = os.path.join(ROOT, "ft8_demodulator_amd", "lib")
    subprocess.run([gcc, "-O2", "-std=c11", "-Wall", "-Werror", "-I", inc, "-I", "/opt/rocm/include", "-o",
                    str(tmp_path / "decode_wav"), os.path.join(ROOT, "examples", "decode_wav.c"), "-L", lib,
                    "-lft8hip", "-L", "/opt/rocm/lib", "-lamdhip64"], check=True)
