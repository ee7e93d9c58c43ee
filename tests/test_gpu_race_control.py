"""Positive control of the barrier-race check build: tools/probe/race_control.hip runs
ft8_internal.h's FT8_RACE_PROLOGUE -- the same code every multi-wave LDS kernel of the
-DFT8_RACE_CHECK library opens with -- in a kernel whose barrier can be left out.  Without the
barrier a wave must read another wave's slot before it was written (the sentinel), with it never;
and the sentinel fill must cover the whole LDS allocation, static and dynamic (the prologue sizes it
from the dispatch packet's group_segment_size)."""
import ctypes
import os

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

LIB = os.path.join(ROOT, "tools", "probe", "librace_control.so")


@pytest.fixture(scope="module")
def control(gpu):
    if not os.path.exists(LIB):
        pytest.skip("tools/probe/librace_control.so not built (make -C tools/probe)")
    lib = ctypes.CDLL(LIB)
    lib.ft8probe_race_control.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.ft8probe_race_control.restype = ctypes.c_int

    def run(barrier, workgroups, dyn_bytes):
        out = (ctypes.c_uint * 2)()
        rc = lib.ft8probe_race_control(barrier, workgroups, dyn_bytes, out)
        assert rc == 0, rc
        return int(out[0]), int(out[1])
    return run


@pytest.mark.parametrize("dyn_bytes", [0, 4096, 70 * 1024])
def test_missing_barrier_is_caught(control, dyn_bytes):
    raced, unfilled = control(0, 64, dyn_bytes)
    # every workgroup has one late wave; the wave before it reads 64 unwritten slots
    assert raced >= 64 * 64, raced
    assert unfilled == 0


@pytest.mark.parametrize("dyn_bytes", [0, 70 * 1024])
def test_barrier_passes(control, dyn_bytes):
    raced, unfilled = control(1, 64, dyn_bytes)
    assert raced == 0 and unfilled == 0
