# Round-5 pass A: the new tests (context reuse, race control, 24/48 kHz subtraction), the whole GPU
# suite, then the whole suite on the barrier-race check build (its prologue now fills the real LDS
# allocation: group_segment_size at offset 28 of the dispatch packet).
set -o pipefail
T=${1:-r5a}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -rP --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_context_reuse.py tests/test_gpu_race_control.py "tests/test_gpu_tx.py::test_subtract_clean_signal_residual" \
  > gpurun_out/${T}_new.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
FT8HIP_LIB=$R/variants/RACE.so FT8HIP_ALLOW_STALE=1 timeout -k 10 900 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_race_tests.log 2>&1
