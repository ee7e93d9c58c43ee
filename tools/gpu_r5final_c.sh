# Round-5 closing pass on the final tree: GPU suite, smoke, the bench line at its defaults and at the
# driver's exact command.  usage: bash tools/gpu_r5final_c.sh TAG
set -o pipefail
T=${1:-r5_w6}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json.log 2> gpurun_out/${T}_bench.err &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver.json.log 2> gpurun_out/${T}_bench_driver.err
