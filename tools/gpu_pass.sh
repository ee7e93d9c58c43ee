# One parametrised GPU pass (replaces the per-round gpu_r*.sh one-offs).  Runs ON the GPU box:
#   bash tools/gpu_call.sh 1100 'bash tools/gpu_pass.sh TAG STEP [STEP ...]'
# Steps run in the order given, each under its own time limit, and the pass stops at the first
# failure (no retries).  Outputs go to gpurun_out/TAG_*.
#   tests            the whole `pytest -m gpu` suite
#   tests=EXPR       `pytest -m gpu -k EXPR`
#   smoke            __graft_entry__.smoke()
#   pmc              PMC passes over tools/bp_only.py (gpu_pmc_r3.sh): SQ x2, FETCH_SIZE, WRITE_SIZE; the
#                    build-stamped JSON summaries are copied into the box's profiles/ so a later bench
#                    step in the same pass reports this build's traffic (copy them here to commit)
#   bench            bench.py at its defaults
#   driver           the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#   prof             rocprofv3 --kernel-trace --stats of the headline workload (gpu_prof.sh)
#   prof1            the same at --depth 1 without the single-call leg: every k_bp launch is one
#                    un-overlapped 256-slot launch, so the --stats average is the line's launch_ms
#   subprof          the config-4 subtract leg under a kernel trace + FETCH/WRITE/SQ passes (gpu_sub_prof.sh)
#   rehearse=N       the N > 1 path with N ranks sharing cuda:0 over gloo (not a measurement)
#   legs             bench.py with every side leg on (sensitivity included), legs file TAG_legs.json
set -o pipefail
T=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
run() {  # name seconds command...
  local n=$1 s=$2
  shift 2
  echo "[$(date +%T)] $T $n" >&2
  timeout -k 10 "$s" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[$(date +%T)] $T $n FAILED rc=$rc" >&2; exit $rc; fi
}
for st in "$@"; do
  case "$st" in
    tests) run tests 900 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu \
             > gpurun_out/${T}_tests.log 2>&1 ;;
    tests=*) run tests 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu \
               -k "${st#tests=}" > gpurun_out/${T}_tests.log 2>&1 ;;
    smoke) run smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 ;;
    pmc) run pmc 700 bash tools/gpu_pmc_r3.sh ${T} &&
         cp gpurun_out/${T}_pmc.json gpurun_out/${T}_pmc2.json gpurun_out/${T}_pmc_traffic.json profiles/ ;;
    bench) run bench 600 python -u bench.py --legs-out gpurun_out/${T}_legs.json \
             > gpurun_out/${T}_bench.json.log 2> gpurun_out/${T}_bench.err ;;
    driver) run driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --legs-out gpurun_out/${T}_driver_legs.json \
              > gpurun_out/${T}_driver.json.log 2> gpurun_out/${T}_driver.err ;;
    prof) run prof 400 bash tools/gpu_prof.sh ${T} ;;
    prof1) run prof1 400 bash tools/gpu_prof.sh ${T}_d1 --depth 1 --no-single-call ;;
    subprof) run subprof 900 bash tools/gpu_sub_prof.sh ${T} ;;
    rehearse=*) n=${st#rehearse=}
        run rehearse 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
          --master-port 29533 bench.py --gpus $n --share-gpu --steps 10 --warmup 3 \
          --legs-out gpurun_out/${T}_rehearse${n}_legs.json \
          > gpurun_out/${T}_rehearse${n}.json.log 2> gpurun_out/${T}_rehearse${n}.err ;;
    legs) run legs 900 python -u bench.py --sensitivity --legs-out gpurun_out/${T}_legs_full.json \
            > gpurun_out/${T}_legs.json.log 2> gpurun_out/${T}_legs.err ;;
    *) echo "unknown step $st" >&2; exit 2 ;;
  esac
done
echo "[$(date +%T)] $T done" >&2
