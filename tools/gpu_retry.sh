# Host-side: run one gpurun call (tools/gpu_call.sh) and, only when gpurun reports that nothing ran
# (status "transient": no box free / the box went away while being prepared; nothing charged),
# try again after a pause, at most 8 times.  A call that ran -- passed or failed -- is never repeated.
#   usage: bash tools/gpu_retry.sh TIMEOUT 'command' LOG
cd "$(dirname "$0")/.."
for i in 1 2 3 4 5 6 7 8; do
  bash tools/gpu_call.sh "$1" "$2" > "$3" 2>&1
  if grep -q "status=transient" "$3"; then
    echo "[gpu_retry] attempt $i: nothing ran (transient); retrying in 120 s" >> "$3.retries"
    sleep 120
    continue
  fi
  break
done
