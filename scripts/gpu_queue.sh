#!/bin/bash
# submit a gpurun command; re-submit ONLY when gpurun says no box / slot was free (status=transient:
# nothing ran, nothing charged), at most 8 times, 150 s apart.  Usage: scripts/gpu_queue.sh OUTFILE TIMEOUT 'cmd'
out=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6 7 8; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > "$out" 2>&1
  grep -q "status=transient" "$out" || exit 0
  sleep 150
done
