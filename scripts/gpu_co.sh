#!/bin/bash
# Co-launch check (OCN_OPT_CO_LAUNCH): the tracer-step GPU tests, the random sequences (in one process and
# over loopback ranks) and the tracer runs over ranks, then the C5 layout's bench line with and without
# the co-launch.  Every GPU step has its own time limit; a failure ends the job.
set -u
OUT=${OUT:-gpurun_out/co}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_pair.py tests/test_gpu_multirank.py -x -q \
    --timeout 120 --timeout-method thread -k "tracer or random" > "$OUT/t.txt" 2>&1
rc=$?; tail -3 "$OUT/t.txt"; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for a in "" "--no-co-launch"; do
    timeout -k 10 120 python bench.py --basin bs_tr --blocks 4x2 --no-cpu-baseline $a > "$OUT/c5_$i$a.log" 2>&1
    rc=$?; [ $rc = 0 ] || { echo "bench rc=$rc"; exit $rc; }
    grep '^{' "$OUT/c5_$i$a.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$a', d['ms_per_step'], c['kernel_launches_per_step'], c.get('co_launch'))"
  done
done
exit 0
