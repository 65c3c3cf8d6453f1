#!/bin/bash
# A/B of the two-step launch's tile height (OCN_PAIR_ROWS, a fixed height instead of the cost
# model's) on the bench workload; each run under its own time limit, a failure ends the job.
set -u
OUT=${OUT:-gpurun_out/prows}
mkdir -p "$OUT"
for r in ${ROWS_LIST:-0 74 148 100 56 37}; do
  for k in 1 2; do
    if [ "$r" = "0" ]; then unset OCN_PAIR_ROWS; else export OCN_PAIR_ROWS=$r; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/rows_${r}_$k.log" 2>&1; rc=$?
    echo "[rows $r #$k] rc=$rc $(python3 -c "import json; d=json.loads(open('$OUT/rows_${r}_$k.log').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), d['stage_ms'])" 2>&1 | tail -1)"
    case $rc in 0) ;; *) exit $rc ;; esac
  done
done
