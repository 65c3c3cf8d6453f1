#!/bin/bash
# Multi-block benches on one GPU (local halo copies): role-flip vs standard steps.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
for v in "--blocks 2x2" "--blocks 2x2 --no-flip" "--blocks 2x1" "--blocks 2x1 --no-flip"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $v > "$OUT/bench_mb.log" 2>&1; rc=$?
  echo "[bench $v] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 "$OUT/bench_mb.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), d['config']['role_flip_steps'], d['config']['recompute_steps'], d['stage_ms'])" || exit 1
done
