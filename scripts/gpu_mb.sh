#!/bin/bash
# Multi-block benches on one GPU (local halo copies).  MB_VARIANTS: ';'-separated bench flag sets.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
IFS=';' read -r -a VARS <<< "${MB_VARIANTS:---blocks 2x2;--blocks 2x2 --no-flip;--blocks 2x1;--blocks 2x1 --no-flip}"
for v in "${VARS[@]}"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $v > "$OUT/bench_mb.log" 2>&1; rc=$?
  echo "[bench $v] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 "$OUT/bench_mb.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), d['config']['role_flip_steps'], d['config']['recompute_steps'], {k: round(v,4) for k,v in d['stage_ms'].items()})" || exit 1
done
