#!/bin/bash
# Pair tile height sweep (OCN_PAIR_ROWS) for small blocks + the VALU issue-cost microbenchmark.
# Prints per run: workload, rows, ms/step, pair launch ms (stage_ms.onepass2).
set -u
OUT=${OUT:-gpurun_out/rows}
mkdir -p "$OUT"
timeout -k 10 120 ./scripts/issuebench > "$OUT/issuebench.txt" 2>&1 || { tail -5 "$OUT/issuebench.txt"; exit 1; }
cat "$OUT/issuebench.txt"
show() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', round(d['ms_per_step'],5), d['stage_ms'].get('onepass2'), d['stage_ms'].get('onepass2_last'))"; }
for wl in "--n 1024" "--box 1024x2048"; do
  for r in 0 8 12 16 24 32 40 48 64; do
    tag="$(echo $wl | tr -d ' -')_r$r"
    if [ $r = 0 ]; then
      timeout -k 10 120 python bench.py $wl --no-cpu-baseline --steps 100 > "$OUT/$tag.log" 2>&1 || { tail -3 "$OUT/$tag.log"; exit 1; }
    else
      OCN_PAIR_ROWS=$r timeout -k 10 120 python bench.py $wl --no-cpu-baseline --steps 100 > "$OUT/$tag.log" 2>&1 || { tail -3 "$OUT/$tag.log"; exit 1; }
    fi
    show "$OUT/$tag.log" "$tag"
  done
done
exit 0
