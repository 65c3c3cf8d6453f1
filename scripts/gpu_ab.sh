#!/bin/bash
# A/B of library builds on one box: bench lines alternating between build_variants/<a>.so and <b>.so
# (OCN_LIB_PATH), AB_ARGS for bench.py, AB_REPS rounds.
set -u
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
A=${AB_A:-base}; B=${AB_B:-sea}
for r in $(seq 1 ${AB_REPS:-2}); do
  for v in $A $B; do
    OCN_LIB_PATH=$PWD/build_variants/$v.so timeout -k 10 120 python3 bench.py --no-cpu-baseline ${AB_ARGS:-} \
        > "$OUT/${v}_$r.json" 2> "$OUT/${v}_$r.err" || { echo "[$v $r] failed"; tail -3 "$OUT/${v}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d.get('stage_ms'))" \
        "$OUT/${v}_$r.json" "$v#$r"
  done
done
