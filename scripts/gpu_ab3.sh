#!/bin/bash
# A/B/C of library builds (build_variants/<v>.so via OCN_LIB_PATH): AB_VARS bench lines per round,
# AB_REPS rounds, AB_ARGS for bench.py.  Each run has its own time limit; a failure ends the job.
set -u
OUT=${OUT:-gpurun_out/ab3}
mkdir -p "$OUT"
for r in $(seq 1 ${AB_REPS:-2}); do
  for v in ${AB_VARS:-base}; do
    OCN_LIB_PATH=$PWD/build_variants/$v.so timeout -k 10 120 python3 bench.py --no-cpu-baseline ${AB_ARGS:-} \
        > "$OUT/${v}_$r.json" 2> "$OUT/${v}_$r.err" || { echo "[$v $r] failed"; tail -3 "$OUT/${v}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],5), d.get('stage_ms'))" \
        "$OUT/${v}_$r.json" "$v#$r"
  done
done
