#!/bin/bash
# The driver's command with and without the per-launch HIP events (stage timing) in the timed region.
set -u
OUT=${OUT:-gpurun_out/tab}
mkdir -p "$OUT"
for r in 1 2 3; do
  for v in on off; do
    a=""; [ $v = off ] && a="--no-stage-timing"
    timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 $a > "$OUT/${v}_$r.json" 2> "$OUT/${v}_$r.err" || { tail -3 "$OUT/${v}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],5))" "$OUT/${v}_$r.json" "$v#$r"
  done
done
