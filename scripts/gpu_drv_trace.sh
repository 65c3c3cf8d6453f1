#!/bin/bash
# The driver's exact bench command (--steps 20 --warmup 5), plain and under rocprofv3 --kernel-trace
# --stats (per-launch durations in the trace CSV: which launches of the timed region are slow), plus
# the default 100-step run for comparison.  Every GPU step has its own time limit; a failure ends the job.
set -u
OUT=${OUT:-gpurun_out/r04a}
R=$(pwd)
mkdir -p "$OUT"
ok() { case $1 in 0) return 0 ;; *) echo "[$2] rc=$1 -> stop"; exit $1 ;; esac; }
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/drv$i.json" 2> "$OUT/drv$i.err"
  ok $? drv$i; cut -c1-220 "$OUT/drv$i.json"
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$OUT/drv_prof" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ${DRV_ARGS:-} ) \
    > "$OUT/drv_prof.log" 2>&1
ok $? drv_prof
grep '^{"metric"' "$OUT/drv_prof.log" | cut -c1-220
for f in $(find "$OUT/drv_prof" -name "*kernel_trace.csv" -o -name "*kernel_stats.csv"); do cp "$f" "$OUT/drv_$(basename $f)"; done
timeout -k 10 240 python3 bench.py --gpus 1 --no-cpu-baseline > "$OUT/default.json" 2> "$OUT/default.err"
ok $? default; cut -c1-220 "$OUT/default.json"
exit 0
