#!/bin/bash
# The driver's bench command's effective shader clock per launch: rocprofv3 --pmc GRBM_GUI_ACTIVE
# with the kernel trace (a counter pass of its own), then the steady state of the same command after
# a long warm-up (--warmup 60), both beside the plain command.  scripts/clock_trace.py renders them.
set -u
OUT=${OUT:-gpurun_out/r04b}
R=$(pwd)
mkdir -p "$OUT"
ok() { case $1 in 0) return 0 ;; *) echo "[$2] rc=$1 -> stop"; exit $1 ;; esac; }
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d "$R/$OUT/clock" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ) \
    > "$OUT/clock.log" 2>&1
ok $? clock
for f in $(find "$OUT/clock" -name "*counter_collection.csv" -o -name "*kernel_trace.csv"); do cp "$f" "$OUT/clock_$(basename $f)"; done
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 60 --no-cpu-baseline > "$OUT/warm60.json" 2> "$OUT/warm60.err"
ok $? warm60; cut -c1-200 "$OUT/warm60.json"
exit 0
