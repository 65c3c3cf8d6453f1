#!/bin/bash
# The gap between back-to-back launches with and without the stage-timing events: bench lines
# (default and the driver's command, each with and without --no-stage-timing) and a rocprofv3
# kernel trace of the default bench without the events.
set -u
OUT=${OUT:-gpurun_out/gap}
R=$(pwd)
mkdir -p "$OUT"
for v in "def:" "def_nt:--no-stage-timing" "drv:--steps 20 --warmup 5" "drv_nt:--steps 20 --warmup 5 --no-stage-timing"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 120 python3 bench.py --no-cpu-baseline $a > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "[$n] failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d.get('stage_ms'))" "$OUT/$n.json" "$n"
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/tr" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-stage-timing ) > "$OUT/tr.log" 2>&1 || { echo "[trace] failed"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, statistics, sys
f = glob.glob(sys.argv[1] + "/tr/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
g = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])
     if "MarchStep" in a["Kernel_Name"] and "MarchStep" in b["Kernel_Name"]]
print("gaps between one-pass launches without events: n", len(g), "median us", statistics.median(g))
PY
