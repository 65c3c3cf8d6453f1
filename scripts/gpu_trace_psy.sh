#!/bin/bash
# HIP API trace of a PSy-style loop (scripts/psy_loop.py: ocn_ctx_step(1) + 3 x ocn_ctx_sync per time
# step, one block) and the synchronising calls inside it (scripts/psy_trace_summary.py).
#   OUT=gpurun_out/x  N=50  BOX=1024
set -u
OUT=${OUT:-gpurun_out/psy}
R=$(pwd)
mkdir -p "$OUT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --hip-trace --output-format csv \
    -d "$R/$OUT/trace" -o psy -- python3 "$R/scripts/psy_loop.py" ${N:-50} ${BOX:-1024} ) > "$OUT/psy.log" 2>&1
rc=$?; echo "[psy trace] rc=$rc"; case $rc in 0) ;; *) exit $rc ;; esac
grep -v "^LOOP" "$OUT/psy.log" | tail -2
python3 scripts/psy_trace_summary.py "$OUT/trace" "$OUT/psy.log" ${N:-50} > "$OUT/psy_summary.json"
head -30 "$OUT/psy_summary.json"
exit 0
