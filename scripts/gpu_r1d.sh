#!/bin/bash
# parity tests + bench + stencil microbench + FETCH_SIZE calibration (8 B/lane loads)
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
R=$(pwd)
ok() { case $1 in 0|1|2|5) return 0 ;; *) echo "[$2] rc=$1 fault/abort/timeout -> stop"; exit $1 ;; esac; }
TESTS=1 BENCH=1 bash scripts/gpu_round.sh || exit $?
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/stenbench scripts/stenbench.hip || exit 1
timeout -k 10 120 /tmp/stenbench > "$OUT/stenbench.log" 2>&1; rc=$?; echo "[stenbench] rc=$rc"; cat "$OUT/stenbench.log"; ok $rc stenbench
for ctr in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
      -d "$R/$OUT/pmc_sten/$ctr" -o run -- /tmp/stenbench ) > "$OUT/pmc_sten_$ctr.log" 2>&1
  rc=$?; echo "[pmc sten $ctr] rc=$rc"; ok $rc pmcsten
done
python3 scripts/pmc_summary.py "$OUT/pmc_sten" > "$OUT/pmc_sten_summary.json" && cat "$OUT/pmc_sten_summary.json"
exit 0
