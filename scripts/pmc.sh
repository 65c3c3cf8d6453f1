#!/bin/bash
# HBM traffic per kernel from PMC counters: two separate rocprofv3 passes (FETCH_SIZE,
# WRITE_SIZE) with kernel-trace only (MI355X_MICROARCH.md: TCC FETCH_SIZE costs 3 slots,
# WRITE_SIZE 2 -- they cannot share a pass).  Then scripts/pmc_summary.py.
set -u
OUT=${OUT:-gpurun_out}
R=$(pwd)
mkdir -p "$OUT/pmc"
for ctr in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
      -d "$R/$OUT/pmc/$ctr" -o run -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline ${PMC_ARGS:-} ) \
      > "$OUT/pmc/$ctr.log" 2>&1
  rc=$?; echo "[pmc $ctr] rc=$rc"
  case $rc in 0) ;; *) echo "stop"; exit $rc ;; esac
done
python3 scripts/pmc_summary.py "$OUT/pmc" > "$OUT/pmc/summary.json" && cat "$OUT/pmc/summary.json"
