#!/bin/bash
# Diagnostics job: stencil microbenchmark + FETCH/WRITE calibration on it, counter list,
# and SQ / TCC counter passes over the bench (one rocprofv3 pass per counter group).
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT/diag"
R=$(pwd)
ok() { case $1 in 0|1|2|5) return 0 ;; *) echo "[$2] rc=$1 fault/abort/timeout -> stop"; exit $1 ;; esac; }
if [ "${STEN:-1}" = "1" ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/stenbench scripts/stenbench.hip || exit 1
  timeout -k 10 120 /tmp/stenbench > "$OUT/diag/stenbench.log" 2>&1; rc=$?; echo "[stenbench] rc=$rc"; cat "$OUT/diag/stenbench.log"; ok $rc stenbench
  for ctr in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
        -d "$R/$OUT/diag/pmc_sten/$ctr" -o run -- /tmp/stenbench ) > "$OUT/diag/pmc_sten_$ctr.log" 2>&1
    rc=$?; echo "[pmc sten $ctr] rc=$rc"; ok $rc pmcsten
  done
  python3 scripts/pmc_summary.py "$OUT/diag/pmc_sten" > "$OUT/diag/pmc_sten_summary.json"
fi
if [ "${LIST:-1}" = "1" ]; then
  ( cd /tmp && timeout -s KILL 60 rocprofv3 -L ) > "$OUT/diag/counters.txt" 2>&1; echo "[list] rc=$?"
fi
run_pass() {  # name counters...
  local name=$1; shift
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
      -d "$R/$OUT/diag/$name" -o run -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline ) \
      > "$OUT/diag/$name.log" 2>&1
  local rc=$?; echo "[pmc $name] rc=$rc"; ok $rc "pmc $name"
}
run_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run_pass tcc TCC_HIT_sum TCC_MISS_sum
python3 scripts/pmc_summary.py "$OUT/diag/sq" > "$OUT/diag/sq_summary.json"
python3 scripts/pmc_summary.py "$OUT/diag/tcc" > "$OUT/diag/tcc_summary.json"
exit 0
