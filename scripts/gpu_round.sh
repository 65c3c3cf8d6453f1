#!/bin/bash
# One GPU job: parity tests + smoke + bench (+ optional variants / membench / rocprof / pmc).
# Every GPU step has its own time limit; a fault/abort/timeout ends the job.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
ok() { case $1 in 0|1|2|5) return 0 ;; *) echo "[$2] rc=$1 fault/abort/timeout -> stop"; exit $1 ;; esac; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?; echo "[pytest] rc=$rc"; tail -4 "$OUT/pytest_gpu.log"; ok $rc pytest
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?; echo "[smoke] rc=$rc"; tail -1 "$OUT/smoke.log"; ok $rc smoke
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1; rc=$?; echo "[bench] rc=$rc"; tail -1 "$OUT/bench.log"; ok $rc bench
fi
if [ "${VARIANTS:-0}" = "1" ]; then bash scripts/gpu_variants.sh || exit $?; fi
if [ "${MEMBENCH:-0}" = "1" ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/membench scripts/membench.hip && \
  timeout -k 10 300 /tmp/membench > "$OUT/membench.log" 2>&1; rc=$?; echo "[membench] rc=$rc"; cat "$OUT/membench.log"; ok $rc membench
fi
if [ "${PROF:-0}" = "1" ]; then
  R=$(pwd)
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/$OUT/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline ) > "$OUT/prof.log" 2>&1
  rc=$?; echo "[rocprof] rc=$rc"; ok $rc rocprof
fi
if [ "${PMC:-0}" = "1" ]; then bash scripts/pmc.sh || exit $?; fi
if [ "${MB:-0}" = "1" ]; then bash scripts/gpu_mb.sh || exit $?; fi
exit 0
