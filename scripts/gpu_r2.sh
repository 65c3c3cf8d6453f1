#!/bin/bash
# Round-2 GPU job: selected parity tests (PYTEST_K), then optionally the full suite, smoke, bench,
# rocprof stats.  Every GPU step has its own time limit; a fault/abort/timeout ends the job.
set -u
OUT=${OUT:-gpurun_out/r02}
mkdir -p "$OUT"
R=$(pwd)
ok() { case $1 in 0|1|2|5) return 0 ;; *) echo "[$2] rc=$1 fault/abort/timeout -> stop"; exit $1 ;; esac; }
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf -x --timeout 120 --timeout-method thread -k "$PYTEST_K" > "$OUT/pytest_sel.log" 2>&1; rc=$?
  echo "[pytest sel] rc=$rc"; grep -E "PASS|FAIL|ERROR|Error|assert" "$OUT/pytest_sel.log" | tail -25; ok $rc pytest_sel
  [ $rc = 0 ] || exit $rc
fi
if [ "${TESTS:-0}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  echo "[pytest] rc=$rc"; tail -4 "$OUT/pytest_gpu.log"; grep -E "FAIL|ERROR" "$OUT/pytest_gpu.log" | head -20; ok $rc pytest
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?; echo "[smoke] rc=$rc"; tail -1 "$OUT/smoke.log"; ok $rc smoke
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1; rc=$?; echo "[bench] rc=$rc"; tail -1 "$OUT/bench.log"; ok $rc bench
fi
for extra in ${EXTRA_BENCH:-}; do
  timeout -k 10 400 python bench.py --no-cpu-baseline ${extra//,/ } > "$OUT/bench_${extra//[ ,=-]/_}.log" 2>&1; rc=$?; echo "[bench $extra] rc=$rc"; tail -1 "$OUT/bench_${extra//[ ,=-]/_}.log"; ok $rc bench_x
done
if [ "${PROF:-0}" = "1" ]; then
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/$OUT/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline ${PROF_ARGS:-} ) > "$OUT/prof.log" 2>&1
  rc=$?; echo "[rocprof] rc=$rc"; ok $rc rocprof
  f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f" | cut -c1-220
fi
exit 0
