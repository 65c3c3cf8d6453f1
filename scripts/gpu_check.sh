#!/bin/bash
# GPU validation + measurement job (run through gpurun from the repo root).
# Every GPU step has its own time limit; a fault/abort/timeout ends the job.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
stop_on_fault() {  # rc name
  local rc=$1
  echo "[$2] rc=$rc"
  case $rc in 0|1|2|5) return 0 ;; *) echo "[$2] fault/abort/timeout -> stop"; exit $rc ;; esac
}
timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
stop_on_fault $? pytest
tail -5 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
stop_on_fault $? smoke
tail -2 "$OUT/smoke.log"
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
stop_on_fault $? bench
tail -1 "$OUT/bench.log"
if [ "${PROF:-1}" = "1" ]; then
  R=$(pwd)
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/$OUT/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline ) > "$OUT/prof.log" 2>&1
  stop_on_fault $? rocprof
  find "$OUT/prof" -name "*stats*" | head
fi
