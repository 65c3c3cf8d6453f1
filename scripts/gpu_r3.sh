#!/bin/bash
# Round-3 GPU job (run through gpurun from the repo root): GPU tests, then bench lines.
# Every GPU step has its own time limit; a fault / abort / timeout ends the job.
#   OUT=gpurun_out/x  TESTS="tests -m gpu"  BENCHES="default;--steps-per-call 1"  PROF=0|1
set -u
OUT=${OUT:-gpurun_out/r3}
mkdir -p "$OUT"
stop_on_fault() {  # rc name
  local rc=$1
  echo "[$2] rc=$rc"
  case $rc in 0|1|2|5) return 0 ;; *) echo "[$2] fault/abort/timeout -> stop"; exit $rc ;; esac
}
if [ -n "${TESTS:-tests -m gpu}" ] && [ "${TESTS:-x}" != "none" ]; then
  timeout -k 10 ${T_TEST:-600} python -u -m pytest ${TESTS:-tests -m gpu} -q -rf --durations=30 --timeout 120 \
      --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  stop_on_fault $? pytest
  tail -4 "$OUT/pytest_gpu.log"
fi
i=0
IFS=';' read -ra BL <<< "${BENCHES:-default}"
for b in "${BL[@]}"; do
  i=$((i + 1))
  args=$b
  [ "$b" = "default" ] && args=""
  timeout -k 10 ${T_BENCH:-300} python bench.py --no-cpu-baseline $args > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
  stop_on_fault $? "bench $i ($b)"
  echo "bench $i ($b): $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_$i.json')); print(round(d['ms_per_step'],4), 'ms/step', round(d['value']/1e9,2), 'Gcu/s', d['roofline'] and d['roofline']['frac'], d['config'].get('kernel_launches_per_step'))" 2>&1)"
done
if [ "${PROF:-0}" = "1" ]; then
  R=$(pwd)
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/$OUT/prof" -o run -- python3 "$R/bench.py" --no-cpu-baseline ${PROF_ARGS:-} ) > "$OUT/prof.log" 2>&1
  stop_on_fault $? rocprof
  find "$OUT/prof" -name "*stats*" | head
fi
exit 0
