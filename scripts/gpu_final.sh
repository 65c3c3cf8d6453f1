#!/bin/bash
# Round-end measurement set: GPU tests, smoke, rocprofv3 --kernel-trace --stats of bench.py per
# workload, PMC traffic passes and SQ VALU class passes, all on this tree's build.  Each GPU step
# has its own time limit; the first failure ends the job.
set -u
OUT=${OUT:-gpurun_out/r05x}
mkdir -p "$OUT"
ok() { case $1 in 0) return 0 ;; *) echo "[$2] rc=$1 -> stop"; exit $1 ;; esac; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1
  rc=$?; tail -3 "$OUT/pytest_gpu.txt"; ok $rc pytest
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1
  rc=$?; tail -2 "$OUT/smoke.txt"; ok $rc smoke
fi
OUT=$OUT PROF_SET="${PROF_SET:-}" PMC=${PMC:-1} bash scripts/gpu_prof_set.sh; ok $? prof_set
if [ "${SQ:-1}" = "1" ]; then
  OUT=$OUT/sqv bash scripts/gpu_sq_valu.sh; ok $? sq_valu
fi
exit 0
