#!/bin/bash
# Round-2 (late) measurement job: GPU parity + smoke + the plain bench line, then rocprofv3 kernel
# stats + bench lines per workload (scripts/gpu_prof_set.sh) and the PMC traffic stamp.
set -u
OUT=${OUT:-gpurun_out/r02q}
mkdir -p "$OUT"
ok() { case $1 in 0) return 0 ;; *) echo "[$2] rc=$1 -> stop"; exit $1 ;; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1
rc=$?; echo "[pytest] rc=$rc"; tail -1 "$OUT/pytest_gpu.txt"; ok $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
rc=$?; echo "[smoke] rc=$rc"; tail -1 "$OUT/smoke.txt"; ok $rc smoke
timeout -k 10 400 python bench.py > "$OUT/bench_default.log" 2>&1
rc=$?; echo "[bench] rc=$rc"; ok $rc bench
grep '^{"metric"' "$OUT/bench_default.log" > "$OUT/bench_default.json"; cut -c1-300 "$OUT/bench_default.json"
OUT=$OUT PROF_SET="main:;main_noonepass:--no-onepass;main_general:--no-known-constants;c1:--basin bs;c1_graph:--basin bs --graph;c2:--n 1024;c2_graph:--n 1024 --graph;c3_1gpu:--n 2048 --blocks 2x2;c4_1gpu:--blocks 4x2;c5_1gpu:--basin bs_tr --blocks 4x2" \
  PMC=${PMC:-1} bash scripts/gpu_prof_set.sh
