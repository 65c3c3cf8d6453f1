#!/bin/bash
# tests + bench (compact, 2-D, stages) + rocprof stats + PMC traffic
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
ok() { case $1 in 0|1|2|5) return 0 ;; *) echo "[$2] rc=$1 fault/abort/timeout -> stop"; exit $1 ;; esac; }
make -s -f ocean_model_arch_amd/csrc/Makefile >/dev/null 2>&1
TESTS=1 BENCH=1 PROF=1 PMC=1 bash scripts/gpu_round.sh || exit $?
timeout -k 10 400 python bench.py --no-compact --no-cpu-baseline > "$OUT/bench_2d.log" 2>&1; rc=$?; echo "[bench 2d] rc=$rc"; tail -1 "$OUT/bench_2d.log"; ok $rc bench2d
timeout -k 10 400 python bench.py --graph --no-cpu-baseline > "$OUT/bench_graph.log" 2>&1; rc=$?; echo "[bench graph] rc=$rc"; tail -1 "$OUT/bench_graph.log"; ok $rc benchgraph
exit 0
