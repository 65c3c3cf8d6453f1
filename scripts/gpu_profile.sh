#!/bin/bash
# Profile job for the committed evidence under profiles/: rocprofv3 kernel-trace stats of the
# default bench, the PMC HBM-traffic passes (FETCH_SIZE, WRITE_SIZE; separate runs) over the
# same bench, the stencil-microbenchmark FETCH_SIZE calibration, and SQ/TCC counter passes.
set -u
OUT=${OUT:-gpurun_out}
ok() { case $1 in 0|1|2|5) return 0 ;; *) echo "[$2] rc=$1 fault/abort/timeout -> stop"; exit $1 ;; esac; }
OUT=$OUT TESTS=0 BENCH=1 PROF=1 BENCH_ARGS="${BENCH_ARGS:-}" bash scripts/gpu_round.sh || exit $?
OUT=$OUT PMC_ARGS="--steps 20 --warmup 5" bash scripts/pmc.sh || exit $?
OUT=$OUT STEN=1 LIST=0 bash scripts/gpu_diag.sh || exit $?
exit 0
