#!/bin/bash
# Band width of the overlapped x2 / x4 steps: parity tests, then A/B of build_variants/base.so (x4 bands a
# pair tile wide, x2 bands 2 wide) against x2w.so (x2 bands a wave wide too) with x4 off, overlap 2.
set -u
mkdir -p gpurun_out/band
timeout -k 10 900 python -u -m pytest tests/test_gpu_x4.py tests/test_gpu_multirank.py tests/test_gpu_multi.py -x -q \
    --timeout 120 --timeout-method thread -k "x4 or random or tracer or ranks" > gpurun_out/band/t.txt 2>&1
rc=$?; tail -2 gpurun_out/band/t.txt; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/band AB_A=base AB_B=x2w AB_REPS=2 AB_ARGS="--blocks 4x2 --no-x4 --overlap 2" bash scripts/gpu_ab.sh || exit 1
OUT=gpurun_out/band2 AB_A=base AB_B=x2w AB_REPS=1 AB_ARGS="--blocks 2x1 --no-x4 --overlap 2" bash scripts/gpu_ab.sh
