#!/bin/bash
# Halo segments (merged column strips, chunk tables): the exchange tests, then rocprof stats of the
# multi-block bench lines.
set -u
mkdir -p gpurun_out/seg
timeout -k 10 900 python -u -m pytest tests/test_gpu_x4.py tests/test_gpu_multirank.py tests/test_gpu_multi.py tests/test_gpu_pair.py -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/seg/t.txt 2>&1
rc=$?; tail -2 gpurun_out/seg/t.txt; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/seg3 PROF_SET="c4:--blocks 4x2;c3:--n 2048 --blocks 2x2;c4o:--blocks 4x2 --overlap 2;c5:--basin bs_tr --blocks 4x2" PMC=0 bash scripts/gpu_prof_set.sh
