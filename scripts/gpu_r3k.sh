#!/bin/bash
# The single-rank RCCL test first (its own time limit; a hang or fault ends the job), then
# scripts/gpu_r3.sh with the caller's OUT / BENCHES.
set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k rccl -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/rccl.log 2>&1
rc=$?; tail -5 gpurun_out/rccl.log; echo "[rccl] rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
bash scripts/gpu_r3.sh
