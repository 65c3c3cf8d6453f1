#!/bin/bash
# x4 pairs with OCN_OPT_OVERLAP 2 (inner pair beside the exchange, then the bands) against 1 (in sequence)
# on one GPU, after the overlapped x4 parity tests.  Each GPU step has its own time limit.
set -u
mkdir -p gpurun_out/ov
timeout -k 10 600 python -u -m pytest tests/test_gpu_x4.py tests/test_gpu_multirank.py -x -q --timeout 120 \
    --timeout-method thread -k "x4 or random" > gpurun_out/ov/t.txt 2>&1
rc=$?; tail -2 gpurun_out/ov/t.txt; [ $rc = 0 ] || exit $rc
for a in "--blocks 4x2 --overlap 1" "--blocks 4x2 --overlap 2" "--n 2048 --blocks 2x2 --overlap 1" "--n 2048 --blocks 2x2 --overlap 2" "--blocks 2x1 --overlap 1" "--blocks 2x1 --overlap 2"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline $a > gpurun_out/ov/run.log 2>&1 || { echo "fail $a"; tail -3 gpurun_out/ov/run.log; exit 1; }
  grep '^{' gpurun_out/ov/run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$a', round(d['ms_per_step'],4), c['kernel_launches_per_step'], d.get('stage_ms'))"
done
