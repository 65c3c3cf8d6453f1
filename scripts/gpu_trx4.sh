#!/bin/bash
# x4 pairs with tracer steps: the x4 / tracer / random-sequence / rank tests, then the C5 layout's bench
# line (x4 on and off).  Each GPU step has its own time limit; the first failure ends the job.
set -u
mkdir -p gpurun_out/trx4
timeout -k 10 900 python -u -m pytest tests/test_gpu_x4.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/trx4/t1.txt 2>&1
rc=$?; tail -3 gpurun_out/trx4/t1.txt; [ $rc = 0 ] || { grep -m3 -B2 -A30 "Error\|assert" gpurun_out/trx4/t1.txt | head -60; exit $rc; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_pair.py tests/test_gpu_multirank.py -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/trx4/t2.txt 2>&1
rc=$?; tail -3 gpurun_out/trx4/t2.txt; [ $rc = 0 ] || { grep -m3 -B2 -A30 "Error\|assert" gpurun_out/trx4/t2.txt | head -60; exit $rc; }
for a in "" "--no-x4"; do
  timeout -k 10 120 python bench.py --basin bs_tr --blocks 4x2 --no-cpu-baseline $a > gpurun_out/trx4/c5.log 2>&1 || { tail -3 gpurun_out/trx4/c5.log; exit 1; }
  grep '^{' gpurun_out/trx4/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$a', round(d['ms_per_step'],4), c['kernel_launches_per_step'], c.get('x4_pairs'), c.get('co_launch'))"
done
exit 0
