#!/bin/bash
# x4 pairs over ranks at full size and with tracer steps: the x4 tests, then the tracer / multi /
# pair / rank suites, then the C5 layout's bench line (x4 on and off).  Each GPU step has its own
# time limit; the first failure ends the job.
set -u
OUT=${OUT:-gpurun_out/trx4}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_x4.py -x -v --timeout 240 --timeout-method thread \
    > "$OUT/t1.txt" 2>&1
rc=$?; tail -3 "$OUT/t1.txt"; [ $rc = 0 ] || { grep -m3 -B2 -A30 "Error\|assert" "$OUT/t1.txt" | head -80; exit $rc; }
[ "${ONLY_X4:-0}" = "1" ] && exit 0
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_pair.py tests/test_gpu_multirank.py -x -q \
    --timeout 120 --timeout-method thread > "$OUT/t2.txt" 2>&1
rc=$?; tail -3 "$OUT/t2.txt"; [ $rc = 0 ] || { grep -m3 -B2 -A30 "Error\|assert" "$OUT/t2.txt" | head -80; exit $rc; }
for a in "" "--no-x4"; do
  timeout -k 10 120 python bench.py --basin bs_tr --blocks 4x2 --no-cpu-baseline $a > "$OUT/c5$a.log" 2>&1 || { tail -3 "$OUT/c5$a.log"; exit 1; }
  grep '^{' "$OUT/c5$a.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$a', round(d['ms_per_step'],4), c['kernel_launches_per_step'], c.get('x4_pairs'), c.get('co_launch'))"
done
exit 0
