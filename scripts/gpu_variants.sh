#!/bin/bash
# Benchmark every library variant in build_variants/ (fused step, 4096^2, stage timing).
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
for lib in build_variants/libocn_sw_*.so; do
  name=$(basename "$lib" .so)
  OCN_LIB_PATH=$PWD/$lib timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${VARGS:-} > "$OUT/var_$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc"
  case $rc in 0|1|2) ;; *) echo "fault/timeout -> stop"; exit $rc ;; esac
  python3 -c "
import json,sys
d=json.loads(open('$OUT/var_$name.log').read().strip().splitlines()[-1])
print('  value %.3e  ms/step %.3f  ' % (d['value'], d['ms_per_step']), {k: round(v,3) for k,v in d['stage_ms'].items()})
" || tail -3 "$OUT/var_$name.log"
done
