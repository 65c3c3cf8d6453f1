#!/bin/bash
# bench.py with every build_variants/lib_*.so (OCN_LIB_PATH) and the in-tree library; prints
# ms/step and the per-launch means of each variant.
set -u
OUT=${OUT:-gpurun_out/var}
mkdir -p "$OUT"
for lib in ocean_model_arch_amd/libocn_sw.so $(ls build_variants/lib_*.so 2>/dev/null); do
  n=$(basename $lib .so)
  OCN_LIB_PATH=$(pwd)/$lib timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/$n.log" 2>&1; rc=$?
  echo "[$n] rc=$rc $(python3 -c "import json,sys; d=json.loads(open('$OUT/$n.log').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), d['stage_ms'])" 2>&1 | tail -1)"
  case $rc in 0) ;; *) echo stop; exit $rc ;; esac
done
