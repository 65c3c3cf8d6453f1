#!/bin/bash
# A/B timing on one box: bench.py alternating between the in-tree library and each
# build_variants/lib_*.so (or the libraries VARIANTS names), ROUNDS times; prints ms/step and the one-pass launch mean per run.
set -u
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in ocean_model_arch_amd/libocn_sw.so $(ls ${VARIANTS:-build_variants/lib_*.so} 2>/dev/null); do
    n=$(basename $lib .so)
    OCN_LIB_PATH=$(pwd)/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-40} ${BENCH_ARGS:-} \
      > "$OUT/${n}_$r.log" 2>&1; rc=$?
    echo "[$n r$r] rc=$rc $(python3 -c "import json; d=json.loads(open('$OUT/${n}_$r.log').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), d['stage_ms'])" 2>&1 | tail -1)"
    case $rc in 0) ;; *) echo stop; exit $rc ;; esac
  done
done
