#!/bin/bash
# A/B of build_variants/$AB_B against build_variants/$AB_A (bench lines, scripts/gpu_ab.sh), then the
# pair / parity GPU tests on the B build (OCN_LIB_PATH).  Each GPU step has its own time limit.
set -u
OUT=${OUT:-gpurun_out/var}
mkdir -p "$OUT"
OUT=$OUT bash scripts/gpu_ab.sh || exit 1
[ -n "${AB_ARGS2:-}" ] && { OUT=$OUT/2 AB_ARGS="$AB_ARGS2" bash scripts/gpu_ab.sh || exit 1; }
OCN_LIB_PATH=$PWD/build_variants/$AB_B.so timeout -k 10 900 python -u -m pytest ${VAR_TESTS:-tests/test_gpu_pair.py} -x -q \
    --timeout 240 --timeout-method thread > "$OUT/tests.txt" 2>&1
rc=$?; tail -3 "$OUT/tests.txt"; [ $rc = 0 ] || { grep -m3 -B2 -A30 "Error\|assert" "$OUT/tests.txt" | head -60; exit $rc; }
exit 0
