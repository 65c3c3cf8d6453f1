#!/bin/bash
# parity tests + smoke + bench + tile-mapping variants
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
TESTS=1 BENCH=1 VARIANTS=1 bash scripts/gpu_round.sh || exit $?
exit 0
