#!/bin/bash
# rocprofv3 kernel-trace stats of the multi-block bench on one GPU (local halo copies).
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
R=$(pwd)
for b in ${BLOCKS:-2x2}; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/$OUT/prof_mb_$b" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --blocks $b ${MB_ARGS:-} ) \
      > "$OUT/prof_mb_$b.log" 2>&1
  rc=$?; echo "[rocprof $b] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
