#!/bin/bash
# A/B of build_variants/{base,fbfast}.so: bench timings (100 steps x3, the driver's command x2) and one
# SQ_INSTS_VALU pass each over the driver's command.  Each GPU step has its own limit; failures stop.
set -u
R=$(pwd)
OUT=gpurun_out/ab_fb AB_VARS="base fbfast" AB_REPS=3 bash scripts/gpu_ab3.sh || exit 1
OUT=gpurun_out/ab_fb_drv AB_VARS="base fbfast" AB_REPS=2 AB_ARGS="--steps 20 --warmup 5" bash scripts/gpu_ab3.sh || exit 1
for v in base fbfast; do
  ( cd /tmp && export TMPDIR=/tmp && OCN_LIB_PATH=$R/build_variants/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES \
      --kernel-trace --output-format csv -d "$R/gpurun_out/ab_fb/pmc_$v" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 \
      --no-cpu-baseline ) > "gpurun_out/ab_fb/pmc_$v.log" 2>&1 || { echo "[pmc $v] failed"; exit 1; }
done
echo done
