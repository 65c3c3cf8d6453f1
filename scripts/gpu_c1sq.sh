#!/bin/bash
# temporary: SQ counters of the Black Sea one-pass kernels, multi-step launch vs single launches
set -u
R=$(pwd)
mkdir -p gpurun_out/c1sq
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
for m in multi nomulti; do
  a=""; [ $m = nomulti ] && a="--no-multi"
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv \
      -d "$R/gpurun_out/c1sq/$m" -o run -- python3 "$R/bench.py" --basin bs --steps 20 --warmup 5 --no-cpu-baseline $a ) \
      > gpurun_out/c1sq/$m.log 2>&1
  rc=$?; echo "$m rc=$rc"; [ $rc = 0 ] || exit $rc
done
