#!/bin/bash
# Shader clock per launch (build_variants/probe.so, built with EXTRA=-DOCN_CLOCK_PROBE=1: workgroup 0
# of every march launch prints s_memtime ticks over 100 MHz s_memrealtime ticks of its tile) for the
# driver's command and the default bench run.
set -u
OUT=${OUT:-gpurun_out/clock}
mkdir -p "$OUT"
for a in "drv:--steps 20 --warmup 5" "default:"; do
  n=${a%%:*}; args=${a#*:}
  OCN_LIB_PATH=$PWD/build_variants/probe.so timeout -k 10 120 python3 bench.py --no-cpu-baseline $args \
      > "$OUT/$n.txt" 2> "$OUT/$n.err" || { echo "[$n] failed"; tail -3 "$OUT/$n.err"; exit 1; }
  grep -c clockprobe "$OUT/$n.txt"
done
