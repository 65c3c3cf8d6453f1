#!/bin/bash
# A/B of AB_VARS over the parity layouts' bench lines (2 rounds each); failures stop.
set -u
V=${AB_VARS:-"base ilp"}
for a in "c2:--n 1024" "c4:--blocks 4x2" "c5:--basin bs_tr --blocks 4x2" "c1:--basin bs" "general:--no-known-constants" "topo:--topography"; do
  n=${a%%:*}; args=${a#*:}
  OUT=gpurun_out/ab_cfg/$n AB_VARS="$V" AB_REPS=2 AB_ARGS="$args" bash scripts/gpu_ab3.sh | sed "s/^/$n /" || exit 1
done
