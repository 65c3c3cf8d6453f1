#!/bin/bash
# Experiment job: HBM ceilings of the fused launches' read/write mixes (mixbench), the library
# variants in build_variants/ (scripts/gpu_variants.sh) and the one-thread-per-point step.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
ok() { case $1 in 0|1|2|5) return 0 ;; *) echo "[$2] rc=$1 fault/abort/timeout -> stop"; exit $1 ;; esac; }
if [ "${MIX:-1}" = "1" ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/mixbench scripts/mixbench.hip || exit 1
  timeout -k 10 120 /tmp/mixbench > "$OUT/mixbench.log" 2>&1; rc=$?; echo "[mixbench] rc=$rc"; cat "$OUT/mixbench.log"; ok $rc mixbench
fi
if [ "${NOMARCH:-1}" = "1" ]; then
  timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-march > "$OUT/nomarch.log" 2>&1; rc=$?
  echo "[nomarch] rc=$rc"; tail -1 "$OUT/nomarch.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stage_ms'])"; ok $rc nomarch
fi
if [ "${VARIANTS:-1}" = "1" ]; then bash scripts/gpu_variants.sh || exit $?; fi
exit 0
