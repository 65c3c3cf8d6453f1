#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, kernel-trace only; the
# MI355X_MICROARCH.md slot limits: <= 8 SQ, FETCH_SIZE and WRITE_SIZE in separate passes).
set -u
OUT=${OUT:-gpurun_out/pmc}
R=$(pwd)
mkdir -p "$OUT"
ARGS="--steps ${PMC_STEPS:-6} --warmup 1 --no-cpu-baseline ${PMC_ARGS:-}"
i=0
for grp in "${PMC_GROUPS[@]:-}"; do :; done
for grp in ${GROUPS_LIST:-"SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU" FETCH_SIZE WRITE_SIZE}; do
  i=$((i+1))
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --pmc ${grp//,/ } --kernel-trace --output-format csv \
      -d "$R/$OUT/p$i" -o run -- python3 "$R/bench.py" $ARGS ) > "$OUT/p$i.log" 2>&1
  rc=$?; echo "[pmc $grp] rc=$rc"
  case $rc in 0) ;; *) tail -5 "$OUT/p$i.log"; echo "stop"; exit $rc ;; esac
done
python3 scripts/pmc_kernels.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
