#!/bin/bash
# SQ instruction-mix counters of the default bench (one rocprofv3 --pmc pass per group, each under
# its own time limit); scripts/sq_mix.py summarises the dominant kernel per wave and per row.
set -u
OUT=${OUT:-gpurun_out/sq}
mkdir -p "$OUT"
R=$(pwd)
ok() { case $1 in 0) return 0 ;; *) echo "[$2] rc=$1 -> stop"; exit $1 ;; esac; }
G1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64"
G2="SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
G3="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
G4="SQ_IFETCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_IFETCH_LEVEL"
i=0
for g in "$G1" "$G2" "$G3" ${SQ_EXTRA:+"$G4"}; do
  i=$((i + 1))
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $g --kernel-trace --output-format csv \
      -d "$R/$OUT/g$i" -o run -- python3 "$R/bench.py" --steps 6 --warmup 1 --no-cpu-baseline ${SQ_ARGS:-} ) \
      > "$OUT/g$i.log" 2>&1
  rc=$?; echo "[sq g$i] rc=$rc"; ok $rc sq
done
python3 scripts/sq_mix.py "$OUT" | tee "$OUT/sq_mix.txt"
