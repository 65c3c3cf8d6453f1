#!/bin/bash
# One rocprofv3 SQ counter pass over the default bench (its own time limit), summarised by
# scripts/sq_valu.py into $OUT/sq_valu.json (bench.py's roofline.valu when committed as
# profiles/sq_valu.json on the same build).
set -u
OUT=${OUT:-gpurun_out/sqv}
R=$(pwd)
mkdir -p "$OUT"
C="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv \
    -d "$R/$OUT/sq" -o run -- python3 "$R/bench.py" ${SQ_STEPS:---steps 20 --warmup 5} --no-cpu-baseline ${SQ_ARGS:-} ) \
    > "$OUT/sq.log" 2>&1
rc=$?; echo "[sq valu] rc=$rc"; case $rc in 0) ;; *) exit $rc ;; esac
DIRS="$OUT/sq"
# VALU instruction classes (SQ_CLASS=1): two more passes of the same command, <= 8 SQ counters each
if [ "${SQ_CLASS:-1}" = "1" ]; then
  P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
  P2="SQ_WAVES SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS"
  i=1
  for C in "$P1" "$P2"; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv \
        -d "$R/$OUT/sqc$i" -o run -- python3 "$R/bench.py" ${SQ_STEPS:---steps 20 --warmup 5} --no-cpu-baseline ${SQ_ARGS:-} ) \
        > "$OUT/sqc$i.log" 2>&1
    rc=$?; echo "[sq class pass $i] rc=$rc"; case $rc in 0) ;; *) exit $rc ;; esac
    DIRS="$DIRS $OUT/sqc$i"; i=$((i + 1))
  done
fi
python3 scripts/sq_valu.py $DIRS --box ${SQ_BOX:-4096x4096} --blocks ${SQ_BLOCKS:-1x1} > "$OUT/sq_valu.json" && cat "$OUT/sq_valu.json"
