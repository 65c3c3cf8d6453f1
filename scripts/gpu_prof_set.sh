#!/bin/bash
# Round-2 measurement job.
#   PROF_SET="name:bench args;name:bench args"  rocprofv3 --kernel-trace --stats of bench.py per
#                                              workload (bench JSON line -> $OUT/<name>.json)
#   PMC=1    FETCH_SIZE / WRITE_SIZE passes (separate, kernel-trace only) over stenbench (the read /
#            write calibration) and over the default bench, then scripts/pmc_traffic.py ->
#            $OUT/pmc_traffic.json stamped with this tree's ocn_build_id()
# Every GPU step has its own time limit; a fault / abort / timeout ends the job.
set -u
OUT=${OUT:-gpurun_out/r02b}
R=$(pwd)
mkdir -p "$OUT"
ok() { case $1 in 0) return 0 ;; *) echo "[$2] rc=$1 -> stop"; exit $1 ;; esac; }
IFS=';' read -ra SETS <<< "${PROF_SET:-}"
for s in "${SETS[@]}"; do
  [ -n "$s" ] || continue
  name=${s%%:*}; args=${s#*:}
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/$OUT/$name" -o run -- python3 "$R/bench.py" --no-cpu-baseline $args ) > "$OUT/$name.log" 2>&1
  rc=$?; echo "[$name] rc=$rc"; ok $rc "$name"
  grep '^{"metric"' "$OUT/$name.log" > "$OUT/$name.json"; cut -c1-400 "$OUT/$name.json"
  f=$(find "$OUT/$name" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$OUT/${name}_kernel_stats.csv"
done
if [ "${PMC:-0}" = "1" ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/stenbench scripts/stenbench.hip || exit 1
  for ctr in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
        -d "$R/$OUT/pmc_sten/$ctr" -o run -- /tmp/stenbench ) > "$OUT/pmc_sten_$ctr.log" 2>&1
    rc=$?; echo "[pmc stenbench $ctr] rc=$rc"; ok $rc pmc_sten
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
        -d "$R/$OUT/pmc/$ctr" -o run -- python3 "$R/bench.py" --steps 6 --warmup 1 --no-cpu-baseline ${PMC_ARGS:-} ) \
        > "$OUT/pmc_$ctr.log" 2>&1
    rc=$?; echo "[pmc bench $ctr] rc=$rc"; ok $rc pmc_bench
  done
  python3 scripts/pmc_traffic.py "$OUT/pmc" "$OUT/pmc_sten" $((4096 * 4096)) --box 4096x4096 --blocks 1x1 --compact \
      > "$OUT/pmc_traffic.json" && cat "$OUT/pmc_traffic.json"
fi
exit 0
