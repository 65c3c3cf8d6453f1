#!/bin/bash
# Instruction-cache counters of the pair launch: the available SQC counters, then one --pmc pass
# (4 counters) over the driver's command.  Each step has its own limit.
set -u
R=$(pwd); OUT=gpurun_out/ic; mkdir -p $OUT
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --list-avail ) > $OUT/avail.txt 2>&1
grep -i -E "ICACHE|IFETCH|SQC_INST" $OUT/avail.txt | cut -c1-200 | head -40
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES \
    --kernel-trace --output-format csv -d "$R/$OUT/pmc" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline ) \
    > $OUT/pmc.log 2>&1
rc=$?; echo "[pmc] rc=$rc"; tail -3 $OUT/pmc.log; exit $rc
