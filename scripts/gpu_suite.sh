#!/bin/bash
# The whole GPU suite in one process, one time limit, output under gpurun_out/suite.
set -u
mkdir -p gpurun_out/suite
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/suite/pytest.txt 2>&1
rc=$?
tail -3 gpurun_out/suite/pytest.txt
exit $rc
