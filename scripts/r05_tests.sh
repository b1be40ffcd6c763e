#!/bin/bash
# the whole GPU test suite (-s: the long full-depth tests print their progress), verbose log
OUT=gpurun_out/${1:-r05t}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc $rc"
grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -8
grep -E "live-floor waiver|distributions, score" $OUT/pytest_gpu.log | head -20
exit 0
