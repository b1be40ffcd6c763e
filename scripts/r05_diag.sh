#!/bin/bash
OUT=gpurun_out/${1:-r05d}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_ops.py -k "mmqs or mmq32" -v -s --timeout 200 --timeout-method thread > $OUT/ops.log 2>&1
rc1=$?; echo "ops rc $rc1"; grep -E "PASS|FAIL|Error" $OUT/ops.log | head -40
timeout -k 10 200 python -u scripts/diag_short.py llama2-7b-q4_k_m 20 > $OUT/diag.log 2>&1; rc=$?
tail -8 $OUT/diag.log
exit $rc
