#!/bin/bash
OUT=gpurun_out/${1:-r05md}
mkdir -p $OUT
MI_MMQS_MAX=0 MI_MMQ_KSPLIT=0 timeout -k 10 400 python -u scripts/diag_moe64.py > $OUT/dks0.log 2>&1; echo "rc $?"; tail -1 $OUT/dks0.log
MI_MMQS_MAX=32 timeout -k 10 400 python -u scripts/diag_moe64.py > $OUT/d32.log 2>&1; echo "rc $?"; tail -1 $OUT/d32.log
exit 0
