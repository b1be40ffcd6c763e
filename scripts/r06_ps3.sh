#!/bin/bash
OUT=gpurun_out/r06_ps3
mkdir -p $OUT
true
cat $OUT/diag.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/ps_stamps.py llama2-7b-q4_k_m 16 > $OUT/stamps.txt 2>&1; rc=$?
cat $OUT/stamps.txt; exit $rc
