#!/bin/bash
# r06: persistent decode step -- correctness against the launch form, then the rate
OUT=gpurun_out/r06_ps
mkdir -p $OUT
timeout -k 10 120 python -u scripts/ps_check.py tiny-q4_k_m tiny-q6_k tiny-q5_k_m > $OUT/tiny.txt 2>&1; rc=$?
cat $OUT/tiny.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u scripts/ps_check.py llama2-7b-q4_k_m > $OUT/7b.txt 2>&1; rc=$?
cat $OUT/7b.txt
exit $rc
