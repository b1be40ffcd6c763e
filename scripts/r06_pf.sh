#!/bin/bash
OUT=gpurun_out/r06_pf
mkdir -p $OUT
timeout -k 10 300 ./scripts/exp_fat 4 > $OUT/exp.txt 2>&1; rc=$?
cat $OUT/exp.txt | grep -v "^chain"
exit $rc
