#!/bin/bash
OUT=gpurun_out/r06_ps2
mkdir -p $OUT
timeout -k 10 120 python -u scripts/ps_stamps.py llama2-7b-q4_k_m 16 > $OUT/stamps.txt 2>&1 || { cat $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
for pr in 2 20; do
timeout -k 10 240 python -u scripts/ps_check.py llama2-7b-q4_k_m --prompt=$pr --obs=24 --steps=30 >> $OUT/7b.txt 2>&1 || { cat $OUT/7b.txt; exit 1; }
done
timeout -k 10 240 python -u scripts/ps_check.py tiny-q4_k_m --prompt=2 --obs=40 --steps=40 >> $OUT/7b.txt 2>&1
cat $OUT/7b.txt
