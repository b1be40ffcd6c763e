#!/bin/bash
# Kernel trace (eager launches) of one config's bench legs: a few decode steps, the 512-token
# prefill and the verify-256 leg.  Usage: scripts/prof_config.sh tag config
OUT=gpurun_out/${1:-pc}
CFG=${2:-mixtral-8x7b-q5_k_m}
mkdir -p $OUT
export TMPDIR=/tmp
export MI_NO_GRAPH=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --no-cpu --steps 4 --warmup 1 --config $CFG > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/prof -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
rm -rf $OUT/prof
head -25 $OUT/kernel_stats.csv | cut -c1-170
