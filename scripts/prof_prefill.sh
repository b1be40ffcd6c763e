#!/bin/bash
# rocprofv3 kernel stats of the bench's prefill leg (decode steps minimal, no CPU leg).
OUT=gpurun_out/${1:-pp}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --no-cpu --steps 2 --warmup 1 --prof-layer -1 > $OUT/bench.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
head -14 $OUT/kernel_stats.csv | cut -c1-160
