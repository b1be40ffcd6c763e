#!/bin/bash
# kernel trace (rocprofv3 --kernel-trace --stats) of a short decode bench; stats -> $OUT/kernel_stats.csv
OUT=gpurun_out/${1:-r05d}
shift
mkdir -p $OUT
export TMPDIR=/tmp
MI_SEGV_MAPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 64 --warmup 8 "$@" > $OUT/bench.json 2> $OUT/prof.err || { grep -E "mi_segv|SIGSEGV" $OUT/prof.err | head -80; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
cut -d, -f1-4 $OUT/kernel_stats.csv | head -30
