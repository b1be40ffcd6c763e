#!/bin/bash
# the rocprofv3 graph-replay crash without the engine, then the decode trace with eager launches
OUT=gpurun_out/${1:-r05e}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/exp_rocprof_graph 200 200 > $OUT/plain.txt 2>&1; echo "plain rc $?"; cat $OUT/plain.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rp -o run -- ./scripts/exp_rocprof_graph 200 200 > $OUT/traced.txt 2> $OUT/traced.err
echo "traced rc $?"; cat $OUT/traced.txt; grep -E "SIGSEGV|PC:" $OUT/traced.err | head -5
rm -rf $OUT/rp
MI_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 64 --warmup 8 > $OUT/bench.json 2> $OUT/prof.err || { grep -E "SIGSEGV" $OUT/prof.err | head; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
cut -d, -f1-4 $OUT/kernel_stats.csv | head -30
