OUT=gpurun_out/r05i; mkdir -p $OUT; export TMPDIR=/tmp
MI_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 64 --warmup 8 > $OUT/trace_bench.json 2> $OUT/prof.err || { grep SIGSEGV $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
