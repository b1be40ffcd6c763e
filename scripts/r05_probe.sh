#!/bin/bash
# r05 probe: the decode-GEMV design experiment (exp_fgemv), then the r04 rocprofv3 crash
# (3968-token prompt, graph mode) with the engine's SIGSEGV mapping dump (MI_SEGV_MAPS=1).
OUT=gpurun_out/${1:-r05a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 ./scripts/exp_fgemv 3 > $OUT/exp_fgemv.txt 2>&1 || { echo "exp_fgemv rc $?"; tail -5 $OUT/exp_fgemv.txt; exit 1; }
cat $OUT/exp_fgemv.txt
MI_SEGV_MAPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 4 --warmup 1 --prompt 3968 --prof-layer -1 > $OUT/lc.json 2> $OUT/lc.err
rc=$?
echo "lc rc $rc"
grep -E "mi_segv|SIGSEGV" $OUT/lc.err | head -60
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/lc_kernel_stats.csv \; 2>/dev/null
rm -rf $OUT/prof
exit 0
