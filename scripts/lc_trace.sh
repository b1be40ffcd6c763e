#!/bin/bash
# Kernel trace of a 3968-token prompt (eight 512-token batches through mmq2 / attn_mfma) and 4
# decode steps at 3968 cells (--prof-layer -1: the bench context takes the batch path).  Eager launches (MI_NO_GRAPH=1): rocprofv3's kernel tracer faults
# inside hipGraphLaunch on this image for this run.  Usage: scripts/lc_trace.sh tag [config]
OUT=gpurun_out/${1:-lct}
CFG=${2:-llama2-7b-q4_k_m}
mkdir -p $OUT
export TMPDIR=/tmp
export MI_NO_GRAPH=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 4 --warmup 1 --prompt 3968 --prof-layer -1 --config $CFG > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/prof -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
rm -rf $OUT/prof
grep -E "attn_mfma|mmq2|attn_long" $OUT/kernel_stats.csv | cut -c1-160
