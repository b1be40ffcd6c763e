#!/bin/bash
# Two SQ counter passes (8 SQ counters each, no tracing) over a short bench run.
TAG=${1:-sq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    --output-format csv -d $OUT/p1 -o run -- python -u bench.py --no-cpu --steps 8 --warmup 2 > $OUT/p1.log 2>&1 || { echo "pass1 failed $?"; tail -20 $OUT/p1.log; exit 1; }
f=$(find $OUT/p1 -name '*counter_collection.csv' | head -1)
python scripts/pmc_sq.py "$f" gemv_kernel attn_fused > $OUT/p1.txt && cat $OUT/p1.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES \
    --output-format csv -d $OUT/p2 -o run -- python -u bench.py --no-cpu --steps 8 --warmup 2 > $OUT/p2.log 2>&1 || { echo "pass2 failed $?"; tail -20 $OUT/p2.log; exit 1; }
f=$(find $OUT/p2 -name '*counter_collection.csv' | head -1)
python scripts/pmc_sq.py "$f" gemv_kernel attn_fused > $OUT/p2.txt && cat $OUT/p2.txt
rm -rf $OUT/p1 $OUT/p2
