#!/bin/bash
# SQ issue/wait breakdown of the short-batch kernels (mmqs1 / mmqs / quant_act / qkv_finish /
# fused attention) over the bench's prefill + verify_short legs; counters only, eager launches
TAG=${1:-r05sq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
K="mmqs1_t mmqs_t quant_act qkv_finish attn_fused dgemv_kernel dv_quant"
MI_NO_GRAPH=1 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    --output-format csv -d $OUT/p1 -o run -- python -u scripts/short_leg.py 20 2 > $OUT/p1.log 2>&1 || { echo "pass1 failed $?"; tail -5 $OUT/p1.log; exit 1; }
f=$(find $OUT/p1 -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_sq.py "$f" $K > $OUT/p1.txt && cat $OUT/p1.txt
MI_NO_GRAPH=1 timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_INSTS_SALU \
    --output-format csv -d $OUT/p2 -o run -- python -u scripts/short_leg.py 20 2 > $OUT/p2.log 2>&1 || { echo "pass2 failed $?"; tail -5 $OUT/p2.log; exit 1; }
f=$(find $OUT/p2 -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_sq.py "$f" $K > $OUT/p2.txt && cat $OUT/p2.txt
rm -rf $OUT/p1 $OUT/p2
exit 0
