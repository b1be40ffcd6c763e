#!/bin/bash
# FETCH_SIZE of the short-batch kernels (one 20-token verification leg, scripts/short_leg.py) and
# an eager kernel trace of the same leg
TAG=${1:-r05sp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
MI_NO_GRAPH=1 timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof -o run -- python -u scripts/short_leg.py 20 2 > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
CSV=$(find $OUT/prof -name '*counter_collection.csv' | head -1)
[ -n "$CSV" ] || { echo "no counter_collection.csv"; exit 1; }
for k in "mmqs1_t<12, true>" "mmqs1_t<12, false>" "mmqs1_t<14, false>" "quant_act_kernel" "qkv_finish" "attn_fused_kernel<1, 16, 1>"; do
  f=$(echo "$k" | tr -c 'a-z0-9' '_')
  python3 scripts/pmc_traffic.py $CSV "$k" $OUT/r05_pmc_short_$f.json || true
done
rm -rf $OUT/prof
MI_NO_GRAPH=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python -u scripts/short_leg.py 20 3 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
find $OUT/tr -name '*kernel_stats.csv' -exec cp {} $OUT/short_kernel_stats.csv \;
rm -rf $OUT/tr
exit 0
