#!/bin/bash
# FETCH_SIZE of Mixtral's grouped short-batch expert launches (one 20-token verification leg) and
# an eager kernel trace of the same leg
TAG=${1:-r05mp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SHORT_CFG=mixtral-8x7b-q5_k_m MI_NO_GRAPH=1 timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof -o run -- python -u scripts/short_leg.py 20 2 > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
CSV=$(find $OUT/prof -name '*counter_collection.csv' | head -1)
[ -n "$CSV" ] || { echo "no counter_collection.csv"; exit 1; }
for k in "mmqs1_lean_t<13, true, true>" "mmqs1_lean_t<13, false, true>" "mmqs1_t<14, false, true>"; do
  f=$(echo "$k" | tr -c 'a-z0-9' '_')
  python3 scripts/pmc_traffic.py $CSV "$k" $OUT/r05_pmc_moe_$f.json mixtral-8x7b-q5_k_m || true
done
rm -rf $OUT/prof
SHORT_CFG=mixtral-8x7b-q5_k_m MI_NO_GRAPH=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python -u scripts/short_leg.py 20 3 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
find $OUT/tr -name '*kernel_stats.csv' -exec cp {} $OUT/moe_short_kernel_stats.csv \;
rm -rf $OUT/tr
exit 0
