#!/bin/bash
# One rocprofv3 FETCH_SIZE pass (counters only: no other trace domain) over a short decode-only
# bench run, then the per-launch HBM read bytes
# (x2 gfx950 correction, scripts/pmc_traffic.py) of each kernel of interest, written under $OUT
# (copy the ones to keep into profiles/).  Eager launches
# (MI_NO_GRAPH=1): the per-launch counters do not depend on graph replay.
# Usage: scripts/pmc_round.sh tag round
TAG=${1:-pmc}; RND=${2:-r05}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
MI_NO_GRAPH=1 timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 8 --warmup 2 > $OUT/pmc_bench.json 2> $OUT/pmc.err || { tail -5 $OUT/pmc.err; exit 1; }
CSV=$(find $OUT/prof -name '*counter_collection.csv' | head -1)
[ -n "$CSV" ] || { echo "no counter_collection.csv"; exit 1; }
cp $CSV $OUT/counter_collection.csv
python3 scripts/pmc_traffic.py $CSV "dgemv_kernel<12, -1, 2, 2, 2>" $OUT/${RND}_pmc_ffn.json
python3 scripts/pmc_traffic.py $CSV "dgemv_kernel<12, -1, 1, 2, 1>" $OUT/${RND}_pmc_wo.json
python3 scripts/pmc_traffic.py $CSV "dv_quant_kernel" $OUT/${RND}_pmc_dv_quant.json
python3 scripts/pmc_traffic.py $CSV "attn_dec_kernel<" $OUT/${RND}_pmc_attn_dec.json
python3 scripts/pmc_traffic.py $CSV "dgemv_kernel<14, -1, 1, 6, 1>" $OUT/${RND}_pmc_down_q6k.json
python3 scripts/pmc_traffic.py $CSV "dgemv_kernel<12, -1, 1, 6, 1>" $OUT/${RND}_pmc_down_q4k.json
true
