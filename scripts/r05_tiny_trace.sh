#!/bin/bash
OUT=gpurun_out/${1:-r05tt}
mkdir -p $OUT
export TMPDIR=/tmp
MI_NO_GRAPH=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 32 --warmup 4 --config tinyllama-1.1b-q8_0 > $OUT/trace_bench.json 2> $OUT/prof.err || { tail -3 $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
python3 - <<PY
import csv
for r in list(csv.DictReader(open('$OUT/kernel_stats.csv')))[:16]:
    n=r['Name'].replace('mi::(anonymous namespace)::','').replace('mi::','')[:60]
    print(f"{n:60s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:7.2f} us")
PY
exit 0
