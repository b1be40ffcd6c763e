#!/bin/bash
# eager kernel trace of the decode bench (the decode kernels' durations); CFG=<config> for another model
OUT=gpurun_out/${1:-r06_trace}; mkdir -p $OUT; export TMPDIR=/tmp
MI_NO_GRAPH=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u bench.py ${CFG:+--config $CFG} --no-cpu --steps 48 --warmup 8 --prefill 0 > $OUT/trace_bench.json 2> $OUT/prof.err || { tail -3 $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
python3 - <<PY
import csv
for r in list(csv.DictReader(open('$OUT/kernel_stats.csv')))[:24]:
    n=r['Name'].replace('mi::(anonymous namespace)::','')[:70]
    print(f"{n:70s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:7.2f} us {float(r['Percentage']):5.1f}%")
PY
