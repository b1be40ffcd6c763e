#!/bin/bash
# r06: eager kernel trace of the 512-token 7B prefill alone (scripts/prefill_only.py, 3 runs),
# for the per-kernel prefill breakdown.
OUT=gpurun_out/${1:-r06_prefill}; mkdir -p $OUT; export TMPDIR=/tmp
MI_NO_GRAPH=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u scripts/prefill_only.py > $OUT/trace_bench.json 2> $OUT/prof.err || { tail -3 $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
python3 - <<PY
import csv
for r in list(csv.DictReader(open('$OUT/kernel_stats.csv')))[:24]:
    n=r['Name'].replace('mi::(anonymous namespace)::','').replace('mi::mmq::','')[:70]
    print(f"{n:70s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:8.2f} us {float(r['TotalDurationNs'])/1e6:7.2f} ms")
PY
