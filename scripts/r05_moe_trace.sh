#!/bin/bash
# eager kernel trace of Mixtral's 20-token verification leg (grouped mmqs experts)
OUT=gpurun_out/${1:-r05mt}
mkdir -p $OUT
export TMPDIR=/tmp
SHORT_CFG=mixtral-8x7b-q5_k_m MI_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u scripts/short_leg.py 20 3 > $OUT/leg.log 2> $OUT/prof.err || { tail -3 $OUT/prof.err; exit 1; }
cat $OUT/leg.log
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
python3 - <<PY
import csv
rows=list(csv.DictReader(open('$OUT/kernel_stats.csv')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:18]:
    n=r['Name'].replace('mi::(anonymous namespace)::','').replace('mi::','')[:70]
    print(f"{n:70s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:8.2f} us {float(r['TotalDurationNs'])/tot*100:5.1f}%")
PY
exit 0
