#!/bin/bash
# round-5 evidence: the default bench line, an eager kernel trace of the bench (decode, prefill,
# verify legs), a FETCH_SIZE pass of the decode kernels; every GPU step bounded, the first failure ends it
OUT=gpurun_out/${1:-r05f}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));p=d['prefill'];print('decode',d['value'],d['roofline'],'prefill',p['ms'],'verify',p['verify']['ms'],'short',p.get('verify_short'),'cpu',d['cpu_baseline']['value'],d.get('logit_comparer_vs_cpu'))"
MI_NO_GRAPH=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u bench.py --no-cpu --steps 64 --warmup 8 > $OUT/trace_bench.json 2> $OUT/prof.err || { tail -3 $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/prof -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
rm -rf $OUT/prof
timeout -k 10 200 bash scripts/pmc_round.sh ${1:-r05f}_pmc r05 || exit 1
exit 0
