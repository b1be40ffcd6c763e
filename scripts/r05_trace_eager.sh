#!/bin/bash
# decode parity subset, the default bench (verify_short legs), an eager kernel trace of the
# streaming decode path and a FETCH_SIZE pass; every GPU step bounded, the first failure ends it
OUT=gpurun_out/r05i; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullwidth.py -k "decode or determin or topk or state or shift or extend or split or crosses" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -10; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 10 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));p=d['prefill'];print('decode',d['value'],d['roofline']['avg_launch_us'],'prefill',p['ms'],'verify',p['verify']['ms'],'short',p.get('verify_short'))"
MI_NO_GRAPH=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u bench.py --no-cpu --steps 64 --warmup 8 > $OUT/trace_bench.json 2> $OUT/prof.err || { grep SIGSEGV $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/prof -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
rm -rf $OUT/prof
python3 - <<PY
import csv
for r in list(csv.DictReader(open('$OUT/kernel_stats.csv')))[:20]:
    n=r['Name'].replace('mi::(anonymous namespace)::','')[:64]
    print(f"{n:64s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:7.2f} us")
PY
timeout -k 10 190 bash scripts/pmc_round.sh r05pmc r05 || exit 1
exit 0
