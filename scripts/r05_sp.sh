#!/bin/bash
# streaming decode path: decode parity tests, then an A/B bench against the gemv_kernel graph
OUT=gpurun_out/${1:-r05c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullwidth.py -k "decode or determin or topk or state or shift or extend or split or crosses" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAIL|Error|error" $OUT/pytest.log | head -20; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
for mode in new old new old; do
  unset MI_DECODE_OLD
  if [ $mode = old ]; then export MI_DECODE_OLD=1; fi
  timeout -k 10 200 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 128 --warmup 16 > $OUT/bench_$mode.json 2> $OUT/bench_$mode.err || { echo "bench $mode failed"; tail -5 $OUT/bench_$mode.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$mode.json'));print('$mode', d['value'], d['roofline']['avg_launch_us'])"
done
unset MI_DECODE_OLD
MI_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 64 --warmup 8 > $OUT/trace_bench.json 2> $OUT/prof.err || { grep SIGSEGV $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
python - <<PY
import csv
for r in list(csv.DictReader(open('$OUT/kernel_stats.csv')))[:16]:
    n=r['Name'].replace('mi::(anonymous namespace)::','')[:60]
    print(f"{n:60s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:7.2f} us")
PY
exit 0
