#!/bin/bash
# r05 probe: the decode-GEMV design experiment (exp_fgemv), the streaming decode path's decode
# tests and an A/B bench against the gemv_kernel graph (MI_DECODE_OLD=1), then the r04 rocprofv3
# crash (3968-token prompt, graph mode) with the engine's SIGSEGV mapping dump (MI_SEGV_MAPS=1).
OUT=gpurun_out/${1:-r05a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 ./scripts/exp_fgemv 3 > $OUT/exp_fgemv.txt 2>&1 || { echo "exp_fgemv rc $?"; tail -5 $OUT/exp_fgemv.txt; exit 1; }
cat $OUT/exp_fgemv.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullwidth.py -k "decode or determin or topk or state or shift or extend or split or crosses" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -5 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
for mode in new old; do
  if [ $mode = old ]; then export MI_DECODE_OLD=1; fi
  timeout -k 10 200 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 128 --warmup 16 > $OUT/bench_$mode.json 2> $OUT/bench_$mode.err || { echo "bench $mode failed"; tail -5 $OUT/bench_$mode.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$mode.json'));print('$mode', d['value'], d['roofline']['avg_launch_us'])"
done
unset MI_DECODE_OLD
MI_SEGV_MAPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 4 --warmup 1 --prompt 3968 --prof-layer -1 > $OUT/lc.json 2> $OUT/lc.err
rc=$?
echo "lc rc $rc"
grep -E "mi_segv|SIGSEGV" $OUT/lc.err | head -60
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/lc_kernel_stats.csv \; 2>/dev/null
rm -rf $OUT/prof
exit 0
