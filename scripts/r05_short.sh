#!/bin/bash
# short-batch GEMM (mmqs): verification parity tests, then the bench's verify_short legs
OUT=gpurun_out/${1:-r05s}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_fullwidth.py tests/test_gpu_batch_ops.py -k "out_all or short or batched or long_prompt or mmqs" -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "PASS|FAIL|Error|error" $OUT/pytest.log | head -30; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --no-cpu --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));p=d['prefill'];print('decode',d['value'],'prefill',p['ms'],'verify',p['verify']['ms'],'short',p.get('verify_short'))"
MI_MMQS_MAX=0 timeout -k 10 200 python -u bench.py --no-cpu --steps 20 --warmup 5 > $OUT/bench_tiled.json 2> $OUT/bench_tiled.err || { tail -5 $OUT/bench_tiled.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_tiled.json'));p=d['prefill'];print('tiled: short',p.get('verify_short'))"
MI_SHORT_ATTN_FUSED=1 timeout -k 10 200 python -u bench.py --no-cpu --steps 20 --warmup 5 > $OUT/bench_fa.json 2> $OUT/bench_fa.err || { tail -5 $OUT/bench_fa.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_fa.json'));p=d['prefill'];print('fused attn: short',p.get('verify_short'))"
MI_NO_GRAPH=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u bench.py --no-cpu --steps 4 --warmup 2 > $OUT/trace_bench.json 2> $OUT/prof.err || { tail -3 $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/prof -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
rm -rf $OUT/prof
exit 0
