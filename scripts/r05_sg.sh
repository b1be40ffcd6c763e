#!/bin/bash
# short-batch hipGraphs: verification / host / HTTP parity tests, then the short legs with and
# without graphs (MI_NO_GRAPH=1 also makes decode eager: only the verify_short legs compare)
OUT=gpurun_out/${1:-r05g}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_fullwidth.py tests/test_host.py tests/test_http.py tests/test_gpu_decode.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -10; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for mode in graph eager graph eager; do
  if [ $mode = eager ]; then export MI_NO_GRAPH=1; else unset MI_NO_GRAPH; fi
  timeout -k 10 200 python -u bench.py --no-cpu --steps 8 --warmup 2 --verify 0 > $OUT/bench_$mode.json 2> $OUT/bench_$mode.err || { tail -5 $OUT/bench_$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$mode.json'));p=d['prefill'];print('$mode short',[v['ms'] for v in p.get('verify_short',[])])"
done
exit 0
