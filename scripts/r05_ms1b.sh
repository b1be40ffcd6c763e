#!/bin/bash
OUT=gpurun_out/${1:-r05m2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_ops.py -k "mmqs" -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for mode in 1 0 1 0; do
  MI_MMQS1=$mode timeout -k 10 200 python -u bench.py --no-cpu --steps 8 --warmup 2 --verify 0 > $OUT/bench_ms$mode.json 2> $OUT/bench_ms$mode.err || { tail -5 $OUT/bench_ms$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_ms$mode.json'));p=d['prefill'];print('mmqs1=$mode short',[v['ms'] for v in p.get('verify_short',[])])"
done
exit 0
