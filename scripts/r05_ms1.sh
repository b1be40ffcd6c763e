#!/bin/bash
# one-wave short GEMM (mmqs1) parity + A/B against the LDS form (MI_MMQS1=0), then the decode A/B
OUT=gpurun_out/${1:-r05m}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_batch_ops.py tests/test_gpu_verify.py tests/test_gpu_fullwidth.py -k "mmqs or out_all or short or batched" -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -10; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for mode in 1 0 1 0; do
  MI_MMQS1=$mode timeout -k 10 200 python -u bench.py --no-cpu --steps 8 --warmup 2 --verify 0 > $OUT/bench_ms$mode.json 2> $OUT/bench_ms$mode.err || { tail -5 $OUT/bench_ms$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_ms$mode.json'));p=d['prefill'];print('mmqs1=$mode short',[v['ms'] for v in p.get('verify_short',[])])"
done
bash scripts/r05_ab.sh ${1:-r05m}_ab || exit 1
exit 0
