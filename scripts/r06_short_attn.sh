#!/bin/bash
# r06 A/B on one box (run before the switch was removed; now the default): a short batch's attention on attn_dec_kernel
# one grid row per token, MI_SHORT_DEC=1) vs the fused kernel; the verify tests first.
OUT=gpurun_out/${1:-r06_sattn}; mkdir -p $OUT; export TMPDIR=/tmp
MI_SHORT_DEC=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_verify.py \
    tests/test_gpu_decode.py -k "verify or batched or gqa16 or short" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for f in 1 0; do
    MI_SHORT_DEC=$f timeout -k 10 300 python -u bench.py --no-cpu --steps 16 --warmup 4 --prof-layer -1 \
        > $OUT/bench_d${f}_$i.json 2> $OUT/bench_d${f}_$i.err || { tail -3 $OUT/bench_d${f}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_d${f}_$i.json'));p=d['prefill'];print('short_dec=$f verify256',p['verify']['ms'],'short',[v['ms'] for v in p['verify_short']])"
  done
done
