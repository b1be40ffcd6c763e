#!/bin/bash
# r06: the tiled prompt-batch GEMM on pre-scaled Q4_K / Q5_K operand planes (QMat::ps) -- op
# tests (bit-identity with the in-LDS decode), the batch / verify / prefill parity tests, then
# alternating bench prefill + verify legs with MI_MMQ_PS=1 / 0 on one box.
OUT=gpurun_out/${1:-r06_psg}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch_ops.py \
    tests/test_gpu_decode.py -k "prescaled or gqa16" \
    > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for ps in 1 0; do
    MI_MMQ_PS=$ps timeout -k 10 300 python -u bench.py --no-cpu --steps 16 --warmup 4 --prof-layer -1 \
        > $OUT/bench_ps${ps}_$i.json 2> $OUT/bench_ps${ps}_$i.err || { tail -3 $OUT/bench_ps${ps}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_ps${ps}_$i.json'));p=d['prefill'];print('ps=$ps prefill',p['ms'],'verify256',p['verify']['ms'],'short',[v['ms'] for v in p['verify_short']])"
  done
done
