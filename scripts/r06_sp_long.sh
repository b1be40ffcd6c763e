#!/bin/bash
# r06: the streaming decode step past 512 cells (split attention, then attn_combine_quant_kernel
# feeding the dgemv WO launch) -- the tests that cross 512 cells, then alternating 3968-cell decode
# benches against the r04 gemv_kernel step (MI_SP_LONG=0, a switch removed once this ran) on one box.
OUT=gpurun_out/${1:-r06_spl}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_decode.py \
    tests/test_gpu_verify.py tests/test_gpu_fullwidth.py -k "split or 512 or long or past or beyond or cross or 1100" > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED" $OUT/pytest.log | cut -c1-120; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 1 0; do
    MI_SP_LONG=$f timeout -k 10 300 python -u bench.py --no-cpu --prefill 0 --verify 0 --prof-layer -1 --steps 64 --warmup 4 --prompt 3968 \
        > $OUT/bench_l${f}_$i.json 2> $OUT/bench_l${f}_$i.err || { tail -3 $OUT/bench_l${f}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_l${f}_$i.json'));print('sp_long=$f 3968 cells', d['value'])"
  done
done
