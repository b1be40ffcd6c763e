#!/bin/bash
# r06: MoE decode with the streaming attention half (dv_quant -> dgemv Q/K/V -> attn_dec -> dgemv WO)
# and the r04 expert FFN -- the MoE tests, then alternating Mixtral decode benches against the
# whole r04 step (MI_SP_MOE=0, a switch removed once this ran) on one box.
OUT=gpurun_out/${1:-r06_spm}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_decode.py \
    tests/test_gpu_verify.py tests/test_gpu_fullwidth.py tests/test_gpu_fulldepth.py -k "moe or mixtral" > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|attribution" $OUT/pytest.log | cut -c1-160; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 1 0; do
    MI_SP_MOE=$f timeout -k 10 300 python -u bench.py --config mixtral-8x7b-q5_k_m --no-cpu --prefill 0 --verify 0 --prof-layer -1 --steps 64 --warmup 8 \
        > $OUT/bench_m${f}_$i.json 2> $OUT/bench_m${f}_$i.err || { tail -3 $OUT/bench_m${f}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_m${f}_$i.json'));print('sp_moe=$f mixtral decode', d['value'])"
  done
done
