#!/bin/bash
# r06: the FFN down launch quantising h itself in every workgroup (dgemv DV_ADDQ, no dv_quant
# launch before it) -- decode / full-width / full-depth tests with it forced on (MI_HQ=1), then
# alternating decode benches on one box, TinyLlama and 7B, MI_HQ=1 vs 0 (a switch removed once
# this ran).
OUT=gpurun_out/${1:-r06_hq}; mkdir -p $OUT; export TMPDIR=/tmp
MI_HQ=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_decode.py \
    tests/test_gpu_fullwidth.py -k "not moe and not mixtral and not batched and not short_batches" > $OUT/pytest.log 2>&1
rc=$?; grep -cE "PASSED" $OUT/pytest.log; grep -E "FAILED|Error" $OUT/pytest.log | head -5; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for cfg in tinyllama-1.1b-q8_0 llama2-7b-q4_k_m; do
    for f in 1 0; do
      MI_HQ=$f timeout -k 10 300 python -u bench.py --config $cfg --no-cpu --prefill 0 --verify 0 --prof-layer -1 --steps 128 --warmup 16 \
          > $OUT/b_${cfg}_${f}_$i.json 2> $OUT/b_${cfg}_${f}_$i.err || { tail -3 $OUT/b_${cfg}_${f}_$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/b_${cfg}_${f}_$i.json'));print('$cfg hq=$f rep $i', d['value'])"
    done
  done
done
