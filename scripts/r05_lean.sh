#!/bin/bash
# mmqs1 one-deep rings at two waves per SIMD (MI_MMQS1_LEAN=1) against the default, same box:
# the short-GEMM op tests on the lean form, then the 7B and Mixtral verify_short legs alternating
OUT=gpurun_out/${1:-r05ln}
mkdir -p $OUT
export TMPDIR=/tmp
MI_MMQS1_LEAN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_ops.py -k mmqs -x -q --timeout 200 --timeout-method thread > $OUT/ops.log 2>&1 || { tail -5 $OUT/ops.log; exit 1; }
tail -1 $OUT/ops.log
for cfg in llama2-7b-q4_k_m mixtral-8x7b-q5_k_m; do
  for lean in 0 1 0 1; do
    MI_MMQS1_LEAN=$lean timeout -k 10 300 python -u bench.py --config $cfg --no-cpu --steps 8 --warmup 2 > $OUT/b_${cfg}_$lean.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${cfg}_$lean.json'));p=d['prefill'];print('$cfg lean $lean','short',[v['ms'] for v in p['verify_short']])"
  done
done
exit 0
