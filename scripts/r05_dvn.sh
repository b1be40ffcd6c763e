#!/bin/bash
# in-launch RMSNorm + quantisation (DV_*_N) vs a dv_quant launch before QKV / gate/up / head:
# decode parity tests, then alternating A/B on one box
OUT=gpurun_out/${1:-r05n}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullwidth.py tests/test_gpu_ops.py -k "decode or determin or topk or state or shift or extend or split or crosses" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -10; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for mode in 1 0 1 0 1 0; do
  MI_DV_NORM=$mode timeout -k 10 150 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 128 --warmup 16 > $OUT/bench_n$mode.json 2> $OUT/bench_n$mode.err || { tail -5 $OUT/bench_n$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_n$mode.json'));print('dv_norm=$mode', d['value'], d['roofline']['avg_launch_us'])"
done
exit 0
