#!/bin/bash
# In-launch activations (dgemv.hip dv_waiter) vs a dv_quant launch between every GEMV pair:
# bit-identity tests, then alternating decode benches on one box.  Usage: scripts/r06_fuse.sh tag
OUT=gpurun_out/${1:-r06_fuse}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_decode.py \
    tests/test_gpu_dgemv.py tests/test_gpu_ops.py tests/test_gpu_fullwidth.py -k "in_launch or bit_determ or matches_oracle or dgemv or attn or decode" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 1 0; do
    MI_DV_FUSE=$f timeout -k 10 200 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 128 --warmup 16 \
        > $OUT/bench_f${f}_$i.json 2> $OUT/bench_f${f}_$i.err || { tail -3 $OUT/bench_f${f}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_f${f}_$i.json'));print('fuse=$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
  done
done
bash scripts/r06_trace.sh ${1:-r06_fuse}_trace
