#!/bin/bash
# r06: the decode attention kernel (attn_dec) -- parity tests, then the bench rate
OUT=gpurun_out/r06_attn
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullwidth.py -x -q --timeout 300 --timeout-method thread -k "not short" > $OUT/t.log 2>&1; rc=$?
tail -5 $OUT/t.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu --steps 128 --warmup 16 --prefill 0 --prof-layer 16 > $OUT/b$i.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/b$i.json'));print('decode',d['value'],'profiled pass',d['roofline']['timed_in'],'ffn us',d['roofline']['avg_launch_us'])"
done
