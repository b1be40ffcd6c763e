#!/bin/bash
# A/B of mmq32 variants on the 7B 512-token prefill leg (bench.py, no CPU leg) + batch tests.
OUT=gpurun_out/${1:-mmq}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
shift
for v in "$@"; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu --steps 8 --warmup 2 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$v','decode',d['value'],'prefill ms',d['prefill']['ms'])"
done
