#!/bin/bash
# Selected GPU tests + the bench's prefill leg (no CPU leg).  Usage: scripts/gpu_quick.sh tag "pytest args" [env...]
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/t.log | tail -40
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
shift 2
for v in "$@"; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu --steps 8 --warmup 2 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$v','decode',d['value'],'prefill ms',d['prefill']['ms'])"
done
