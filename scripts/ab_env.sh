#!/bin/bash
# Decode bench A/B over environment settings (no CPU leg, no prefill/verify legs).
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
shift
for v in "$@"; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 256 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$v',d['value'],d['roofline']['avg_launch_us'])"
done
