#!/bin/bash
# Prefill / verify A/B over environment settings (bench legs only, decode short, no CPU leg), e.g.
#   scripts/ab_prefill.sh tag MI_MMQ2_DIAG=0 MI_MMQ2_DIAG=1 MI_MMQ2_DIAG=2
OUT=gpurun_out/${1:-abp}
mkdir -p $OUT
shift
for v in "$@"; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu --steps 4 --warmup 2 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$v','prefill ms',d['prefill']['ms'],'verify ms',d['prefill']['verify']['ms'])"
done
