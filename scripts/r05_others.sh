#!/bin/bash
# the other BASELINE configs' bench lines (decode with the CPU leg and LogitComparer where the
# bench runs it, prefill, verify, verify_short)
OUT=gpurun_out/${1:-r05ot}
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in tinyllama-1.1b-q8_0 llama3-8b-q6_k mixtral-8x7b-q5_k_m; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 64 --warmup 8 > $OUT/bench_other_$cfg.json 2> $OUT/$cfg.err || { tail -5 $OUT/$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_other_$cfg.json'));p=d['prefill'];print('$cfg decode',d['value'],'prefill',p['ms'],'verify',p['verify']['ms'],'short',[v['ms'] for v in p['verify_short']],'lc',d.get('logit_comparer_vs_cpu',{}).get('pass'))"
done
exit 0
