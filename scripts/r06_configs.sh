#!/bin/bash
# r06: the other BASELINE configs' bench lines (decode with the CPU leg and the LogitComparer gate,
# prefill, verify, verify_short) and the 3968-cell decode of the dense models.
OUT=gpurun_out/${1:-r06_cfg}; mkdir -p $OUT; export TMPDIR=/tmp
for cfg in tinyllama-1.1b-q8_0 llama3-8b-q6_k mixtral-8x7b-q5_k_m; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 64 --warmup 8 --cpu-seconds 10 > $OUT/bench_other_$cfg.json 2> $OUT/$cfg.err || { tail -5 $OUT/$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_other_$cfg.json'));p=d['prefill'];print('$cfg decode',d['value'],'frac',d['whole_step_hbm_frac'],'prefill',p['ms'],'verify',p['verify']['ms'],'short',[v['ms'] for v in p['verify_short']],'cpu',d['cpu_baseline']['value'],'lc',d.get('logit_comparer_vs_cpu',{}).get('pass'))"
done
for cfg in llama2-7b-q4_k_m llama3-8b-q6_k; do
  timeout -k 10 400 python -u bench.py --config $cfg --no-cpu --prefill 0 --verify 0 --prof-layer -1 --steps 64 --warmup 4 --prompt 3968 > $OUT/bench_long_$cfg.json 2> $OUT/long_$cfg.err || { tail -5 $OUT/long_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_long_$cfg.json'));print('$cfg 3968 cells decode',d['value'])"
done
