#!/bin/bash
# The other BASELINE configs on the current code (decode + 512-token prefill + verify-256/64/20
# legs; Mixtral with the CPU leg, so its line carries logit_comparer_vs_cpu), then decode at 3968
# cells for 7B and Llama-3-8B.  Usage: scripts/gpu_configs.sh tag
OUT=gpurun_out/${1:-cfg}
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in tinyllama-1.1b-q8_0 llama3-8b-q6_k mixtral-8x7b-q5_k_m; do
  cpu="--no-cpu"
  if [ $cfg = mixtral-8x7b-q5_k_m ]; then cpu="--cpu-seconds 45"; fi
  timeout -k 10 400 python -u bench.py $cpu --steps 64 --warmup 8 --config $cfg > $OUT/$cfg.json 2> $OUT/$cfg.err || { tail $OUT/$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$cfg.json'));p=d.get('prefill') or {};print('$cfg','decode',d['value'],'frac',d['whole_step_hbm_frac'],'prefill ms',p.get('ms'),'verify ms',(p.get('verify') or {}).get('ms'),'short',[v['ms'] for v in p.get('verify_short',[])],'lc',d.get('logit_comparer_vs_cpu'))" | tee -a $OUT/summary.txt
done
for cfg in llama2-7b-q4_k_m llama3-8b-q6_k; do
  timeout -k 10 300 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 64 --warmup 4 --config $cfg --prompt 3968 > $OUT/lc_$cfg.json 2> $OUT/lc_$cfg.err || { tail $OUT/lc_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/lc_$cfg.json'));print('$cfg','3968 cells decode',d['value'])" | tee -a $OUT/summary.txt
done
