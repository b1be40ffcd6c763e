#!/bin/bash
# r06: TinyLlama's bench line (CPU leg + LogitComparer gate) after the in-launch quantisations, and
# its decode at 1900 cells (the split attention + combine path with the in-launch quantisations).
OUT=gpurun_out/${1:-r06_tiny}; mkdir -p $OUT; export TMPDIR=/tmp
cfg=tinyllama-1.1b-q8_0
timeout -k 10 400 python -u bench.py --config $cfg --steps 64 --warmup 8 --cpu-seconds 10 > $OUT/bench_other_$cfg.json 2> $OUT/$cfg.err || { tail -5 $OUT/$cfg.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_other_$cfg.json'));p=d['prefill'];print('$cfg decode',d['value'],'frac',d['whole_step_hbm_frac'],'prefill',p['ms'],'verify',p['verify']['ms'],'short',[v['ms'] for v in p['verify_short']],'cpu',d['cpu_baseline']['value'],'lc',d.get('logit_comparer_vs_cpu'))"
timeout -k 10 400 python -u bench.py --config $cfg --no-cpu --prefill 0 --verify 0 --prof-layer -1 --steps 64 --warmup 4 --prompt 1900 > $OUT/bench_long_$cfg.json 2> $OUT/long_$cfg.err || { tail -5 $OUT/long_$cfg.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_long_$cfg.json'));print('$cfg 1900 cells decode',d['value'])"
