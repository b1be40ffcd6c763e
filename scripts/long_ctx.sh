#!/bin/bash
# Decode tok/s at long contexts (verdict r01 item 7): prompt of P tokens ingested by the batch
# path, then 64 decode steps at n_past ~ P.  7B (n_ctx_train 4096) and Llama-3-8B.
OUT=gpurun_out/${1:-lc}
mkdir -p $OUT
for cfg in llama2-7b-q4_k_m llama3-8b-q6_k; do
  for P in 512 2048 3968; do
    timeout -k 10 300 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 64 --warmup 4 --config $cfg --prompt $P > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$cfg', $P, d['value'])" | tee -a $OUT/summary.txt
  done
done
