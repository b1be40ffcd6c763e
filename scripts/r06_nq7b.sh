#!/bin/bash
# r06: the normed-input in-launch quantisation forced on for 7B and Llama-3-8B (MI_NQ=1) vs their
# dv_quant launches, alternating decode benches on one box.
OUT=gpurun_out/${1:-r06_nq7b}; mkdir -p $OUT; export TMPDIR=/tmp
for i in 1 2; do
  for cfg in llama2-7b-q4_k_m llama3-8b-q6_k; do
    for f in 1 ""; do
      MI_NQ=$f timeout -k 10 300 python -u bench.py --config $cfg --no-cpu --prefill 0 --verify 0 --prof-layer -1 --steps 128 --warmup 16 \
          > $OUT/b_${cfg}_${f:-d}_$i.json 2> $OUT/b_${cfg}_${f:-d}_$i.err || { tail -3 $OUT/b_${cfg}_${f:-d}_$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/b_${cfg}_${f:-d}_$i.json'));print('$cfg nq=${f:-default} rep $i', d['value'])"
    done
  done
done
