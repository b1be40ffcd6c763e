#!/bin/bash
# A/B on one box: h-only in-launch activation (MI_DV_FUSE=2) and the decode attention's entry
# prefetch depth (MI_ATTN_PF: cell steps per wave requested at entry; 0 = the first 256 cells).
OUT=gpurun_out/${1:-r06_fuse3}; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 128 --warmup 16 \
      > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -3 $OUT/bench_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
}
for i in 1 2 3; do
  run f0pf2_$i MI_DV_FUSE=0 MI_ATTN_PF=2
  run f2pf2_$i MI_DV_FUSE=2 MI_ATTN_PF=2
  run f0pf1_$i MI_DV_FUSE=0 MI_ATTN_PF=1
  run f0pf3_$i MI_DV_FUSE=0 MI_ATTN_PF=3
  run f0pf4_$i MI_DV_FUSE=0 MI_ATTN_PF=4
done
