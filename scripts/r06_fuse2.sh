#!/bin/bash
# A/B on one box: in-launch activations per edge (MI_DV_FUSE 0 none, 1 all, 2 h only, 3 normed x only)
# and the decode attention's entry prefetch (MI_ATTN_PF2=1: two steps, the r06 kernel's depth).
OUT=gpurun_out/${1:-r06_fuse2}; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 128 --warmup 16 \
      > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -3 $OUT/bench_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
}
for i in 1 2; do
  run f0_$i MI_DV_FUSE=0
  run f2_$i MI_DV_FUSE=2
  run f3_$i MI_DV_FUSE=3
  run f0pf2_$i MI_DV_FUSE=0 MI_ATTN_PF2=1
done
