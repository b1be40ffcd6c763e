#!/bin/bash
# Split-attention variants at long contexts: kernel stats of a 7B decode at ~3968 cells per
# MI_ATTN_U setting, and the bench rate.  Usage: scripts/attn_long.sh tag [U...]
OUT=gpurun_out/${1:-al}
shift
mkdir -p $OUT
export TMPDIR=/tmp
for U in "$@"; do
  MI_ATTN_U=$U timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$U -o run -- \
      python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 32 --warmup 4 --prompt 3968 --prof-layer -1 \
      > $OUT/b$U.json 2> $OUT/b$U.err || { tail $OUT/b$U.err; exit 1; }
  find $OUT/prof$U -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_u$U.csv \;
  echo "U=$U"; grep -E "attn_|gemv_kernel<12, -1, 1, 1" $OUT/kernel_stats_u$U.csv | cut -d, -f1,2,4 | cut -c1-140
  MI_ATTN_U=$U timeout -k 10 300 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 64 --warmup 4 --prompt 3968 \
      > $OUT/r$U.json 2> $OUT/r$U.err || { tail $OUT/r$U.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/r$U.json'));print('U=$U tok/s', d['value'])"
done
