#!/bin/bash
# decode A/B on one box: the streaming step against the gemv_kernel step (MI_DECODE_OLD=1) as the
# same-box control, alternating, one process each
OUT=gpurun_out/${1:-r05ab}
mkdir -p $OUT
export TMPDIR=/tmp
for mode in new old new old; do
  unset MI_DECODE_OLD
  if [ $mode = old ]; then export MI_DECODE_OLD=1; fi
  timeout -k 10 150 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 128 --warmup 16 > $OUT/bench_$mode.json 2> $OUT/bench_$mode.err || { echo "bench $mode failed"; tail -5 $OUT/bench_$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$mode.json'));print('$mode', d['value'], d['roofline']['avg_launch_us'])"
done
exit 0
