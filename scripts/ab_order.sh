#!/bin/bash
# Decode A/B over environment settings: the decode parity tests under each setting, then the
# decode bench alternating settings (twice).  Usage: scripts/ab_order.sh tag "ENV=.. ENV=.." ...
# (a setting is a space-separated list of VAR=value; "-" for none)
OUT=gpurun_out/${1:-ab_order}
mkdir -p $OUT
shift
TESTS=${TESTS:-"tests/test_gpu_decode.py tests/test_gpu_fullwidth.py"}
i=0
for v in "$@"; do
  i=$((i+1)); [ "$v" = "-" ] && v=""
  env $v timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t_$i.log 2>&1
  rc=$?; echo "[$v] tests: $(tail -1 $OUT/t_$i.log)"
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1)); [ "$v" = "-" ] && v=""
    env $v timeout -k 10 200 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 256 > $OUT/b_$i.json 2> $OUT/b_$i.err || { tail $OUT/b_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_$i.json'));print('[$v]',d['value'],d['roofline']['avg_launch_us'])"
  done
done
