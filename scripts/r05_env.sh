#!/bin/bash
# HIP runtime environment A/B on the decode bench (one process per setting, alternating)
OUT=gpurun_out/${1:-r05e}
mkdir -p $OUT
export TMPDIR=/tmp
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 150 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 128 --warmup 16 > $OUT/b_$name.json 2> $OUT/b_$name.err || { echo "$name failed"; tail -3 $OUT/b_$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/b_$name.json'));print('$name', d['value'], d['roofline']['avg_launch_us'])"
}
for r in 1 2; do
  run base || exit 1
  run devkernarg HIP_FORCE_DEV_KERNARG=1 || exit 1
  run nodevkernarg HIP_FORCE_DEV_KERNARG=0 || exit 1
  run pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
  run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
done
exit 0
