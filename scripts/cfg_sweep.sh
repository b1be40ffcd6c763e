#!/bin/bash
# Whole-bench sweep of per-role GEMV configurations (MI_GEMV_CFG_<ROLE>, indices into
# kGemvCfgs): one short bench process per variant, each under its own time limit.
mkdir -p gpurun_out/sweep
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 90 python -u bench.py --no-cpu --prefill 0 --steps 128 --warmup 16 \
      > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep/$tag.json')); print('$tag', d['value'], d['roofline']['avg_launch_us'])"
}
run base X=1
for v in 0 3 4; do run down$v MI_GEMV_CFG_DOWN=$v; done
for v in 0 2 3; do run qkv$v MI_GEMV_CFG_QKV=$v; done
for v in 0 2; do run wo$v MI_GEMV_CFG_WO=$v; done
for v in 0 3; do run out$v MI_GEMV_CFG_OUT=$v; done
run up3 MI_GEMV_CFG_UP=3
run base2 X=1
