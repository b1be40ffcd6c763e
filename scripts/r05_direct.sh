#!/bin/bash
# decode GEMVs reading their activation slices from global memory (libmi_engine_exp.so built with
# -DMI_DV_DIRECT) against the LDS copy (libmi_engine.so): decode parity on the exp build, then
# alternating A/B on one box
OUT=gpurun_out/${1:-r05x}
mkdir -p $OUT
export TMPDIR=/tmp
MI_ENGINE_LIB=exp timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullwidth.py -k "decode or determin or topk or state or shift or extend or split or crosses" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -10; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for mode in exp base exp base exp base; do
  if [ $mode = exp ]; then export MI_ENGINE_LIB=exp; else unset MI_ENGINE_LIB; fi
  timeout -k 10 150 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 128 --warmup 16 > $OUT/bench_$mode.json 2> $OUT/bench_$mode.err || { tail -5 $OUT/bench_$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$mode.json'));print('$mode', d['value'], d['roofline']['avg_launch_us'])"
done
exit 0
