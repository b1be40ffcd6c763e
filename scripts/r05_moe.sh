#!/bin/bash
# MoE short batches on the grouped mmqs: the Mixtral parity tests, then the Mixtral bench line
# (verify_short legs) with the grouped path and with MI_MOE_SHORT_OFF=1 (the tiled control)
OUT=gpurun_out/${1:-r05moe}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullwidth.py -k mixtral -x -v -s --timeout 300 --timeout-method thread > $OUT/t_fw.log 2>&1
rc=$?; echo "fullwidth rc $rc"; grep -E "passed|failed|Error|assert" $OUT/t_fw.log | tail -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fulldepth.py -k mixtral -x -v -s --timeout 500 --timeout-method thread > $OUT/t_fd.log 2>&1
rc=$?; echo "fulldepth rc $rc"; grep -E "passed|failed|score|assert" $OUT/t_fd.log | tail -5
[ $rc -eq 0 ] || exit 1
for mode in on off; do
  if [ $mode = off ]; then export MI_MOE_SHORT_OFF=1; fi
  timeout -k 10 300 python -u bench.py --config mixtral-8x7b-q5_k_m --no-cpu --steps 16 --warmup 4 > $OUT/bench_$mode.json 2> $OUT/bench_$mode.err || { tail -5 $OUT/bench_$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$mode.json'));p=d['prefill'];print('$mode decode',d['value'],'prefill',p['ms'],'verify',p['verify']['ms'],'short',[v['ms'] for v in p['verify_short']])"
done
exit 0
