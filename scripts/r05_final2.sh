#!/bin/bash
# round-end check: smoke(), the whole GPU suite, then the default bench line
OUT=gpurun_out/${1:-r05z}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2; grep -E "live-floor waiver|distributions, score" $OUT/pytest_gpu.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));p=d['prefill'];print('decode',d['value'],d['roofline']['frac'],d['roofline']['traffic'],'prefill',p['ms'],'verify',p['verify']['ms'],'short',[v['ms'] for v in p['verify_short']],'cpu',d['cpu_baseline']['value'],d['logit_comparer_vs_cpu']['pass'])"
exit 0
