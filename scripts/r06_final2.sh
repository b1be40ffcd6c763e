#!/bin/bash
# r06 round-end check after the small-model in-launch quantisations: GPU parity suite, smoke, the
# default bench line, the TinyLlama decode line.
OUT=gpurun_out/${1:-r06_final2}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -3 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], d['prefill']['ms'], [v['ms'] for v in d['prefill']['verify_short']])"
timeout -k 10 300 python -u bench.py --config tinyllama-1.1b-q8_0 --no-cpu > $OUT/bench_tinyllama.json 2> $OUT/bench_tinyllama.err || { tail -3 $OUT/bench_tinyllama.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_tinyllama.json'));print('tinyllama', d['value'], [v['ms'] for v in d['prefill']['verify_short']])"
