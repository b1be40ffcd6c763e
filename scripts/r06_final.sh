#!/bin/bash
# r06 round-end check: GPU parity suite, smoke, the default bench line (CPU leg included), and the
# eager kernel trace of the decode bench (rocprofv3 --kernel-trace --stats; the graph run's tracer
# fault, DESIGN.md §8 r05, keeps profiles on eager launches).
OUT=gpurun_out/${1:-r06_final}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -3 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], d['prefill']['ms'], [v['ms'] for v in d['prefill']['verify_short']])"
bash scripts/r06_trace.sh ${1:-r06_final}_trace
