#!/bin/bash
# One GPU-box session: GPU parity tests, the N=1 bench line, and a rocprofv3
# kernel-trace summary of a shorter bench run.  Each GPU step has its own time
# limit; a crash/abort/timeout of any step ends the script (no retries).
# Usage: scripts/gpu_round.sh [tag]
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ok() {  # continue only on 0 (pass) or 1 (pytest test failures)
  local rc=$1 what=$2
  echo "[$what] exit $rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what"; exit "$rc"; fi
}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1
  ok $? pytest
  tail -3 $OUT/pytest_gpu.log
fi
if [ -n "$SWEEP" ]; then
  timeout -k 10 600 python -u scripts/gemv_sweep.py $SWEEP > $OUT/sweep.txt 2>&1
  ok $? sweep
  cat $OUT/sweep.txt
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
  ok $? bench
  cat $OUT/bench.json
fi
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
      python -u bench.py --no-cpu --steps 32 --warmup 4 ${PROF_ARGS} > $OUT/prof_bench.json 2> $OUT/prof.err
  ok $? rocprof
  find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
  head -20 $OUT/kernel_stats.csv
fi
