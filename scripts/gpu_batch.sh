#!/bin/bash
# Batch-path check: GEMM / attention / verification parity tests, then the bench's prefill and
# verify legs (no decode timing, no CPU leg) and a kernel trace of them.  Usage: scripts/gpu_batch.sh tag
OUT=gpurun_out/${1:-batch}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch_ops.py tests/test_gpu_verify.py tests/test_gpu_fullwidth.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu --steps 8 --warmup 2 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/b.json'));print('decode',d['value'],'prefill ms',d['prefill']['ms'],'verify ms',d['prefill']['verify']['ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u bench.py --no-cpu --steps 4 --warmup 2 > $OUT/pb.json 2> $OUT/pb.err || exit 1
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
head -14 $OUT/kernel_stats.csv | cut -c1-200
