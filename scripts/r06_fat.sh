#!/bin/bash
# r06: fat-workgroup GEMV experiment + bench with/without the profiling split
OUT=gpurun_out/r06_fat
mkdir -p $OUT
timeout -k 10 240 ./scripts/exp_fat 3 > $OUT/exp.txt 2>&1 || { echo "exp rc=$?"; tail $OUT/exp.txt; exit 1; }
cat $OUT/exp.txt
for pl in 16 -1 16 -1; do
  timeout -k 10 200 python -u bench.py --no-cpu --steps 128 --warmup 16 --prefill 0 --prof-layer $pl > $OUT/b_$pl.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b_$pl.json'));print('prof-layer $pl decode',d['value'])"
done
