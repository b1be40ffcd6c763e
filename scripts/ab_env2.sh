#!/bin/bash
# A/B of environment settings on the decode bench (no CPU leg): one line per setting.
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
for e in "$@"; do
  env $e timeout -k 10 120 python -u bench.py --no-cpu --steps 128 --warmup 16 > $OUT/b.json 2> $OUT/b.err || { echo "fail $e"; tail -5 $OUT/b.err; exit 1; }
  python - "$e" $OUT/b.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:40s} {d['value']:8.1f} tok/s  gate/up {d['roofline']['avg_launch_us']:.2f} us  prefill {d.get('prefill', {}).get('ms')}")
PY
done
