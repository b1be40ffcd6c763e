set -o pipefail
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_ops.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for i in 1 2; do
for v in nomix mix; do
  if [ $v = nomix ]; then export MI_NO_MIX=1; else unset MI_NO_MIX; fi
  timeout -k 10 200 python -u bench.py --no-cpu --steps 256 --warmup 16 --prefill 0 > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail -20 $O/bench_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v', d['value'], d['roofline']['frac'])"
done
done
