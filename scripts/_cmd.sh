set -o pipefail
O=gpurun_out/r02b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 ./scripts/exp_mfma_layout || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc $rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u bench.py --no-cpu --steps 64 --warmup 8 > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d.get('prefill'))"
