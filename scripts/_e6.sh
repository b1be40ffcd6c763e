mkdir -p gpurun_out/e6
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_decode.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e6/pytest.log 2>&1; echo "pytest rc $?"; tail -3 gpurun_out/e6/pytest.log
MI_ENGINE_LIB=stamps timeout -k 10 300 python -u scripts/timeline.py llama2-7b-q4_k_m 64 > gpurun_out/e6/timeline.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu --steps 64 --warmup 8 --prefill 0 > gpurun_out/e6/bench.json 2> gpurun_out/e6/bench.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/e6/bench.json'));print('bench', d['value'], d['roofline']['avg_launch_us'])"
sed -n 1,25p gpurun_out/e6/timeline.txt; tail -3 gpurun_out/e6/timeline.txt
