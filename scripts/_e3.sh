mkdir -p gpurun_out/e3
timeout -k 10 200 ./scripts/exp_gemv2_st 1 > gpurun_out/e3/stamps.txt 2>&1 || exit $?
timeout -k 10 200 ./scripts/exp_gemv2 2 > gpurun_out/e3/chain.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_http.py tests/test_host.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/e3/pytest.log 2>&1
echo "pytest rc $?"
grep -E "stamps|chain" gpurun_out/e3/stamps.txt gpurun_out/e3/chain.txt
tail -15 gpurun_out/e3/pytest.log
