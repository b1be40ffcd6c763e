set -o pipefail
O=gpurun_out/r02j; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_http.py -m gpu > $O/pytest_host.log 2>&1 || { tail -40 $O/pytest_host.log; exit 1; }
tail -5 $O/pytest_host.log
