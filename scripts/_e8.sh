mkdir -p gpurun_out/e8
for v in "1 8" "0 8" "2 8" "2 1" "2 0" "1 1" "0 1" "1 0"; do
  set -- $v
  MI_GEMV_ORDER=$1 MI_GEMV_PRE=$2 timeout -k 10 200 python -u bench.py --no-cpu --steps 64 --warmup 8 --prefill 0 > gpurun_out/e8/b_$1_$2.json 2> gpurun_out/e8/b_$1_$2.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/e8/b_$1_$2.json'));print('order $1 pre $2:', d['value'], 'tok/s  gate/up', d['roofline']['avg_launch_us'], 'us')"
done
