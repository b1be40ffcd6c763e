mkdir -p gpurun_out/e9
for v in "2 0" "0 8"; do
  set -- $v
  MI_GEMV_ORDER=$1 MI_GEMV_PRE=$2 MI_ENGINE_LIB=stamps timeout -k 10 300 python -u scripts/timeline.py llama2-7b-q4_k_m 64 > gpurun_out/e9/timeline_$1_$2.txt 2>&1 || exit $?
  echo "=== order $1 pre $2"; sed -n 1,12p gpurun_out/e9/timeline_$1_$2.txt; tail -1 gpurun_out/e9/timeline_$1_$2.txt
done
MI_GEMV_ORDER=0 MI_GEMV_PRE=8 timeout -k 10 200 python -u bench.py --no-cpu --steps 64 --warmup 8 --prefill 0 > gpurun_out/e9/b.json 2> gpurun_out/e9/b.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/e9/b.json'));print('bench', d['value'], 'tok/s  gate/up', d['roofline']['avg_launch_us'], 'us')"
