mkdir -p gpurun_out/e5
export TMPDIR=/tmp
MI_ENGINE_LIB=stamps timeout -k 10 300 python -u scripts/timeline.py llama2-7b-q4_k_m 64 > gpurun_out/e5/timeline.txt 2>&1 || exit $?
for g in 256 512; do
  MI_GEMV_GRID=$g timeout -k 10 300 python -u bench.py --no-cpu --steps 64 --warmup 8 --prefill 0 > gpurun_out/e5/bench_g$g.json 2> gpurun_out/e5/bench_g$g.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/e5/bench_g$g.json'));print('grid $g', d['value'], d['roofline']['avg_launch_us'])"
done
head -60 gpurun_out/e5/timeline.txt
