set -o pipefail
O=gpurun_out/r01y; mkdir -p $O
export TMPDIR=/tmp
run() { tag=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --no-cpu --steps 64 --warmup 8 --prefill 0 > $O/b_$tag.json 2> $O/b_$tag.err || exit $?; echo "$tag: $(python -c "import json;d=json.load(open('$O/b_$tag.json'));print(d['value'], d['roofline']['avg_launch_us'])")"; }
run default X=1
run down0 MI_GEMV_CFG_DOWN=0
run qkv0 MI_GEMV_CFG_QKV=0
run wo0 MI_GEMV_CFG_WO=0
run out0 MI_GEMV_CFG_OUT=0
