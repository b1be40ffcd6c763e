#!/bin/bash
# r06: small dense models with the normed Q/K/V and gate/up inputs quantised inside their launches
# (dgemv DV_QKVN / DV_SWIGLUN) -- logits bit-identical to the dv_quant step (MI_NQ=0), the decode
# tests, then alternating TinyLlama decode benches (MI_NQ=0 vs on).
OUT=gpurun_out/${1:-r06_nq}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/nq_dump.py $OUT on > $OUT/dump_on.log 2>&1 || { tail -5 $OUT/dump_on.log; exit 1; }
MI_NQ=0 timeout -k 10 300 python -u scripts/nq_dump.py $OUT off > $OUT/dump_off.log 2>&1 || { tail -5 $OUT/dump_off.log; exit 1; }
python3 - $OUT <<'PY' || exit 1
import sys, numpy as np, glob, os
bad = 0
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_on.npy"))):
    a, b = np.load(f), np.load(f.replace("_on.npy", "_off.npy"))
    same = np.array_equal(a.view(np.uint32), b.view(np.uint32))
    print(os.path.basename(f)[:-7], "bit-identical" if same else f"DIFFER max {np.abs(a - b).max():.3e}")
    bad += not same
sys.exit(1 if bad else 0)
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_dgemv.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 0 1; do
    MI_NQ=$f timeout -k 10 300 python -u bench.py --config tinyllama-1.1b-q8_0 --no-cpu --prefill 0 --verify 0 --prof-layer -1 --steps 128 --warmup 16 \
        > $OUT/b_${f}_$i.json 2> $OUT/b_${f}_$i.err || { tail -3 $OUT/b_${f}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${f}_$i.json'));print('tinyllama nq=$f rep $i', d['value'])"
  done
done
