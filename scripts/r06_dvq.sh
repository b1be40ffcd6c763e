#!/bin/bash
# r06 A/B on one box: the RMSNorm quantisation launch as one wave per 256-block (MI_DVQ1=1, no LDS
# or barrier, bit-identical) vs four waves (dv_quant_kernel); decode bit-identity first.
OUT=gpurun_out/${1:-r06_dvq}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u - > $OUT/ident.txt 2>&1 <<'PY'
import os, subprocess, sys, numpy as np
code = r'''
import sys, numpy as np
sys.path.insert(0, ".")
from blama_amd import engine, synthetic
out = []
for name in ["tiny-q4_k_m", "tiny-q8_0"]:
    cfg = synthetic.CONFIGS[name]
    m = engine.Model(synthetic.build_gguf(cfg, seed=3))
    c = engine.Context(m, n_ctx=64)
    c.decode([1, 5, 9])
    for t in [4, 8, 15, 16, 23]:
        c.decode([t]); out.append(c.logits())
    c.close(); m.close()
np.save(sys.argv[1], np.concatenate(out))
'''
for f in ("0", "1"):
    env = dict(os.environ, MI_DVQ1=f, MI_NO_BATCH="1")
    subprocess.run([sys.executable, "-c", code, f"/tmp/dvq{f}.npy"], env=env, check=True)
a, b = np.load("/tmp/dvq0.npy"), np.load("/tmp/dvq1.npy")
print("bit-identical:", np.array_equal(a.view(np.uint32), b.view(np.uint32)))
PY
rc=$?; cat $OUT/ident.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for f in 1 0; do
    MI_DVQ1=$f timeout -k 10 200 python -u bench.py --no-cpu --prefill 0 --verify 0 --steps 128 --warmup 16 --prof-layer -1 \
        > $OUT/bench_f${f}_$i.json 2> $OUT/bench_f${f}_$i.err || { tail -3 $OUT/bench_f${f}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_f${f}_$i.json'));print('dvq1=$f', d['value'], d['ms_per_step'])"
  done
done
