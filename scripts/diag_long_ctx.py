"""Diagnostic (GPU): per-step oracle error of decode past 512 cells for a few small configs."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
from blama_amd import engine, synthetic
from util import oracle_from_gguf

def run(name, plen, steps, **kw):
    cfg = synthetic.small_config(name, **kw)
    buf = synthetic.build_gguf(cfg, seed=5)
    m = engine.Model(buf)
    ctx = engine.Context(m, n_ctx=plen + steps + 8)
    orc = oracle_from_gguf(buf, n_ctx=plen + steps + 8)
    prompt = list(np.random.default_rng(4).integers(0, cfg.n_vocab, plen))
    out = []
    ctx.decode(prompt)
    ref = orc.decode(prompt)
    rng = np.random.default_rng(2)
    for s in range(steps + 1):
        rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
        out.append(f"{float(np.max(np.abs(ctx.logits() - ref))) / rms:.1e}")
        if s == steps:
            break
        t = int(rng.integers(0, cfg.n_vocab))
        ctx.decode([t])
        ref = orc.decode_one(t)
    print(name, plen, os.environ.get("MI_NO_GRAPH", ""), out, flush=True)

run("tiny-gpt2-q6_k", 520, 6, n_ctx_train=1024)
run("tiny-gpt2-q6_k", 500, 20, n_ctx_train=1024)
run("tiny-gpt2-q8_0", 520, 6, n_ctx_train=1024)
run("tiny-q6_k", 520, 6)
