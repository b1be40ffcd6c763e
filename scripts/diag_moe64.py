"""Mixtral (2 layers, n_ff 14336): a 64-token verification batch on the short (grouped mmqs)
and on the tiled path, every row against the C oracle decoding the same tokens one at a time."""
import os, sys, time
import numpy as np
sys.path[:0] = [".", "tests", "oracle"]
import ggml_cpu
from blama_amd import engine, synthetic

cfg = synthetic.small_config("mixtral-8x7b-q5_k_m", n_layer=2)
buf = synthetic.build_gguf(cfg, seed=3)
m = engine.Model(buf)
rng = np.random.default_rng(21)
prompt = [int(t) for t in rng.integers(0, cfg.n_vocab, 12)]
_ = [int(t) for t in rng.integers(0, cfg.n_vocab, 20)]
claimed = [int(t) for t in rng.integers(0, cfg.n_vocab, 64)]
orc = ggml_cpu.Model(buf, n_ctx=128)
for t in prompt:
    orc.decode_one(t)
refs = [orc.decode_one(t).astype(np.float64) for t in claimed]
alt = ggml_cpu.Model(buf, n_ctx=128)
for t in prompt:
    alt.decode_one(t, alt=True)
for i, t in enumerate(claimed):
    ra = alt.decode_one(t, alt=True).astype(np.float64)
    r = np.abs(ra - refs[i]).max() / np.sqrt(np.mean(refs[i] ** 2))
    if r > 0.05:
        print("cpu reversed-order oracle: row", i, "max/rms", round(float(r), 3), flush=True)
print("oracle done", flush=True)
ctx = engine.Context(m, n_ctx=128)
ctx.decode(prompt)
ctx.decode(claimed, all_logits=True)
bad = []
for i, ref in enumerate(refs):
    g = ctx.logits(row=i).astype(np.float64)
    d = np.abs(g - ref)
    rms = np.sqrt(np.mean(ref ** 2))
    r = d.max() / rms
    if r > 0.12:
        bad.append((i, round(float(r), 3)))
print("mode", os.environ.get("MI_MMQS_MAX"), "rows over 0.12 rms:", bad, flush=True)
