"""Diagnostic: a short verification batch at full width (2-layer 7B) through each batch path --
mmqs (default), mmq2 split-K 4 (MI_MMQS_MAX=0), mmq2 split-K 2 (+ MI_MMQ_KS4=0), per-token decode
(MI_NO_BATCH=1) -- each row's max |dlogit| / rms against the C oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import ggml_cpu  # noqa: E402
from blama_amd import engine, synthetic  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "llama2-7b-q4_k_m"
n_claim = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = synthetic.small_config(name, n_layer=2)
buf = synthetic.build_gguf(cfg, seed=3)
m = engine.Model(buf)
rng = np.random.default_rng(21)
prompt = [int(t) for t in rng.integers(0, cfg.n_vocab, 12)]
claimed = [int(t) for t in rng.integers(0, cfg.n_vocab, n_claim)]
orc = ggml_cpu.Model(buf, n_ctx=128)
orc.decode(prompt)
refs = [orc.decode_one(t).astype(np.float64) for t in claimed]
modes = {"mmqs": {}, "mmq2_ks4": {"MI_MMQS_MAX": "0"}, "mmq2_ks2": {"MI_MMQS_MAX": "0", "MI_MMQ_KS4": "0"},
         "serial": {"MI_NO_BATCH": "1"}}
for mode, env in modes.items():
    for k in ("MI_MMQS_MAX", "MI_MMQ_KS4", "MI_NO_BATCH"):
        os.environ.pop(k, None)
    os.environ.update(env)
    ctx = engine.Context(m, n_ctx=128)
    ctx.decode(prompt)
    ctx.decode(claimed, all_logits=True)
    errs = []
    for i, ref in enumerate(refs):
        rms = float(np.sqrt(np.mean(ref ** 2)))
        errs.append(float(np.max(np.abs(ctx.logits(row=i) - ref))) / rms)
    ctx.close()
    print(f"{mode:9s} max err/rms {max(errs):.3e}  rows: " + " ".join(f"{e:.1e}" for e in errs[:8]), flush=True)
