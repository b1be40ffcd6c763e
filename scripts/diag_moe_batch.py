"""Diagnostic (GPU): MoE batch rows vs the per-token decode graphs vs the oracle (tiny-moe)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
from blama_amd import engine, synthetic
from util import oracle_from_gguf

cfg = synthetic.CONFIGS["tiny-moe-q5_k_m"]
buf = synthetic.build_gguf(cfg, seed=31)
m = engine.Model(buf)
rng = np.random.default_rng(9)
prompt = [int(t) for t in rng.integers(0, cfg.n_vocab, 7)]
claimed = [int(t) for t in rng.integers(0, cfg.n_vocab, 40)]
a = engine.Context(m, n_ctx=96)
a.decode(prompt)
a.decode(claimed, all_logits=True)
os.environ["MI_NO_BATCH"] = "1"
b = engine.Context(m, n_ctx=96)
b.decode(prompt)
b.decode(claimed, all_logits=True)
orc = oracle_from_gguf(buf, n_ctx=96)
orc.decode(prompt)
for i, t in enumerate(claimed):
    ref = orc.decode_one(t)
    rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
    la, lb = a.logits(row=i), b.logits(row=i)
    print(i, f"batch-oracle {np.max(np.abs(la - ref)) / rms:.1e}  serial-oracle {np.max(np.abs(lb - ref)) / rms:.1e}  "
          f"batch-serial {np.max(np.abs(la - lb)) / rms:.1e}", flush=True)
