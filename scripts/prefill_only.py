"""r06 diagnostic: the bench's 512-token 7B prefill leg alone, 3 times (for an eager kernel trace)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blama_amd import engine, synthetic  # noqa: E402

cfg = synthetic.CONFIGS["llama2-7b-q4_k_m"]
model = engine.Model(synthetic.build_gguf(cfg, seed=0), device=0)
ctx = engine.Context(model, n_ctx=0)
toks = np.random.default_rng(4321).integers(0, cfg.n_vocab, 512).astype(np.int32)
for i in range(3):
    ctx.kv_clear()
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.decode(toks)
    ctx.synchronize()
    print(f"prefill {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
ctx.close()
model.close()
