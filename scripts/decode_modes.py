"""Diagnostic: per-token decode time of the 7B graph (a) with a host synchronisation per step
(the bench's shape: top-k read, sample), (b) with 64 steps queued back to back (no host wait),
(c) as (a) with the stamps build's per-launch timeline length.  Separates GPU-side per-launch
costs from host/idle effects between steps.  Usage: python scripts/decode_modes.py [config]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from blama_amd import engine, synthetic  # noqa: E402

cfg = synthetic.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "llama2-7b-q4_k_m"]
model = engine.Model(synthetic.build_gguf(cfg, seed=0), device=0)
ctx = engine.Context(model, n_ctx=0)
prompt = np.random.default_rng(1234).integers(0, cfg.n_vocab, 32).astype(np.int32)
ctx.decode(prompt)
toks = np.random.default_rng(5).integers(0, cfg.n_vocab, 200).astype(np.int32)
for t in toks[:8]:
    ctx.decode([int(t)])
ctx.synchronize()
n = 64
t0 = time.perf_counter()
for t in toks[8:8 + n]:
    ctx.decode([int(t)])
    ctx.topk(40)
dt_sync = (time.perf_counter() - t0) / n
ctx.synchronize()
t0 = time.perf_counter()
for t in toks[8 + n:8 + 2 * n]:
    ctx.decode([int(t)])
ctx.synchronize()
dt_async = (time.perf_counter() - t0) / n
print(f"per token: synced {dt_sync * 1e3:.3f} ms ({1 / dt_sync:.1f} tok/s)  back-to-back {dt_async * 1e3:.3f} ms "
      f"({1 / dt_async:.1f} tok/s)")
