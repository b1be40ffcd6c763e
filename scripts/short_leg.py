"""One short verification leg on the synthetic Llama-2-7B Q4_K_M (SHORT_CFG: another config) (bench.py's verify_short shape:
a 32-token prompt, then `n` claimed tokens in one MI_OUT_ALL pass), printing progress -- a small
program for counter passes (rocprofv3 --pmc) of the short-batch kernels."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from blama_amd import engine, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cfg = synthetic.CONFIGS[os.environ.get("SHORT_CFG", "llama2-7b-q4_k_m")]
t0 = time.time()
m = engine.Model(synthetic.build_gguf(cfg, seed=1))
print(f"model loaded {time.time() - t0:.1f}s", flush=True)
ctx = engine.Context(m, n_ctx=256)
prompt = np.random.default_rng(4321).integers(0, cfg.n_vocab, 32).astype(np.int32)
claimed = np.random.default_rng(97).integers(0, cfg.n_vocab, n).astype(np.int32)
for r in range(reps):
    ctx.kv_clear()
    ctx.decode(prompt)
    ctx.synchronize()
    t = time.perf_counter()
    ctx.decode(claimed, all_logits=True)
    ctx.synchronize()
    print(f"rep {r}: {n} claimed tokens {1e3 * (time.perf_counter() - t):.3f} ms", flush=True)
