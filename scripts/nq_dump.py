"""r06: decode logits of the small dense models, dumped for a bit-for-bit comparison between the
step with the normed Q/K/V and gate/up inputs quantised inside their launches and the one with
dv_quant launches (MI_NQ=0, a switch removed once this ran).  argv: output dir, tag."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blama_amd import engine, synthetic  # noqa: E402

out, tag = sys.argv[1], sys.argv[2]
os.makedirs(out, exist_ok=True)
for name in ["tiny-q4_k_m", "tiny-q8_0", "tiny-q6_k", "tiny-gqa16-q4_k_m", "tinyllama-1.1b-q8_0"]:
    cfg = synthetic.CONFIGS[name]
    m = engine.Model(synthetic.build_gguf(cfg, seed=3))
    ctx = engine.Context(m, n_ctx=64)
    ctx.decode([1, 5, 9, 13])
    a = [ctx.logits()]
    for t in [4, 8, 15, 16, 23, 42, 7, 11, 99, 123, 200, 3]:
        ctx.decode([t % cfg.n_vocab])
        a.append(ctx.logits())
    ctx.close()
    np.save(os.path.join(out, f"{name}_{tag}.npy"), np.stack(a))
    print(name, tag, flush=True)
