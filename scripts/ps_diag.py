"""Diagnostic: persistent step and launch form each against the numpy oracle, per decode step,
at full 7B width and reduced depth (where does the persistent step diverge)."""
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "oracle")
from blama_amd import engine, synthetic  # noqa: E402
from util import oracle_from_gguf  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "llama2-7b-q4_k_m"
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 1
cfg = synthetic.small_config(name, n_layer=nl)
buf = synthetic.build_gguf(cfg, seed=3)
model = engine.Model(buf)
toks = [int(t) for t in np.random.default_rng(3).integers(0, cfg.n_vocab, 24)]
res = {}
for mode in (1, 0):
    ctx = engine.Context(model, n_ctx=64)
    ctx.set_decode_mode(mode)
    ctx.decode(toks[:2])
    outs = []
    for t in toks[2:]:
        ctx.decode([t])
        outs.append(ctx.logits())
    st = ctx.state_get()
    ctx.close()
    res[mode] = (outs, st)
orc = oracle_from_gguf(buf, n_ctx=64)
orc.decode(toks[:2])
for i, t in enumerate(toks[2:]):
    ref = orc.decode_one(t)
    rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
    e0 = float(np.abs(res[1][0][i] - ref).max()) / rms
    e1 = float(np.abs(res[0][0][i] - ref).max()) / rms
    print(f"step {i} cells {3 + i}: persistent {e0:.2e}  launches {e1:.2e}", flush=True)
a, b = np.frombuffer(res[0][1], np.uint8), np.frombuffer(res[1][1], np.uint8)
print("state bytes", a.size, b.size, "differing", int((a != b).sum()), "first", int(np.argmax(a != b)) if (a != b).any() else -1)
