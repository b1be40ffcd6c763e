"""Diagnostic: where a persistent decode step's time goes, per phase of one layer (per-CU
s_memrealtime stamps, 100 MHz).  Usage: python scripts/ps_stamps.py [config] [layer]"""
import sys
import numpy as np
sys.path.insert(0, ".")
from blama_amd import engine, synthetic  # noqa: E402

NAMES = ["layer start", "E_X gathered", "act(attn_norm)", "QKV done", "attention done", "E_ATT act",
         "WO done", "E_XA gathered", "act(ffn_norm)", "GU done", "E_H gathered", "act(h)", "DN done",
         "loader: layer start", "loader: all fills issued", "kernel start"]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "llama2-7b-q4_k_m"
    layer = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    cfg = synthetic.CONFIGS[name]
    model = engine.Model(synthetic.build_gguf(cfg, seed=0))
    ctx = engine.Context(model, n_ctx=512)
    ctx.set_decode_mode(1)
    ctx.decode(np.arange(1, 33, dtype=np.int32))
    ctx.ps_stamps(layer)
    for t in range(8):
        ctx.decode([t + 7])
    st = ctx.ps_stamps(layer, read=True).astype(np.int64)
    ctx.ps_stamps(-1)
    t0 = st[:, 15].min()
    rel = (st - t0) / 100.0   # us
    print(f"{name} layer {layer}: {st.shape[0]} CUs; microseconds from the first kernel start")
    for k in [15, 13, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 14]:
        col = rel[:, k]
        print(f"  {k:2d} {NAMES[k]:26s} min {col.min():8.2f}  med {np.median(col):8.2f}  max {col.max():8.2f}")
    # per-phase durations (per CU), medians
    for a, b in [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 7), (7, 8), (8, 9), (9, 10), (10, 11), (11, 12)]:
        d = (st[:, b] - st[:, a]) / 100.0
        print(f"  {NAMES[a]:>20s} -> {NAMES[b]:22s} med {np.median(d):7.2f}  max {d.max():7.2f}")
    ctx.close()


if __name__ == "__main__":
    main()
