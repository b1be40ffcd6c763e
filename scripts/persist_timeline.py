"""Diagnostic (GPU): per-stage timeline of the persistent decode step from its s_memrealtime stamps
(MI_PERSIST_STAMPS=1).  Prints, for each stage of the last step, the median over workgroups of
the prefill time (entry -> barrier start), the barrier wait, and the work after the barrier, plus
the stage's span and its algorithmic bytes rate, then totals per stage kind.
Usage: MI_PERSIST_STAMPS=1 python scripts/persist_timeline.py [config] [n_ctx_cells]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MI_PERSIST_STAMPS", "1")
os.environ.setdefault("MI_PERSIST", "1")
from blama_amd import engine, synthetic  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "llama2-7b-q4_k_m"
cells = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cfg = synthetic.CONFIGS[name]
m = engine.Model(synthetic.build_gguf(cfg, seed=0))
ctx = engine.Context(m, n_ctx=0)
ctx.decode(list(np.random.default_rng(1).integers(0, cfg.n_vocab, cells)))
for t in range(8):
    ctx.decode([t + 5])
ctx.topk(10)
ns = ctx.persist_stages
grid = 256
st = ctx.persist_stamps(ns, grid).astype(np.int64)
print(f"{name}: {ns} stages, n_cells {ctx.n_cells}")
kinds = []
per_layer = (ns - 1) // cfg.n_layer
names = {5: ["qkv", "attn", "wo", "gateup", "down"], 6: ["qkv", "qkv2", "attn", "wo", "gateup", "down"]}
t0 = st[0, :, 0][st[0, :, 0] > 0].min()
tot = {}
last_end = t0
for s in range(ns):
    e = st[s]
    act = e[:, 3] > 0
    ent, b0, b1, pro = (e[act, k] for k in range(4))
    nxt = st[s + 1][act, 0] if s + 1 < ns else pro
    end = np.maximum(nxt, pro)
    lay = s // per_layer if s < ns - 1 else -1
    kind = "output" if s == ns - 1 else names.get(per_layer, ["?"] * per_layer)[s % per_layer] if per_layer in names else "?"
    span_end = end.max()
    pre = np.median(b0 - ent) / 100
    bar = np.median(b1 - b0) / 100
    work = np.median(end - b1) / 100
    prol = np.median(pro - b1) / 100
    stage_us = (span_end - last_end) / 100
    last_end = span_end
    d = tot.setdefault(kind, [0, 0.0, 0.0, 0.0, 0.0, 0.0])
    d[5] += prol
    d[0] += 1
    d[1] += stage_us
    d[2] += pre
    d[3] += bar
    d[4] += work
    if lay in (0, 1, cfg.n_layer - 1) or s == ns - 1:
        print(f"stage {s:3d} L{lay:2d} {kind:7s} wgs {act.sum():3d}: end-to-end {stage_us:6.2f} us | "
              f"median prefill {pre:5.2f} barrier {bar:5.2f} prologue {prol:5.2f} work {work:6.2f} | "
              f"barrier exit spread {(b1.max() - b1.min()) / 100:5.2f} us, last arrival wg {int(np.argmax(e[:, 1]))}")
print(f"whole launch: {(last_end - t0) / 100:.1f} us")
for k, (n, us, pre, bar, work, prol) in tot.items():
    print(f"{k:7s} x{n:3d}: {us:8.1f} us total ({us / n:6.2f}/stage) median prefill {pre / n:5.2f} barrier {bar / n:5.2f} "
          f"prologue {prol / n:5.2f} work {work / n:6.2f}")

# straggler analysis: work after the barrier (stage end - barrier end) per workgroup
print("\nwork after the barrier per workgroup (us): p10 / p50 / p90 / max, slowest workgroups (wg %8 = XCD)")
for s in range(5 * 4, 5 * 4 + per_layer):
    e = st[s]
    act = e[:, 3] > 0
    w = (st[s + 1][act, 0] - e[act, 2]) / 100
    ids = np.nonzero(act)[0]
    slow = ids[np.argsort(w)[-6:]]
    print(f"stage {s} {names.get(per_layer, ['?'] * per_layer)[s % per_layer]:7s}: {np.percentile(w, 10):5.2f} {np.percentile(w, 50):5.2f} "
          f"{np.percentile(w, 90):5.2f} {w.max():5.2f}  slowest {list(slow)} xcd {[int(x) % 8 for x in slow]}")
    xcd = [float(np.mean(w[(ids % 8) == k])) for k in range(8)]
    print("   mean by XCD:", " ".join(f"{v:5.2f}" for v in xcd))
