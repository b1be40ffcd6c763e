"""Diagnostic: per-launch timeline of one decode step from in-kernel stamps.

Runs the diagnostic build (libmi_engine_stamps.so, `make -C blama_amd/csrc
stamps`) on the bench's synthetic model, decodes a prompt plus a few steps
through the normal graph path, then reads the per-workgroup s_memrealtime
stamps (100 MHz) of the last step and prints, per launch, relative to the
first workgroup entry of the step:
  entry min / median, prologue-done median (GEMV stamp 2), end median / max,
the gap from the previous launch's last workgroup end to this launch's first
entry, and the launch's span (first entry -> last end).
Usage: MI_ENGINE_LIB=stamps python scripts/timeline.py [config] [n_past]
"""
import os
import sys

import numpy as np

os.environ.setdefault("MI_ENGINE_LIB", "stamps")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from blama_amd import engine, synthetic  # noqa: E402


def main():
    cfg = synthetic.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "llama2-7b-q4_k_m"]
    n_past = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    model = engine.Model(synthetic.build_gguf(cfg, seed=0), device=0)
    ctx = engine.Context(model, n_ctx=0)
    prompt = np.random.default_rng(1234).integers(0, cfg.n_vocab, 32).astype(np.int32)
    ctx.decode(prompt)
    for i in range(max(0, n_past - 32)):
        ctx.decode([int(prompt[i % 32])])
    ctx.synchronize()
    NL = 320
    buf = np.zeros((NL, 512, 8), np.uint64)
    n = engine.lib().mi_debug_stamps(ctx.h, buf.ctypes.data, NL)
    if n <= 0:
        raise SystemExit("not the diagnostic build (mi_debug_stamps returned 0)")
    launches = []
    for i in range(n):
        ent = buf[i, :, 0].astype(np.int64)
        m = ent > 0
        if not m.any():
            continue   # an unused slab (e.g. the second attention launch in fused mode)
        end = buf[i, :, 4].astype(np.int64)
        end5 = buf[i, :, 5].astype(np.int64)   # GEMV: last wave of the workgroup (atomic max)
        if (end5 > 0).any():
            end = np.where(end5 > 0, end5, end)
        pro = buf[i, :, 2].astype(np.int64)
        pre = buf[i, :, 1].astype(np.int64)
        launches.append((ent[m], end[m & (end > 0)], pro[m & (pro > 0)], pre[m & (pre > 0)]))
    t0 = launches[0][0].min()
    prev_end = None
    rows = []
    print(f"{'#':>3} {'wgs':>4} {'entry_min':>9} {'entry_med':>9} {'pre_med':>8} {'pro_med':>8} {'end_med':>8} {'end_max':>8}"
          f" {'gap':>6} {'span':>6}")
    for i, (ent, end, pro, pre) in enumerate(launches):
        us = lambda v: (v - t0) / 100.0  # noqa: E731
        e0, em = us(ent.min()), us(np.median(ent))
        pm = us(np.median(pro)) if len(pro) else float("nan")
        qm = us(np.median(pre)) if len(pre) else float("nan")
        dm, dx = us(np.median(end)), us(end.max())
        gap = e0 - prev_end if prev_end is not None else 0.0
        prev_end = dx
        rows.append((dx - e0, gap))
        print(f"{i:3d} {len(ent):4d} {e0:9.2f} {em:9.2f} {qm:8.2f} {pm:8.2f} {dm:8.2f} {dx:8.2f} {gap:6.2f} {dx - e0:6.2f}")
    spans = np.array([r[0] for r in rows])
    gaps = np.array([r[1] for r in rows])
    total = (launches[-1][1].max() - t0) / 100.0
    # prologue detail of the roofline-sized launches (GEMV stamps 5/6/7: before / after
    # the RMSNorm barrier, end of the prologue before its final barrier), wave 0 medians
    for i, (ent, end, pro, pre) in enumerate(launches):
        if i < len(launches) - 12:
            continue
        d = buf[i, :, :].astype(np.int64)
        m = d[:, 0] > 0
        det = []
        for k in (1, 7, 3, 2, 4):
            v = d[m, k]
            v = v[v > 0]
            det.append(f"{(np.median(v) - np.median(d[m, 0])) / 100.0:6.2f}" if len(v) else "   -  ")
        # gemv_k stamps (wave 0): 1 ring issued, 7 activation slice quantised, 3 first ring
        # round consumed (first weights landed), 2 stream done + barrier, 4 epilogue done
        print(f"{i:3d} from params-in-LDS: issued {det[0]}  act-quantised {det[1]}  first-weights {det[2]}"
              f"  stream-done {det[3]}  epilogue-done {det[4]}")
    # GEMV workgroup skew (stamps 6, 7: last wave started / last wave's activation landed, atomic
    # max over the waves), medians over workgroups, relative to wave 0's entry
    for i in range(n):
        d = buf[i, :, :].astype(np.int64)
        m = (d[:, 0] > 0) & (d[:, 6] > 0)
        if not m.any():
            continue
        e0 = d[m, 0]
        s6 = np.median(d[m, 6] - e0) / 100.0
        s7 = np.median(d[m, 7] - e0) / 100.0 if (d[m, 7] > 0).any() else float("nan")
        s2 = np.median(d[m, 2] - e0) / 100.0
        s5 = np.median(d[m, 5] - e0) / 100.0 if (d[m, 5] > 0).any() else float("nan")
        if i < 12:
            print(f"  launch {i:3d}: last wave started +{s6:5.2f}  last activation landed +{s7:5.2f}  "
                  f"activation in LDS +{s2:5.2f}  last wave done +{s5:5.2f} us")
    print(f"launches {len(rows)}  first entry -> last end {total:.1f} us;  sum of spans {spans.sum():.1f}"
          f"  sum of gaps {gaps.sum():.1f}")


if __name__ == "__main__":
    main()
