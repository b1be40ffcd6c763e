"""Diagnostic (not a test): the persistent decode step (mode 0) against the launch form (mode 1)
on the same model and tokens -- logits of every step, and the decode rate of both.
Usage: python scripts/ps_check.py [config ...] [--steps N]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from blama_amd import engine, synthetic  # noqa: E402


def run(model, cfg, mode, steps, timed, nprompt=8, nobs=12):
    ctx = engine.Context(model, n_ctx=512)
    ctx.set_decode_mode(mode)
    rng = np.random.default_rng(5)
    prompt = rng.integers(0, cfg.n_vocab, nprompt).astype(np.int32)
    ctx.decode(prompt)
    toks = rng.integers(0, cfg.n_vocab, steps).astype(np.int32)
    path = (ctx.decode_path(), ctx.decode_path_note())
    outs = []
    for t in toks[:nobs]:
        ctx.decode([int(t)])
        outs.append(ctx.logits())
    rate = None
    if timed:
        ctx.synchronize()
        t0 = time.perf_counter()
        for t in toks[nobs:]:
            ctx.decode([int(t)])
        ctx.synchronize()
        rate = (len(toks) - nobs) / (time.perf_counter() - t0)
    ctx.close()
    return np.array(outs), path, rate


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = 140
    for a in sys.argv[1:]:
        if a.startswith("--steps="):
            steps = int(a.split("=")[1])
    for name in args or ["tiny-q4_k_m"]:
        cfg = synthetic.CONFIGS[name]
        model = engine.Model(synthetic.build_gguf(cfg, seed=0))
        timed = cfg.n_embd >= 2048
        nprompt = int(next((x.split("=")[1] for x in sys.argv if x.startswith("--prompt=")), 8))
        nobs = int(next((x.split("=")[1] for x in sys.argv if x.startswith("--obs=")), 12))
        a, pa, ra = run(model, cfg, 1, steps, timed, nprompt, nobs)
        b, pb, rb = run(model, cfg, 0, steps, timed, nprompt, nobs)
        rms = float(np.sqrt(np.mean(b.astype(np.float64) ** 2)))
        err = np.abs(a - b).max(axis=1) / rms
        top_eq = [int(np.argmax(x) == np.argmax(y)) for x, y in zip(a, b)]
        print(f"{name} prompt {nprompt}: path persistent={pa} launches={pb}; max|d|/rms per step {np.round(err, 6).tolist()}; "
              f"top1 equal {sum(top_eq)}/{len(top_eq)}; tok/s persistent {ra} launches {rb}", flush=True)
        model.close()


if __name__ == "__main__":
    main()
