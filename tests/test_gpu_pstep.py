"""The persistent decode step (blama_amd/csrc/pstep.hip) against the launch form of the same step
(dgemv.hip; mi_decode_set_mode(ctx, 0), the default) and against the CPU oracle.

Both forms run the same per-superblock integer dots (Kq<T>::dot, same lane order and wave sum) and
the same Q8_K quantisation rules; they differ in the fp32 / double order of the RMSNorm sum of
squares and of the attention's softmax sum and PV partials.  Bar: logits within 1e-4 x rms of each
other (orders of magnitude under the oracle bar LOGIT_TOL = 2e-3 x rms of test_gpu_decode.py) and
identical top-10, at tiny and at full Llama-2-7B / Llama-3-8B widths (reduced depth)."""
import numpy as np
import pytest

import ggml_ref as R
from blama_amd import engine, synthetic
from util import oracle_from_gguf

pytestmark = pytest.mark.gpu

PAIR_TOL = 1e-4
LOGIT_TOL = 2e-3


def _decode(model, cfg, mode, prompt, toks, n_ctx=256):
    ctx = engine.Context(model, n_ctx=n_ctx)
    ctx.set_decode_mode(mode)
    ctx.decode(prompt)
    outs, paths = [], []
    for t in toks:
        paths.append(ctx.decode_path())
        ctx.decode([int(t)])
        outs.append((ctx.logits(), ctx.topk(10)))
    note = ctx.decode_path_note()
    ctx.close()
    return outs, paths, note


def _pair(name, n_layer=None, steps=8, seed=3):
    cfg = synthetic.CONFIGS[name]
    if n_layer:
        cfg = synthetic.small_config(name, n_layer=n_layer)
    buf = synthetic.build_gguf(cfg, seed=seed)
    model = engine.Model(buf)
    rng = np.random.default_rng(seed)
    prompt = rng.integers(0, cfg.n_vocab, 6).astype(np.int32)
    toks = rng.integers(0, cfg.n_vocab, steps).astype(np.int32)
    ps, pp, note = _decode(model, cfg, 1, prompt, toks)
    ls, lp, _ = _decode(model, cfg, 0, prompt, toks)
    model.close()
    assert all(p == 2 for p in pp), f"{name}: the persistent step did not run ({note!r})"
    assert all(p == 1 for p in lp)
    for i, ((a, (ia, _)), (b, (ib, _))) in enumerate(zip(ps, ls)):
        rms = float(np.sqrt(np.mean(b.astype(np.float64) ** 2)))
        err = float(np.max(np.abs(a - b)))
        print(f"{name} step {i}: persistent vs launches max|d|/rms {err / rms:.2e}")
        assert err <= PAIR_TOL * rms, (name, i)
        assert list(ia) == list(ib), (name, i)
    return buf, prompt, toks, ps


@pytest.mark.parametrize("name", ["tiny-q4_k_m", "tiny-q5_k_m", "tiny-q6_k", "tiny1-q4_k_m"])
def test_persistent_matches_launch_form_tiny(gpu_lib, name):
    buf, prompt, toks, ps = _pair(name, steps=10)
    # and the oracle, under the decode tests' bar
    orc = oracle_from_gguf(buf, n_ctx=256)
    orc.decode([int(t) for t in prompt])
    for (got, (ids, _)), t in zip(ps, toks):
        ref = orc.decode_one(int(t))
        rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
        assert float(np.max(np.abs(got - ref))) <= LOGIT_TOL * rms
        assert [int(i) for i in ids] == [i for i, _ in R.topk(ref, 10)]


@pytest.mark.parametrize("name", ["llama2-7b-q4_k_m", "llama3-8b-q6_k"])
def test_persistent_matches_launch_form_full_width(gpu_lib, name):
    _pair(name, n_layer=2, steps=6)


def test_persistent_step_is_bit_deterministic(gpu_lib):
    cfg = synthetic.CONFIGS["tiny-q4_k_m"]
    buf = synthetic.build_gguf(cfg, seed=9)
    model = engine.Model(buf)
    toks = np.arange(1, 13, dtype=np.int32)
    a, pa, _ = _decode(model, cfg, 1, [3, 4, 5], toks)
    b, pb, _ = _decode(model, cfg, 1, [3, 4, 5], toks)
    model.close()
    assert all(p == 2 for p in pa + pb)
    for (x, _), (y, _) in zip(a, b):
        assert np.array_equal(x, y)


def test_second_context_falls_back_to_launches(gpu_lib):
    """The persistent launch needs every CU: with two live contexts on the device, steps take the
    launch form (the server's replicas may decode concurrently)."""
    cfg = synthetic.CONFIGS["tiny-q4_k_m"]
    model = engine.Model(synthetic.build_gguf(cfg, seed=2))
    c1 = engine.Context(model, n_ctx=64)
    c1.set_decode_mode(1)
    c1.decode([1, 2])
    assert c1.decode_path() == 2
    c2 = engine.Context(model, n_ctx=64)
    c2.set_decode_mode(1)
    assert c1.decode_path() == 1 and c2.decode_path() == 1
    assert "other contexts" in c1.decode_path_note()
    c1.decode([5])
    c2.decode([1, 2])
    c2.decode([5])
    assert np.array_equal(c1.logits(), c2.logits())   # both on the launch form
    c2.close()
    assert c1.decode_path() == 2
    c1.close()
    model.close()
