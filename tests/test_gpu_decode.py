"""End-to-end decode parity: the HIP engine's llama graph vs the CPU
restatement of the ggml CPU path, on synthetic GGUFs with the per-tensor quant
mixes of the BASELINE configs (small shapes so the numpy oracle runs in seconds).

Tolerance: logits within LOGIT_TOL x rms(logits) element-wise, identical top-10
ids, and the reference's own acceptance gate (LogitComparer,
t-LogitComparer.cpp:76-78).  LOGIT_TOL = 2e-3: per-block integer sums and the
attention's f16 rounding of q and of the softmax weights are the CPU's, but the
fp32 accumulation order differs, and a last-bit difference can flip one
activation quantum downstream."""
LOGIT_TOL = 2e-3
import numpy as np
import pytest

import ggml_ref as R
from blama_amd import engine, synthetic
from util import oracle_from_gguf, parse_state

pytestmark = pytest.mark.gpu

CFGS = ["tiny-q4_k_m", "tiny-q5_k_m", "tiny-q6_k", "tiny-q8_0", "tiny-moe-q5_k_m"]


def _run(cfg_name, prompt, steps, n_ctx=64):
    cfg = synthetic.CONFIGS[cfg_name]
    buf = synthetic.build_gguf(cfg, seed=5)
    m = engine.Model(buf)
    ctx = engine.Context(m, n_ctx=n_ctx)
    orc = oracle_from_gguf(buf, n_ctx=n_ctx)
    outs = []
    ctx.decode(prompt)
    ref = orc.decode(prompt)
    outs.append((ctx.logits(), ref, ctx.topk(10)))
    rng = np.random.default_rng(1)
    for _ in range(steps):
        t = int(rng.integers(0, cfg.n_vocab))
        ctx.decode([t])
        ref = orc.decode_one(t)
        outs.append((ctx.logits(), ref, ctx.topk(10)))
    return m, ctx, outs


@pytest.mark.parametrize("cfg_name", CFGS)
def test_decode_matches_oracle(gpu_lib, cfg_name):
    m, ctx, outs = _run(cfg_name, [1, 17, 42, 99, 7], steps=6)
    agg = R.MetricsAggregator()
    sims = []
    for got, ref, (ids, vals) in outs:
        rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
        err = float(np.max(np.abs(got - ref)))
        print(f"{cfg_name}: max|dlogit|/rms = {err / rms:.2e}")
        assert err <= LOGIT_TOL * rms, cfg_name
        top_ref = R.topk(ref, 10)
        assert [int(i) for i in ids] == [i for i, _ in top_ref]
        a = [(int(i), float(v)) for i, v in zip(ids, vals)]
        b = R.gather(ref, [i for i, _ in a])
        cm = R.compare(a, b)
        assert cm.top1Match == 1.0
        score = agg.push_and_verify([cm])
        sims.append(R.logit_similarity(a, b))
    assert score >= 0.95 and np.mean(sims) >= 0.98


def test_topk_gather_consistent_with_logits(gpu_lib):
    m, ctx, outs = _run("tiny-q4_k_m", [1, 2, 3], steps=0)
    lg = ctx.logits()
    ids, vals = ctx.topk(40)
    assert [int(i) for i in ids] == [i for i, _ in R.topk(lg, 40)]
    assert np.array_equal(vals, lg[ids])
    g = ctx.gather(ids[::-1])
    assert np.array_equal(g, lg[ids[::-1]])


def test_decode_bit_deterministic(gpu_lib):
    """Same inputs on two contexts -> bit-identical logits (t-integration.cpp:219-248)."""
    cfg = synthetic.CONFIGS["tiny-q4_k_m"]
    buf = synthetic.build_gguf(cfg, seed=9)
    m = engine.Model(buf)
    res = []
    for _ in range(2):
        ctx = engine.Context(m, n_ctx=32)
        ctx.decode([1, 5, 9, 13])
        a = [ctx.logits()]
        for t in [4, 8, 15, 16, 23, 42]:
            ctx.decode([t])
            a.append(ctx.logits())
        res.append(np.stack(a))
        ctx.close()
    assert np.array_equal(res[0].view(np.uint32), res[1].view(np.uint32))


def test_kv_full_returns_1(gpu_lib):
    cfg = synthetic.CONFIGS["tiny-q8_0"]
    m = engine.Model(synthetic.build_gguf(cfg))
    ctx = engine.Context(m, n_ctx=8)
    assert ctx.decode(list(range(1, 9))) == 0
    assert ctx.decode([3]) == 1          # llama_decode: 1 = no KV slot
    ctx.kv_clear()
    assert ctx.decode([3]) == 0 and ctx.pos_max == 0


def test_state_roundtrip(gpu_lib):
    """getState/setState reproduce generation (t-integration.cpp:304-421)."""
    cfg = synthetic.CONFIGS["tiny-q6_k"]
    m = engine.Model(synthetic.build_gguf(cfg))
    a = engine.Context(m, n_ctx=32)
    a.decode([1, 2, 3, 4])
    st = a.state_get()
    a.decode([5])
    la = a.logits()
    b = engine.Context(m, n_ctx=32)
    b.state_set(st)
    assert b.pos_max == 3 and b.n_cells == 4
    b.decode([5])
    assert np.array_equal(la.view(np.uint32), b.logits().view(np.uint32))


@pytest.mark.parametrize("cfg_name", ["tiny-q4_k_m", "tiny-q6_k"])
def test_context_shift_matches_oracle(gpu_lib, cfg_name):
    """Context shift (Session.cpp:324-347): seq_rm [keep, keep+discard) then
    seq_add(keep+discard, n_past, -discard) with the K-shift re-rotation, on the
    engine and on the oracle's restatement of the same cell operations."""
    buf = synthetic.build_gguf(synthetic.CONFIGS[cfg_name], seed=2)
    m = engine.Model(buf)
    toks = [1, 11, 22, 33, 44, 55, 66, 77]
    keep, discard = 2, 3
    a = engine.Context(m, n_ctx=32)
    o = oracle_from_gguf(buf, n_ctx=32)
    a.decode(toks)
    o.decode(toks)
    a.kv_seq_rm(keep, keep + discard)
    o.kv_seq_rm(keep, keep + discard)
    a.kv_seq_add(keep + discard, len(toks), -discard)
    o.kv_seq_shift(keep + discard, len(toks), delta=-discard)
    assert a.pos_max == len(toks) - discard - 1 and a.n_cells == len(toks) - discard
    for t in [5, 6]:
        a.decode([t])
        ref = o.decode_one(t)
        got = a.logits()
        rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
        assert np.max(np.abs(got - ref)) <= LOGIT_TOL * rms


def _kshift_ref(k16, deltas, hp):
    """The K-shift applied to a cache snapshot: f16(rope(f32(K), delta)) per cell."""
    out = k16.copy()
    for c, d in enumerate(deltas):
        if d:
            for il in range(k16.shape[0]):
                k = k16[il, c].astype(np.float32).reshape(hp.n_head_kv, hp.head_dim)
                out[il, c] = R.f32_to_f16(R.rope_norm(k, d, hp.n_rot, hp.rope_base).reshape(-1))
    return out


def test_self_extend_div_matches_oracle(gpu_lib):
    """Self-Extend group attention (Session.cpp:348-368): seq_add + seq_div + seq_add.
    (1) the K-shift kernel equals the restatement applied to the engine's own
    pre-shift cache (<= 1 fp16 ulp: cosf/sinf may differ by an ulp); (2) the next
    token's logits agree with the oracle doing the same cell operations."""
    buf = synthetic.build_gguf(synthetic.CONFIGS["tiny-q4_k_m"], seed=4)
    m = engine.Model(buf)
    toks = list(range(3, 15))
    a = engine.Context(m, n_ctx=32)
    o = oracle_from_gguf(buf, n_ctx=32)
    hp = o.hp
    kvd = hp.n_head_kv * hp.head_dim
    a.decode(toks)
    o.decode(toks)
    _, k_before, v_before = parse_state(a.state_get(), hp.n_layer, kvd)
    # ga_n = 2, ga_w = 8: ib = 0, bd = 4, dd = -4
    a.kv_seq_add(0, 12, 0)
    a.kv_seq_div(0, 8, 2)
    a.kv_seq_add(8, 12, -4)
    o.kv_seq_shift(0, 8, div=2)
    o.kv_seq_shift(8, 12, delta=-4)
    pos, k_after, v_after = parse_state(a.state_get(), hp.n_layer, kvd)
    assert list(pos) == o.cell_pos and a.pos_max == max(o.cell_pos)
    deltas = [p // 2 - p for p in range(8)] + [-4] * 4
    ref = _kshift_ref(k_before, deltas, hp)
    ulp = np.abs(k_after.view(np.int16).astype(np.int32) - ref.view(np.int16).astype(np.int32))
    assert ulp.max() <= 1
    assert np.array_equal(v_after, v_before)
    a.decode([40])
    ref = o.decode_one(40)
    got = a.logits()
    rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
    assert np.max(np.abs(got - ref)) <= 5e-2 * rms
    assert int(np.argmax(got)) == int(np.argmax(ref))


def test_split_attention_beyond_short_context(gpu_lib):
    """Contexts past ATTN_SHORT (512) cells switch from the fused single-launch attention to the
    split two-launch one (a different decode graph); both must match the oracle, including the
    steps that cross the threshold."""
    cfg = synthetic.CONFIGS["tiny-q4_k_m"]
    buf = synthetic.build_gguf(cfg, seed=3)
    m = engine.Model(buf)
    ctx = engine.Context(m, n_ctx=576)
    orc = oracle_from_gguf(buf, n_ctx=576)
    rng = np.random.default_rng(21)
    prompt = [int(t) for t in rng.integers(0, cfg.n_vocab, 509)]
    ctx.decode(prompt)
    orc.decode(prompt)
    for t in [int(v) for v in rng.integers(0, cfg.n_vocab, 6)]:   # cells 510 .. 515
        ctx.decode([t])
        ref = orc.decode_one(t)
        got = ctx.logits()
        rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
        assert np.max(np.abs(got - ref)) <= LOGIT_TOL * rms, ctx.n_cells
        ids, _ = ctx.topk(10)
        assert [int(i) for i in ids] == [i for i, _ in R.topk(ref, 10)]


def _logits_close(got, ref, tol=LOGIT_TOL):
    rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
    return float(np.max(np.abs(got - ref))) <= tol * rms


def test_batched_prompt_matches_token_by_token(gpu_lib, monkeypatch):
    """Prompt ingestion through the batched GEMMs (int8-MFMA: chunks of 16 tokens, 16+4;
    v_dot4 with MI_NO_MMQ=1: chunks of 8, 8+8+4) against the same prompt decoded token by
    token (MI_NO_BATCH=1) and against the oracle:
    the per-token integer arithmetic is the same, only fp32 sum orders differ."""
    cfg = synthetic.CONFIGS["tiny-q4_k_m"]
    buf = synthetic.build_gguf(cfg, seed=13)
    m = engine.Model(buf)
    prompt = [int(t) for t in np.random.default_rng(5).integers(0, cfg.n_vocab, 20)]
    a = engine.Context(m, n_ctx=64)
    a.decode(prompt)
    monkeypatch.setenv("MI_NO_MMQ", "1")          # the v_dot4 GEMM instead of the int8-MFMA one
    c = engine.Context(m, n_ctx=64)
    c.decode(prompt)
    monkeypatch.setenv("MI_NO_BATCH", "1")
    b = engine.Context(m, n_ctx=64)
    b.decode(prompt)
    ref = oracle_from_gguf(buf, n_ctx=64).decode(prompt)
    la, lb = a.logits(), b.logits()
    assert _logits_close(la, ref) and _logits_close(lb, ref) and _logits_close(c.logits(), ref)
    assert [int(i) for i in a.topk(10)[0]] == [i for i, _ in R.topk(ref, 10)]
    # the caches the batch wrote serve the following single-token steps
    for t in [3, 4]:
        a.decode([t])
        b.decode([t])
        assert _logits_close(a.logits(), b.logits())


@pytest.mark.parametrize("cfg_name", ["tiny-q6_k", "tiny-q8_0"])
def test_batched_prompt_other_quant_types(gpu_lib, cfg_name):
    cfg = synthetic.CONFIGS[cfg_name]
    buf = synthetic.build_gguf(cfg, seed=17)
    m = engine.Model(buf)
    prompt = [int(t) for t in np.random.default_rng(6).integers(0, cfg.n_vocab, 11)]
    a = engine.Context(m, n_ctx=32)
    a.decode(prompt)
    ref = oracle_from_gguf(buf, n_ctx=32).decode(prompt)
    assert _logits_close(a.logits(), ref)
    assert [int(i) for i in a.topk(10)[0]] == [i for i, _ in R.topk(ref, 10)]


def test_prefill_512_tokens_matches_oracle(gpu_lib):
    """The 512-token prefill config (BASELINE configs[2]) at small shapes: 64 chunks of 8,
    causal attention up to 512 cells, logits of the last token."""
    cfg = synthetic.CONFIGS["tiny1-q4_k_m"]
    buf = synthetic.build_gguf(cfg, seed=19)
    m = engine.Model(buf)
    prompt = [int(t) for t in np.random.default_rng(7).integers(0, cfg.n_vocab, 512)]
    a = engine.Context(m, n_ctx=520)
    a.decode(prompt)
    ref = oracle_from_gguf(buf, n_ctx=520).decode(prompt)
    assert _logits_close(a.logits(), ref)
    assert [int(i) for i in a.topk(10)[0]] == [i for i, _ in R.topk(ref, 10)]


def test_gqa16_layout_decode_and_short_batch(gpu_lib):
    """32 q heads over 16 kv heads of 64: decode against the oracle, and a short
    verification batch (MI_OUT_ALL, the split-K streaming GEMMs) row by row against the same
    tokens decoded one at a time."""
    cfg = synthetic.CONFIGS["tiny-gqa16-q4_k_m"]
    buf = synthetic.build_gguf(cfg, seed=12)
    m = engine.Model(buf)
    a = engine.Context(m, n_ctx=64)
    b = engine.Context(m, n_ctx=64)
    orc = oracle_from_gguf(buf, n_ctx=64)
    try:
        prompt = [3, 77, 120, 9]
        assert a.decode(prompt) == 0
        ref = orc.decode(prompt)
        assert _logits_close(a.logits(), ref)
        for t in [5, 300, 41]:
            a.decode([t])
            ref = orc.decode_one(t)
            assert _logits_close(a.logits(), ref), t
            assert [int(i) for i in a.topk(10)[0]] == [i for i, _ in R.topk(ref, 10)]
        claimed = [int(t) for t in np.random.default_rng(3).integers(0, cfg.n_vocab, 20)]
        assert b.decode(prompt + [5, 300, 41]) == 0
        assert b.decode(claimed, all_logits=True) == 0
        # the batch's GEMMs sum in another fp32 order, which can flip a Q8_K rounding of a later
        # activation (test_gpu_fullwidth.py's docstring): rows within 2e-2 rms of the per-token
        # path, the same top-1 unless the two ids are within twice the row's largest difference
        for i, t in enumerate(claimed):
            a.decode([t])
            x, y = b.logits(row=i).astype(np.float64), a.logits().astype(np.float64)
            d = float(np.max(np.abs(x - y)))
            assert d <= 2e-2 * float(np.sqrt(np.mean(y ** 2))), (i, d)
            ix, iy = int(np.argmax(x)), int(np.argmax(y))
            assert ix == iy or y[iy] - y[ix] <= 2 * d, (i, ix, iy)
    finally:
        a.close()
        b.close()
        m.close()
