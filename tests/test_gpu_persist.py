"""The persistent decode step (gemv.hip decode_step_kernel): the layers and the output head of a
batch-1 llama_decode as ONE launch of one 16-wave workgroup per CU, stages separated by grid
barriers (SURVEY.md §8a rows a3-a14 on one launch).

Checked: the step is taken (mi_persist_stages > 0) for every compiled type class; its logits
against the CPU oracle (LOGIT_TOL x rms, identical top-10, the reference gate); against the
per-op hipGraph path of the same model (the default: the same GEMV arithmetic and work
partition, only the attention's cell reduction spread over 16 waves instead of 4); bit-exact
determinism across contexts (t-integration.cpp:219-248); contexts of one device interleaving
their persistent steps; and the hand-over to the graph path past 512 cells."""
import numpy as np
import pytest

import ggml_ref as R
from blama_amd import engine, synthetic
from util import oracle_from_gguf, parse_state

pytestmark = pytest.mark.gpu
LOGIT_TOL = 2e-3


@pytest.fixture(autouse=True)
def _persist(monkeypatch):
    """The persistent step is opt-in (MI_PERSIST=1, read when a context is created)."""
    monkeypatch.setenv("MI_PERSIST", "1")

# model -> the compiled class its matrices fall in
CLASSES = ["tiny-q4_k_m", "tiny-q5_k_m", "tiny-q6_k", "tiny-q8_0"]


def _rms(a):
    return float(np.sqrt(np.mean(a.astype(np.float64) ** 2)))


@pytest.mark.parametrize("name", CLASSES)
def test_persistent_step_matches_oracle(gpu_lib, name):
    cfg = synthetic.CONFIGS[name]
    buf = synthetic.build_gguf(cfg, seed=51)
    m = engine.Model(buf)
    ctx = engine.Context(m, n_ctx=96)
    orc = oracle_from_gguf(buf, n_ctx=96)
    rng = np.random.default_rng(3)
    prompt = [int(t) for t in rng.integers(0, cfg.n_vocab, 9)]
    ctx.decode(prompt)
    ref = orc.decode(prompt)
    agg = R.MetricsAggregator()
    for s in range(8):
        t = int(rng.integers(0, cfg.n_vocab))
        ctx.decode([t])
        ref = orc.decode_one(t)
        got = ctx.logits()
        assert ctx.persist_stages > 0, "the decode step did not run as the persistent launch"
        err = float(np.max(np.abs(got - ref)))
        assert err <= LOGIT_TOL * _rms(ref), (s, err / _rms(ref))
        ids, vals = ctx.topk(10)
        assert [int(i) for i in ids] == [i for i, _ in R.topk(ref, 10)], s
        a = [(int(i), float(v)) for i, v in zip(ids, vals)]
        cm = R.compare(a, R.gather(ref, [i for i, _ in a]))
        assert cm.top1Match == 1.0
        score = agg.push_and_verify([cm])
    assert score >= 0.95
    # stages: per layer 1-2 QKV launches, attention, WO, gate/up, down; then the output head
    assert cfg.n_layer * 5 + 1 <= ctx.persist_stages <= cfg.n_layer * 6 + 1


@pytest.mark.parametrize("name", ["tiny-q4_k_m", "tiny-q8_0"])
def test_persistent_step_matches_graph_path(gpu_lib, monkeypatch, name):
    cfg = synthetic.CONFIGS[name]
    m = engine.Model(synthetic.build_gguf(cfg, seed=52))
    a = engine.Context(m, n_ctx=64)
    a.decode([1])
    assert a.persist_stages > 0
    monkeypatch.delenv("MI_PERSIST")
    b = engine.Context(m, n_ctx=64)
    b.decode([1])
    assert b.persist_stages == 0
    rng = np.random.default_rng(4)
    for t in [int(x) for x in rng.integers(0, cfg.n_vocab, 20)]:
        a.decode([t])
        b.decode([t])
        la, lb = a.logits(), b.logits()
        assert float(np.max(np.abs(la - lb))) <= 1e-4 * _rms(lb)
        assert np.array_equal(a.topk(10)[0], b.topk(10)[0])
    # the KV cache rows the two paths appended agree to f16 rounding
    kv_dim = cfg.n_embd // cfg.n_head * cfg.n_head_kv
    pa, ka, va = parse_state(a.state_get(), cfg.n_layer, kv_dim)
    pb, kb, vb = parse_state(b.state_get(), cfg.n_layer, kv_dim)
    assert np.array_equal(pa, pb)
    for x, y in ((ka, kb), (va, vb)):
        x, y = x.astype(np.float32), y.astype(np.float32)
        assert np.max(np.abs(x - y)) <= 2e-3 * max(1.0, float(np.max(np.abs(y))))


def test_persistent_step_bit_deterministic(gpu_lib):
    cfg = synthetic.CONFIGS["tiny-q4_k_m"]
    m = engine.Model(synthetic.build_gguf(cfg, seed=53))
    out = []
    for _ in range(2):
        ctx = engine.Context(m, n_ctx=48)
        ctx.decode([5, 6, 7])
        rows = []
        for t in [11, 12, 13, 14, 15]:
            ctx.decode([t])
            rows.append(ctx.logits())
        assert ctx.persist_stages > 0
        out.append(np.stack(rows))
        ctx.close()
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))


def test_persistent_contexts_interleave_on_one_device(gpu_lib):
    """Three contexts on one device enqueue persistent steps back to back without waiting on
    each other: the engine chains them on the device (two grids of one workgroup per CU at once
    would not be co-resident), and each matches a context decoding alone."""
    cfg = synthetic.CONFIGS["tiny-q6_k"]
    m = engine.Model(synthetic.build_gguf(cfg, seed=54))
    seqs = [[int(t) for t in np.random.default_rng(10 + i).integers(0, cfg.n_vocab, 12)] for i in range(3)]
    solo = []
    for sq in seqs:
        c = engine.Context(m, n_ctx=32)
        for t in sq:
            c.decode([t])
        solo.append(c.logits())
        c.close()
    ctxs = [engine.Context(m, n_ctx=32) for _ in seqs]
    for i in range(len(seqs[0])):
        for c, sq in zip(ctxs, seqs):
            c.decode([sq[i]])   # no readback in between: the three streams run concurrently
    for c, ref in zip(ctxs, solo):
        assert c.persist_stages > 0
        assert np.array_equal(c.logits().view(np.uint32), ref.view(np.uint32))


def test_persistent_hands_over_past_512_cells(gpu_lib):
    """Past ATTN_SHORT cells the step takes the split-attention graph; the persistent and graph
    steps share the cache."""
    cfg = synthetic.CONFIGS["tiny-q4_k_m"]
    buf = synthetic.build_gguf(cfg, seed=55)
    m = engine.Model(buf)
    ctx = engine.Context(m, n_ctx=600)
    orc = oracle_from_gguf(buf, n_ctx=600)
    prompt = [int(t) for t in np.random.default_rng(6).integers(0, cfg.n_vocab, 505)]
    ctx.decode(prompt)
    orc.decode(prompt)
    for t in range(20, 32):   # cells 505 .. 516: persistent up to 512, the graph after
        ctx.decode([t])
        ref = orc.decode_one(t)
        assert float(np.max(np.abs(ctx.logits() - ref))) <= LOGIT_TOL * _rms(ref), ctx.n_cells
    assert ctx.persist_stages > 0
