"""Oracle parity of every shipped kernel instantiation at the BASELINE models' real widths.

The small configs of test_gpu_decode.py all have n_embd 256 with GQA, so they never run the
instantiations the benchmarks run.  These tests build full-width, reduced-depth synthetic
models (2 layers; real n_embd, heads, head_dim, n_ff, vocabulary and Q*_K_M tensor mix) and
compare the HIP engine with the C restatement of the ggml CPU path (oracle/ggml_cpu.c):

  Llama-2-7B Q4_K_M   R=1, hd=128: attn_fused_kernel<1,16>, split attention past 512 cells,
                      the mixed Q4_K/Q6_K QKV launch (layer 1 is a use_more_bits layer),
                      16-wave FFN gate/up over 11008 rows, Q6_K output over 32000 rows
  Llama-3-8B Q6_K     R=4, hd=128, V=128256 (the top-k over 126 blocks)
  Mixtral Q5_K_M      8 experts (so attn_k/attn_v are Q8_0, llama_tensor_get_type's
                      8-expert rule), top-2 routing, R=4; n_ff cut to 1024, and once at the
                      real 14336 (the real expert GEMV / GEMM shapes and expert stride)
  TinyLlama Q8_0      R=8, hd=64, Q8_0 everywhere

Tolerance.  At these widths the CPU algorithm is not stable to its own fp32 summation order:
the C oracle run with the 8 float lanes of every k-quant dot summed in the reverse order (an
equally valid order; ggml's AVX2 and generic paths differ in exactly this way) moves the
logits by up to 6.6e-2 x rms (max) and 1.4e-2 x rms (L2) on these models (measured over 11
steps x 3 models; profiles/r02_fullwidth_floor.txt).  The cause is the Q8_K / Q8_0
re-quantisation of every GEMV input: a last-bit difference flips an activation quantum, and
the flips compound through the layers.  The element-wise 2e-3 of the small configs is below
that floor, so here each step must satisfy
  * max|dlogit| <= TOL_MAX x rms and ||dlogit||_2 <= TOL_L2 x ||logit||_2 (about twice the
    floor), and the run's mean L2 error within twice the live floor (the same oracle in the
    reversed order, decoded alongside: k-quant lanes, or Q8_0 blocks, summed in reverse);
  * top-10 ids identical up to near ties: the GPU's rank-i id, scored by the oracle, is within
    2 max|dlogit| of the oracle's rank-i logit;
and the run must pass the reference's acceptance gate (t-LogitComparer.cpp:76-78: aggregate
score >= 0.95, mean logitSimilarity >= 0.98, top-1 match on every step).  The kernels' own
arithmetic is checked without this chaos at op level (test_gpu_ops.py: GEMV at these shapes,
attention at these head shapes)."""
import warnings

import numpy as np
import pytest

import ggml_cpu
import ggml_ref as R
from blama_amd import engine, synthetic
from util import ROUTE_TIE, c_alt_floor

pytestmark = pytest.mark.gpu

TOL_MAX = 0.12
TOL_L2 = 0.03
# MoE: router probabilities of the last expert picked and the first left out closer than this
# (in the oracle) are a near-tie that another fp32 order of the same arithmetic may swap

FULL = {
    "llama2-7b-q4_k_m": dict(n_layer=2),
    "llama3-8b-q6_k": dict(n_layer=2),
    "mixtral-8x7b-q5_k_m": dict(n_layer=2, n_ff=1024),
    # the real 14336 x 4096 Q5_K experts (8 per layer, ~1 GB a layer) at the real expert stride
    "mixtral-8x7b-q5_k_m-ff14336": dict(base="mixtral-8x7b-q5_k_m", n_layer=2),
    "tinyllama-1.1b-q8_0": dict(n_layer=2),
}

_cache = {}


def full_model(name):
    """(cfg, gguf image, engine model) -- built once per test session."""
    if name not in _cache:
        kw = dict(FULL[name])
        cfg = synthetic.small_config(kw.pop("base", name), **kw)
        buf = synthetic.build_gguf(cfg, seed=3)
        _cache[name] = (cfg, buf, engine.Model(buf))
    return _cache[name]


def _err(got, ref):
    d = np.abs(got.astype(np.float64) - ref)
    rms = float(np.sqrt(np.mean(ref ** 2)))
    return float(d.max()), float(d.max()) / rms, float(np.sqrt(np.mean(d ** 2))) / rms


def _check_run(name, ctx, orc, prompt, steps, rng):
    """Decode `prompt` then `steps` tokens on the engine, the oracle and the oracle in the
    reversed lane order; check every distribution."""
    cfg = _cache[name][0]
    assert ctx.decode(prompt) == 0
    alt = ggml_cpu.Model(_cache[name][1], n_ctx=orc.n_ctx)
    for t in prompt:
        ref = orc.decode_one(t).astype(np.float64)
        ref_alt = alt.decode_one(t, alt=True)
    agg = R.MetricsAggregator()
    sims, top1, l2s, alt_l2s = [], [], [], []
    score = None
    try:
        for s in range(steps + 1):
            got = ctx.logits()
            ids, vals = ctx.topk(10)
            dmax, rmax, rl2 = _err(got, ref)
            _, amax, al2 = _err(ref_alt, ref)
            l2s.append(rl2)
            alt_l2s.append(al2)
            print(f"{name} step {s} cells {ctx.n_cells}: max/rms {rmax:.1e} l2 {rl2:.1e} "
                  f"(cpu reorder floor: max {amax:.1e} l2 {al2:.1e})")
            assert rmax <= TOL_MAX and rl2 <= TOL_L2, (name, s, rmax, rl2)
            ref_sorted = np.sort(ref)[::-1][:10]
            assert len(set(int(i) for i in ids)) == 10
            assert np.all(np.abs(ref[ids.astype(np.int64)] - ref_sorted) <= 2 * dmax + 1e-6), (name, s)
            a = [(int(i), float(v)) for i, v in zip(ids, vals)]
            b = R.gather(ref.astype(np.float32), [i for i, _ in a])
            cm = R.compare(a, b)
            top1.append(cm.top1Match)
            score = agg.push_and_verify([cm])
            sims.append(R.logit_similarity(a, b))
            if s == steps:
                break
            # follow the model's own preference most of the time (a realistic trajectory)
            t = int(ids[0]) if rng.random() < 0.7 else int(rng.integers(0, cfg.n_vocab))
            assert ctx.decode([t]) == 0
            ref = orc.decode_one(t).astype(np.float64)
            ref_alt = alt.decode_one(t, alt=True)
    finally:
        alt.close()
    # the run's mean error within twice the live floor (Q8_0: its blocks summed in reverse order)
    assert max(alt_l2s) > 0, "the reversed-order oracle did not move: no floor measured"
    assert np.mean(l2s) <= 2 * np.mean(alt_l2s) + 2e-3, (np.mean(l2s), np.mean(alt_l2s))
    assert score >= 0.95 and float(np.mean(sims)) >= 0.98 and min(top1) == 1.0, (score, np.mean(sims))


@pytest.mark.parametrize("name", list(FULL))
def test_fullwidth_decode_matches_oracle(gpu_lib, name):
    cfg, buf, m = full_model(name)
    ctx = engine.Context(m, n_ctx=64)
    orc = ggml_cpu.Model(buf, n_ctx=64)
    rng = np.random.default_rng(11)
    prompt = [int(t) for t in rng.integers(0, cfg.n_vocab, 12)]
    try:
        _check_run(name, ctx, orc, prompt, steps=10, rng=rng)
    finally:
        ctx.close()
        orc.close()


def test_fullwidth_7b_crosses_512_cells(gpu_lib):
    """hd=128 past ATTN_SHORT: a 508-token prompt (batched ingestion), then decode steps over
    cells 509..518, switching from the fused attention graph to the split one at 512."""
    name = "llama2-7b-q4_k_m"
    cfg, buf, m = full_model(name)
    ctx = engine.Context(m, n_ctx=600)
    orc = ggml_cpu.Model(buf, n_ctx=600)
    rng = np.random.default_rng(12)
    prompt = [int(t) for t in rng.integers(0, cfg.n_vocab, 508)]
    try:
        _check_run(name, ctx, orc, prompt, steps=10, rng=rng)
        assert ctx.n_cells == 518
    finally:
        ctx.close()
        orc.close()


@pytest.mark.parametrize("name", ["llama2-7b-q4_k_m", "llama3-8b-q6_k", "tinyllama-1.1b-q8_0",
                                  "mixtral-8x7b-q5_k_m-ff14336"])
def test_fullwidth_batched_verification_matches_oracle(gpu_lib, name):
    """MI_OUT_ALL at real widths: 24 claimed tokens after a 20-token prompt in one batched pass
    (mmq32 for every projection and the output head, MFMA attention; Mixtral: the router per
    token, each expert's GEMMs over the tokens routed to it, Q8_0 attn_k / attn_v on their own
    Q8_0 activations); every row against the C
    oracle decoding the same tokens one at a time, with this file's tolerances and the
    reference gate, and the claimed ids gathered per row (mi_gather_rows) as fillCtx does."""
    cfg, buf, m = full_model(name)
    ctx = engine.Context(m, n_ctx=64)
    orc = ggml_cpu.Model(buf, n_ctx=64)
    rng = np.random.default_rng(13)
    prompt = [int(t) for t in rng.integers(0, cfg.n_vocab, 20)]
    claimed = [int(t) for t in rng.integers(0, cfg.n_vocab, 24)]
    try:
        ctx.decode(prompt)
        orc.decode(prompt)
        assert ctx.decode(claimed, all_logits=True) == 0
        agg = R.MetricsAggregator()
        sims, top1, ties = [], [], []
        score = None
        ids_rows = np.zeros((len(claimed), 10), np.int32)
        refs = []
        for i, t in enumerate(claimed):
            ref = orc.decode_one(t).astype(np.float64)
            refs.append(ref)
            got = ctx.logits(row=i)
            dmax, rmax, rl2 = _err(got, ref)
            assert rmax <= TOL_MAX and rl2 <= TOL_L2, (name, i, rmax, rl2)
            ids, vals = ctx.topk(10, row=i)
            ids_rows[i] = ids
            ref_sorted = np.sort(ref)[::-1][:10]
            assert np.all(np.abs(ref[ids.astype(np.int64)] - ref_sorted) <= 2 * dmax + 1e-6), (name, i)
            a = [(int(x), float(v)) for x, v in zip(ids, vals)]
            cm = R.compare(a, R.gather(ref.astype(np.float32), [x for x, _ in a]))
            # top-1 on every row, as the reference gate demands (t-LogitComparer.cpp:76-78); a
            # mismatch is re-examined below against the CPU algorithm's own floor at that row
            if cm.top1Match != 1.0:
                ties.append((i, int(ids[0]), int(np.argmax(ref)), float(ref.max() - ref[int(ids[0])])))
            top1.append(cm.top1Match)
            score = agg.push_and_verify([cm])
            sims.append(R.logit_similarity(a, R.gather(ref.astype(np.float32), [x for x, _ in a])))
        g = ctx.gather_rows(0, ids_rows)
        for i in range(len(claimed)):
            assert np.array_equal(g[i], ctx.logits(row=i)[ids_rows[i]])
        if ties:
            # A top-1 mismatch passes only as a genuine CPU-side tie: the oracle's own margin
            # between its top id and the GPU's is within the live floor at that row (the same
            # C oracle with the 8 lanes of every k-quant dot summed in reverse, an equally valid
            # ggml order: util.c_alt_floor), i.e. the CPU algorithm itself ranks them either way.
            _, floor = c_alt_floor(buf, 64, prompt, claimed)
            for i, gid, cid, margin in ties:
                msg = (f"live-floor waiver: {name} row {i}: GPU top-1 {gid}, CPU {cid}, CPU margin {margin:.3e}, "
                       f"CPU reorder floor {floor[i + 1]:.3e}")
                print(msg)
                warnings.warn(msg)   # listed in pytest's warnings summary, also under -q
                assert margin <= floor[i + 1], (name, i, gid, cid, margin, floor[i + 1])
                top1[i] = 1.0
        assert score >= 0.95 and float(np.mean(sims)) >= 0.98 and min(top1) == 1.0, (score, np.mean(sims))
    finally:
        ctx.close()
        orc.close()


@pytest.mark.parametrize("name", ["llama2-7b-q4_k_m", "llama3-8b-q6_k", "tinyllama-1.1b-q8_0",
                                  "mixtral-8x7b-q5_k_m-ff14336"])
def test_fullwidth_short_batches_match_tiled_gemm(gpu_lib, monkeypatch, name):
    """Short verification batches (20 and 64 claimed tokens) on the split-K streaming GEMM
    (mmqs: K-parts summed by the consumer kernels; Mixtral: the routed experts on the grouped
    form, each expert's rows over its own matrix) against the same batches on the tiled GEMM
    (mmq2, MI_MMQS_MAX=0).  Per matrix the two agree to the GEMM op bar (test_gpu_batch_ops:
    the same integer sub-block sums, only the fp32 order of the K-parts differs); through the
    layers such differences flip Q8_K roundings of the next activation the way any fp32 order
    does -- on these random-weight models every batch path (and the per-token path) sits 4-7 % of
    rms from the C oracle at its worst element (scripts/diag_short.py) -- so the two paths are
    held to this file's bars against each other, with top-1 equal unless within twice the row's
    largest difference of a tie; the KV cache each batch wrote serves the next step alike.
    Mixtral: a row may differ beyond the bars only where the oracle's router separates the last
    expert picked from the first left out by less than ROUTE_TIE (the same noise then picks a
    different expert: measured on this model at 64 tokens, row 60, last layer, gap 0.0037),
    at most 2 rows per batch, each printed as a waiver."""
    cfg, buf, m = full_model(name)
    rng = np.random.default_rng(21)
    prompt = [int(t) for t in rng.integers(0, cfg.n_vocab, 12)]
    for n_claim in (20, 64):
        claimed = [int(t) for t in rng.integers(0, cfg.n_vocab, n_claim)]
        margins = [np.inf] * n_claim
        if cfg.n_expert:   # the oracle's router gap per claimed token (routing near-ties, below)
            orc = ggml_cpu.Model(buf, n_ctx=128)
            try:
                for t in prompt:
                    orc.decode_one(t)
                for i, t in enumerate(claimed):
                    orc.decode_one(t)
                    margins[i] = orc.last_moe_margin
            finally:
                orc.close()
        outs = []
        for mode in ("64", "0"):
            monkeypatch.setenv("MI_MMQS_MAX", mode)
            ctx = engine.Context(m, n_ctx=128)
            try:
                assert ctx.decode(prompt) == 0
                assert ctx.decode(claimed, all_logits=True) == 0
                rows = [ctx.logits(row=i).astype(np.float64) for i in range(n_claim)]
                ctx.decode([7])
                rows.append(ctx.logits().astype(np.float64))
                outs.append(rows)
            finally:
                ctx.close()
        flips = []
        for i, (a, b) in enumerate(zip(*outs)):
            dmax, rmax, rl2 = _err(a, b)
            if i < n_claim and margins[i] < ROUTE_TIE and not (rmax <= TOL_MAX and rl2 <= TOL_L2):
                # a routing near-tie: the two paths' activations differ by the usual Q8_K
                # re-quantisation noise, enough to swap two experts whose router probabilities
                # the oracle separates by less than ROUTE_TIE -- a different expert, a different row
                flips.append((i, margins[i], rmax))
                continue
            assert rmax <= TOL_MAX and rl2 <= TOL_L2, (name, n_claim, i, rmax, rl2, margins[min(i, n_claim - 1)])
            ia, ib = int(np.argmax(a)), int(np.argmax(b))
            assert ia == ib or b[ib] - b[ia] <= 2 * dmax, (name, n_claim, i, ia, ib)
        if flips:
            msg = f"routing near-tie waiver: {name} {n_claim} tokens: (row, oracle router gap, max/rms) {flips}"
            print(msg)
            warnings.warn(msg)
        assert len(flips) <= 2, flips
    monkeypatch.delenv("MI_MMQS_MAX")
