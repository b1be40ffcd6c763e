"""Full-depth parity: the whole 32-layer models of BASELINE configs[1] and configs[3] against the
C restatement of the ggml CPU path (oracle/ggml_cpu.c), the way the reference's own GPU-vs-CPU
test runs the whole model (inference/test/t-LogitComparer.cpp:41-79).

Synthetic Llama-2-7B Q4_K_M, Llama-3-8B Q6_K and Mixtral-8x7B Q5_K_M (configs[4]: 8 experts, top-2
routing, n_ff 14336, Q8_0 attn_k / attn_v) (exact tensor names, shapes and type mix; random valid
blocks -- no checkpoint can be fetched).  Per model: a 16-token prompt, 16 greedy decode steps,
then a 64-token MI_OUT_ALL verification pass (the batched fillCtx path), every distribution
compared with the oracle decoding the same tokens one at a time.  Plus BASELINE configs[2]: the
7B with one full 512-token physical batch as the prompt, through the prefill path (MI_OUT_LAST)
and the batched verification path (MI_OUT_ALL), against the oracle at the last token and at every
32nd row.

Acceptance is the reference gate (t-LogitComparer.cpp:76-78): the MetricsAggregator score >= 0.95,
the mean logit similarity >= 0.98, and the top-1 id matching on every step and every verified row,
except where the oracle's own top-1 margin at that row is within the CPU algorithm's live reorder
floor (util.c_alt_floor, computed only when a mismatch occurs); every such waiver is printed and
raised as a warning (none fired in the r05 runs).  The element-wise error is printed, not gated:
at 32 layers the CPU algorithm's own re-quantisation floor (test_gpu_fullwidth.py's docstring)
grows past any fixed tolerance.

MoE rows are attributed (VERDICT r05 "What's weak" 3): every Mixtral row whose l2/rms error exceeds
3x the model's median must follow a routing near-tie -- a token, at or before that row, whose
oracle router gap (the last expert picked vs the first left out, min over the layers) is below
ROUTE_TIE: any fp32 order may pick the other expert there, and a different expert's output then
lives on in the residual and in that token's K/V cells.  The attribution is printed per row."""
import warnings

import numpy as np
import pytest

import ggml_cpu
import ggml_ref as R
from blama_amd import engine, synthetic
from util import ROUTE_TIE, c_alt_floor

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]   # the 32-layer oracle: ~1 min per model

MODELS = ["llama2-7b-q4_k_m", "llama3-8b-q6_k", "mixtral-8x7b-q5_k_m"]


def _gate(name, rows, floor_of=None):
    """rows: [(gpu top-10 [(id, logit)], oracle logits, tokens decoded)] -> assert the reference
    gate.  A top-1 mismatch passes only as a genuine CPU-side tie: when the oracle's own margin
    between its top id and the GPU's is within the CPU algorithm's reorder floor at that row
    (floor_of(): util.c_alt_floor over the same tokens, computed only if a mismatch occurs); each
    such waiver is printed and raised as a warning."""
    agg = R.MetricsAggregator()
    sims, top1, score, ties = [], [], None, []
    for i, (a, ref, ntok) in enumerate(rows):
        b = R.gather(ref.astype(np.float32), [x for x, _ in a])
        cm = R.compare(a, b)
        if cm.top1Match != 1.0:
            ties.append((i, ntok, a[0][0], int(np.argmax(ref)), float(ref.max() - ref[a[0][0]])))
        top1.append(cm.top1Match)
        score = agg.push_and_verify([cm])
        sims.append(R.logit_similarity(a, b))
    if ties:
        assert floor_of is not None, (name, ties)
        floor = floor_of()
        for i, ntok, gid, cid, margin in ties:
            msg = (f"live-floor waiver: {name} row {i} ({ntok} tokens): GPU top-1 {gid}, CPU {cid}, "
                   f"CPU margin {margin:.3e}, CPU reorder floor {floor[ntok]:.3e}")
            print(msg)
            warnings.warn(msg)
            assert margin <= floor[ntok], msg
            top1[i] = 1.0
    print(f"{name}: {len(rows)} distributions, score {score:.5f}, mean similarity {np.mean(sims):.5f}")
    assert score >= 0.95 and float(np.mean(sims)) >= 0.98 and min(top1) == 1.0, (name, score, np.mean(sims))


def _floor_by_tokens(buf, n_ctx, seq, n0):
    """c_alt_floor over seq (seq[:n0] as the prompt), indexed by the number of tokens decoded."""
    def f():
        print(f"computing the CPU reorder floor over {len(seq)} tokens", flush=True)
        _, fl = c_alt_floor(buf, n_ctx, seq[:n0], seq[n0:])
        out = np.full(len(seq) + 1, np.inf)
        out[n0:] = fl
        return out
    return f


def _attribute_moe_rows(name, errs, gaps):
    """Every row whose l2/rms exceeds 3x the median must follow a routing near-tie: a token at or
    before the row's last token with an oracle router gap < ROUTE_TIE.  Prints the attribution."""
    med = float(np.median([e for _, e, _ in errs]))
    ties = [j for j, g in enumerate(gaps) if g < ROUTE_TIE]
    print(f"{name}: median l2/rms {med:.2e}; routing near-ties (token index, gap): "
          f"{[(j, round(float(gaps[j]), 5)) for j in ties]}")
    bad, lines = [], []
    for label, e, j in errs:
        if e <= 3 * med:
            continue
        prev = [k for k in ties if k <= j]
        if not prev:
            bad.append((label, e))
            lines.append(f"{label}: l2/rms {e:.2e} ({e / med:.1f}x median) -- NO routing near-tie at or before token {j}")
            continue
        k = prev[-1]
        where = "at this token" if k == j else f"carried from token {k} ({j - k} tokens earlier)"
        lines.append(f"{label}: l2/rms {e:.2e} ({e / med:.1f}x median) <- routing near-tie {where}, "
                     f"oracle router gap {gaps[k]:.4f}")
    for ln in lines:
        print(f"{name} {ln}")
    if lines:   # in pytest's warnings summary, so the attribution is in every run's log
        warnings.warn(f"MoE row attribution, {name} (median l2/rms {med:.2e}): " + "; ".join(lines))
    assert not bad, (name, "rows above 3x the median error with no routing near-tie", bad)


@pytest.mark.parametrize("name", MODELS)
def test_fulldepth_decode_and_verify_match_oracle(gpu_lib, name):
    cfg = synthetic.CONFIGS[name]
    buf = synthetic.build_gguf(cfg, seed=21)
    print(f"{name}: synthetic GGUF built ({len(buf) / 1e9:.1f} GB)", flush=True)
    m = engine.Model(buf)
    ctx = engine.Context(m, n_ctx=128)
    orc = ggml_cpu.Model(buf, n_ctx=128)
    print(f"{name}: model loaded", flush=True)
    rng = np.random.default_rng(17)
    prompt = [int(t) for t in rng.integers(0, cfg.n_vocab, 16)]
    rows = []
    seq = list(prompt)
    gaps = []      # the oracle's router gap of every token decoded (inf: dense)
    errs = []      # (row label, l2/rms, index into gaps of the row's last token)
    try:
        assert ctx.decode(prompt) == 0
        for t in prompt:
            ref = orc.decode_one(t).astype(np.float64)
            gaps.append(orc.last_moe_margin)
        for s in range(17):
            got = ctx.logits()
            ids, vals = ctx.topk(10)
            d = np.abs(got.astype(np.float64) - ref)
            rms = float(np.sqrt(np.mean(ref ** 2)))
            print(f"{name} decode step {s}: max/rms {d.max() / rms:.2e} l2/rms {np.sqrt(np.mean(d ** 2)) / rms:.2e}",
                  flush=True)
            errs.append((f"decode step {s}", float(np.sqrt(np.mean(d ** 2)) / rms), len(gaps) - 1))
            rows.append(([(int(i), float(v)) for i, v in zip(ids, vals)], ref, len(seq)))
            if s == 16:
                break
            t = int(ids[0])                       # greedy: the model's own trajectory
            seq.append(t)
            assert ctx.decode([t]) == 0
            ref = orc.decode_one(t).astype(np.float64)
            gaps.append(orc.last_moe_margin)
        # the batched verification pass of 64 claimed tokens (Session::fillCtx, batchedVerify)
        claimed = [int(t) for t in rng.integers(0, cfg.n_vocab, 64)]
        assert ctx.decode(claimed, all_logits=True) == 0
        for i, t in enumerate(claimed):
            ref = orc.decode_one(t).astype(np.float64)
            gaps.append(orc.last_moe_margin)
            seq.append(t)
            ids, vals = ctx.topk(10, row=i)
            got = ctx.logits(row=i)
            d = np.abs(got.astype(np.float64) - ref)
            rms = float(np.sqrt(np.mean(ref ** 2)))
            if i % 16 == 0 or i == len(claimed) - 1:
                print(f"{name} verify row {i}: max/rms {d.max() / rms:.2e} l2/rms {np.sqrt(np.mean(d ** 2)) / rms:.2e}",
                      flush=True)
            errs.append((f"verify row {i}", float(np.sqrt(np.mean(d ** 2)) / rms), len(gaps) - 1))
            rows.append(([(int(x), float(v)) for x, v in zip(ids, vals)], ref, len(seq)))
        if cfg.n_expert:
            _attribute_moe_rows(name, errs, gaps)
        _gate(name, rows, _floor_by_tokens(buf, 128, seq, len(prompt)))
    finally:
        ctx.close()
        orc.close()
        m.close()


def test_fulldepth_512_token_prefill_matches_oracle(gpu_lib):
    """configs[2] at full depth: a 512-token prompt (one whole n_ubatch physical batch) through
    the int8-MFMA GEMMs and the MFMA causal attention, (a) as a prompt (MI_OUT_LAST: the last
    token's logits) and (b) as one MI_OUT_ALL verification pass; rows 0, 32, ..., 480 and 511
    against the oracle decoding the same tokens one at a time, under the reference gate with
    top-1 on every compared row."""
    name = "llama2-7b-q4_k_m"
    cfg = synthetic.CONFIGS[name]
    buf = synthetic.build_gguf(cfg, seed=23)
    print("512-prefill: synthetic GGUF built", flush=True)
    m = engine.Model(buf)
    last_ctx = engine.Context(m, n_ctx=544)
    all_ctx = engine.Context(m, n_ctx=544)
    orc = ggml_cpu.Model(buf, n_ctx=544)
    prompt = [int(t) for t in np.random.default_rng(29).integers(0, cfg.n_vocab, 512)]
    try:
        assert last_ctx.decode(prompt) == 0
        assert all_ctx.decode(prompt, all_logits=True) == 0
        want = set(range(0, 512, 32)) | {511}
        rows = []
        for i, t in enumerate(prompt):
            ref = orc.decode_one(t)
            if i % 64 == 0:
                print(f"512-prefill: oracle at token {i}", flush=True)
            if i not in want:
                continue
            ref = ref.astype(np.float64)
            rms = float(np.sqrt(np.mean(ref ** 2)))
            for tag, ctx, row in (("all", all_ctx, i), ("last", last_ctx, -1)):
                if tag == "last" and i != 511:
                    continue
                got = ctx.logits(row=row).astype(np.float64)
                ids, vals = ctx.topk(10, row=row)
                d = np.abs(got - ref)
                print(f"512-prefill {tag} row {i}: max/rms {d.max() / rms:.2e} l2/rms {np.sqrt(np.mean(d ** 2)) / rms:.2e}",
                      flush=True)
                rows.append(([(int(x), float(v)) for x, v in zip(ids, vals)], ref, i + 1))
        assert len(rows) == len(want) + 1
        _gate(name + " 512-token prefill", rows, _floor_by_tokens(buf, 544, prompt, 1))
    finally:
        last_ctx.close()
        all_ctx.close()
        orc.close()
        m.close()
