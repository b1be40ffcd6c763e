"""CPU tests of the oracle (no GPU): the reference's LogitComparer known-answer
test, the two independent restatements (numpy oracle/ggml_ref.py and C
oracle/ggml_cpu.c) against each other, the committed golden fixtures, and
format invariants."""
import os

import numpy as np
import pytest

import ggml_ref as R
from util import QTYPES, rand_matrix, rand_x, oracle_from_gguf
from blama_amd import synthetic

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.npz")


def test_logit_comparer_kat_no_model():
    """inference/test/t-LogitComparer.cpp:13-39 ("compare - no model")."""
    tdv = [(i, 17.5 - 0.5 * i) for i in range(10)]
    assert R.logit_similarity(tdv, tdv) == 1.0
    m = R.compare(tdv, tdv)
    assert m.top1Match == 1.0 and m.distance == 0.0 and m.jsd == 0.0
    assert R.MetricsAggregator().push_and_verify([m]) == 1.0


def test_logit_comparer_behaviour():
    a = [(1, 10.0), (2, 9.0), (3, 8.0)]
    b = [(2, 10.0), (1, 9.0), (3, 8.0)]
    m = R.compare(a, b)
    assert m.top1Match == 0.0 and m.distance == 0.0 and m.jsd > 0.0
    # similarity is |logit|-weighted 1 - |d|/|max|
    s = R.logit_similarity(a, b)
    assert 0.8 < s < 1.0
    agg = R.MetricsAggregator()
    s1 = agg.push_and_verify([R.compare(a, a)])
    s2 = agg.push_and_verify([m])
    assert s1 == 1.0 and s2 < 1.0


def test_topk_and_gather_semantics():
    lg = np.array([0.5, 3.0, 3.0, -1.0, 2.0], np.float32)
    assert [i for i, _ in R.topk(lg, 3)] == [1, 2, 4]          # ties by id ascending
    assert [i for i, _ in R.gather(lg, [4, 0, 4, 1])] == [1, 4, 0]  # set semantics, sorted desc


@pytest.mark.parametrize("t", QTYPES)
def test_c_oracle_matches_numpy_oracle_gemv(t):
    import ggml_cpu
    w = rand_matrix(t, 45, 2048, seed=9)
    x = rand_x(2048, seed=2)
    a = ggml_cpu.gemv(t, w, 45, 2048, x).astype(np.float64)
    b = R.mul_mat_vec(w, t, 2048, x).astype(np.float64)
    bound = R.mul_mat_vec_abs(w, t, 2048, x) * 2e-6
    assert np.all(np.abs(a - b) <= bound)


@pytest.mark.parametrize("t", QTYPES)
def test_c_oracle_avx2_dots_match_generic(t):
    """The AVX2 dot kernels the bench's CPU-baseline leg times (ggml's x86 technique) form the
    generic loops' integers; only the fp32 lane grouping differs -- at the GEMV bar."""
    import ggml_cpu
    rows, K = 45, 4096
    w = rand_matrix(t, rows, K, seed=19)
    x = rand_x(K, seed=4)
    try:
        ggml_cpu.set_simd(True)
        a = ggml_cpu.gemv(t, w, rows, K, x).astype(np.float64)
    finally:
        ggml_cpu.set_simd(False)
    b = ggml_cpu.gemv(t, w, rows, K, x).astype(np.float64)
    bound = R.mul_mat_vec_abs(w, t, K, x) * 2e-6
    assert np.all(np.abs(a - b) <= bound), float(np.max(np.abs(a - b) / bound))


@pytest.mark.parametrize("cfg", ["tiny-q4_k_m", "tiny-q8_0", "tiny-moe-q5_k_m"])
def test_c_oracle_matches_numpy_oracle_decode(cfg):
    import ggml_cpu
    buf = synthetic.build_gguf(synthetic.CONFIGS[cfg], seed=5)
    c = ggml_cpu.Model(buf, n_ctx=32)
    o = oracle_from_gguf(buf, n_ctx=32)
    for tok in [1, 17, 42, 99, 7]:
        a, b = c.decode_one(tok), o.decode_one(tok)
        rms = float(np.sqrt(np.mean(b.astype(np.float64) ** 2)))
        assert np.max(np.abs(a - b)) <= 1e-4 * rms
        assert [i for i, _ in R.topk(a, 10)] == [i for i, _ in R.topk(b, 10)]


@pytest.mark.parametrize("t", QTYPES)
def test_dequant_consistent_with_vec_dot(t):
    """sum_k dequant(w)_k * dequant(q8(x))_k == the integer-block vec_dot (two code paths)."""
    K = 512
    w = rand_matrix(t, 3, K, seed=1)
    x = rand_x(K, seed=3)
    W = R.dequantize(w, t).reshape(3, K).astype(np.float64)
    if t == R.Q8_0:
        a = R.quantize_q8_0(x)
        xq = (a.qs * a.d[:, None]).reshape(-1)
    else:
        a = R.quantize_q8_K(x)
        xq = (a.qs * a.d[:, None].astype(np.float64)).reshape(-1)
    y = R.mul_mat_vec(w, t, K, x).astype(np.float64)
    assert np.allclose(W @ xq, y, rtol=2e-5, atol=1e-6 * np.abs(W).sum(1).max())


def test_quantize_q8_K_invariants():
    x = rand_x(1024, seed=7, scale=5.0)
    q = R.quantize_q8_K(x)
    assert q.qs.min() >= -127 and q.qs.max() <= 127
    assert np.all(q.bsums == q.qs.reshape(-1, 16, 16).sum(-1))
    err = np.abs(q.qs * q.d[:, None] - x.reshape(-1, 256))
    assert np.all(err <= np.abs(q.d)[:, None] * 0.5 + 1e-6)


def test_golden_fixtures():
    """Committed golden vectors (tests/golden/make_golden.py) still reproduce."""
    g = np.load(GOLDEN, allow_pickle=False)
    for t in QTYPES:
        w = g[f"w_{t}"]
        x = g[f"x_{t}"]
        K = x.size
        rows = w.size // R.row_bytes(t, K)
        assert np.array_equal(R.dequantize(w, t).view(np.uint32), g[f"deq_{t}"].view(np.uint32))
        y = R.mul_mat_vec(w, t, K, x)
        assert np.array_equal(y.view(np.uint32), g[f"y_{t}"].view(np.uint32)), R.TYPE_NAME[t]
    qk = R.quantize_q8_K(g["xq"])
    assert np.array_equal(qk.qs.reshape(-1).astype(np.int8), g["q8k_qs"])
    assert np.array_equal(qk.d.view(np.uint32), g["q8k_d"].view(np.uint32))
    buf = synthetic.build_gguf(synthetic.CONFIGS["tiny-q4_k_m"], seed=11)
    o = oracle_from_gguf(buf, n_ctx=16)
    lg = o.decode(list(g["prompt"]))
    assert np.array_equal(lg.view(np.uint32), g["logits"].view(np.uint32))
