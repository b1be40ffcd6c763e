"""Op-level parity of the HIP kernels against the CPU restatement (oracle/ggml_ref.py).

Integer / byte work is checked bit-exactly (Q8_K activation quantisation,
dequantisation, top-k ids); the fp32 GEMV within an fp32-accumulation bound
relative to sum_b |coef_b * isum_b| (the exact per-block integer sums are
identical, only the float accumulation order differs)."""
import numpy as np
import pytest

import ggml_ref as R
from blama_amd import engine
from util import QTYPES, rand_matrix, rand_x

pytestmark = pytest.mark.gpu

GEMV_TOL = 2e-5   # relative to sum |terms| (fp32 accumulation of <= 2*K/16 partials)


@pytest.mark.parametrize("t", QTYPES)
@pytest.mark.parametrize("rows,K", [(2, 256), (7, 512), (64, 2048), (130, 4096), (33, 11008), (16, 14336)])
def test_gemv_matches_oracle(gpu_lib, t, rows, K):
    w = rand_matrix(t, rows, K, seed=rows * 7 + K)
    x = rand_x(K, seed=K)
    y = engine.op_gemv(t, w, rows, K, x)
    ref = R.mul_mat_vec(w, t, K, x).astype(np.float64)
    bound = R.mul_mat_vec_abs(w, t, K, x) * GEMV_TOL + 1e-30
    err = np.abs(y.astype(np.float64) - ref)
    assert np.all(err <= bound), (R.TYPE_NAME[t], float((err / bound).max()))


# the decode GEMVs at the BASELINE models' real shapes (multi-workgroup unit splits, K = 11008's
# 43 superblocks per row, the 32000- and 128256-row output heads)
@pytest.mark.parametrize("t,rows,K", [(R.Q4_K, 11008, 4096), (R.Q4_K, 4096, 11008), (R.Q6_K, 4096, 11008),
                                      (R.Q6_K, 32000, 4096), (R.Q6_K, 128256, 4096), (R.Q5_K, 14336, 4096),
                                      (R.Q8_0, 1024, 4096), (R.Q8_0, 5632, 2048), (R.Q8_0, 2048, 5632)])
def test_gemv_real_shapes_match_oracle(gpu_lib, t, rows, K):
    w = rand_matrix(t, rows, K, seed=rows + K)
    x = rand_x(K, seed=K + 1)
    y = engine.op_gemv(t, w, rows, K, x)
    # the oracle on a row subset for the large heads (every workgroup's range is still sampled)
    sel = np.arange(rows) if rows <= 16384 else np.unique(np.r_[np.arange(0, rows, 7), np.arange(rows - 64, rows)])
    ws = w.reshape(rows, R.row_bytes(t, K))[sel].reshape(-1)
    ref = R.mul_mat_vec(ws, t, K, x).astype(np.float64)
    bound = R.mul_mat_vec_abs(ws, t, K, x) * GEMV_TOL + 1e-30
    err = np.abs(y[sel].astype(np.float64) - ref)
    assert np.all(err <= bound), (R.TYPE_NAME[t], float((err / bound).max()))


@pytest.mark.parametrize("t", QTYPES)
def test_gemv_deterministic(gpu_lib, t):
    w = rand_matrix(t, 96, 4096, seed=3)
    x = rand_x(4096, seed=4)
    a = engine.op_gemv(t, w, 96, 4096, x)
    b = engine.op_gemv(t, w, 96, 4096, x)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("t", QTYPES)
def test_dequant_bit_exact(gpu_lib, t):
    rows, K = 5, 1024
    w = rand_matrix(t, rows, K, seed=11)
    got = engine.op_dequant(t, w, rows, K)
    ref = R.dequantize(w, t)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("K", [256, 4096, 11008])
def test_quantize_q8_K_bit_exact(gpu_lib, K):
    x = rand_x(K, seed=K, scale=3.0)
    x[17] = 0.0
    x[256 * (K // 512):256 * (K // 512) + 256] = 0.0         # an all-zero block
    if K >= 512:
        x[300], x[301] = 7.5, -7.5                            # |max| tie: first index wins
    qs, d, bs = engine.op_quantize_q8_K(x)
    ref = R.quantize_q8_K(x)
    assert np.array_equal(qs.astype(np.int32), ref.qs.reshape(-1))
    assert np.array_equal(d.view(np.uint32), ref.d.view(np.uint32))
    assert np.array_equal(bs, ref.bsums.reshape(-1))


@pytest.mark.parametrize("n", [1000, 32000, 128256])
def test_topk_exact(gpu_lib, n):
    rng = np.random.default_rng(n)
    lg = rng.standard_normal(n).astype(np.float32)
    lg[5] = lg[7] = lg.max() + 1.0                            # a tie at the top: id order
    ids, vals = engine.op_topk(lg, 64)
    ref = R.topk(lg, 64)
    assert [int(i) for i in ids] == [i for i, _ in ref]
    assert np.array_equal(vals, np.array([v for _, v in ref], np.float32))


def _attn_ref(q, k16, v16, n_head_kv, cell_pos, pos):
    n_head, hd = q.shape
    vis = [c for c in range(k16.shape[0]) if cell_pos[c] <= pos]
    K = k16[vis].reshape(len(vis), n_head_kv, hd)
    V = v16[vis].reshape(len(vis), n_head_kv, hd)
    scale = np.float32(1.0) / np.sqrt(np.float32(hd), dtype=np.float32)
    r = n_head // n_head_kv
    return np.stack([R.attention_head(q[h], K[:, h // r], V[:, h // r], scale) for h in range(n_head)])


# every (GQA ratio, head_dim) the BASELINE models instantiate -- 7B (32/32, 128), Llama-3-8B and
# Mixtral (32/8, 128), TinyLlama (32/4, 64) -- plus the small test shapes, on both sides of
# ATTN_SHORT (fused single launch <= 512 cells, split launches beyond)
@pytest.mark.parametrize("n_head,n_head_kv,hd", [(32, 32, 128), (32, 8, 128), (32, 4, 64), (4, 2, 64), (8, 8, 32)])
@pytest.mark.parametrize("n_cells", [1, 37, 512, 513, 2048])
def test_attention_matches_oracle(gpu_lib, n_head, n_head_kv, hd, n_cells):
    """Op-level attention vs the CPU graph's KQ -> soft_max -> KQV (f16 q and p, double sums).
    Bound: a one-ulp f16 rounding difference of a softmax weight p moves the output by at most
    2^-11 p |v|, so the error is within 2^-10 max|V| even if every weight rounds differently;
    the fp32 sum order adds ~1e-6 relative."""
    rng = np.random.default_rng(n_cells * 7 + hd + n_head_kv)
    q = (rng.standard_normal((n_head, hd)) * 0.6).astype(np.float32)
    k16 = (rng.standard_normal((n_cells, n_head_kv * hd)) * 0.6).astype(np.float16)
    v16 = rng.standard_normal((n_cells, n_head_kv * hd)).astype(np.float16)
    got = engine.op_attention(q, k16, v16, n_head_kv)
    ref = _attn_ref(q, k16, v16, n_head_kv, np.arange(n_cells), n_cells - 1)
    err = np.abs(got - ref)
    assert err.max() <= 2.0 ** -10 * np.abs(v16.astype(np.float32)).max(), float(err.max())
    assert err.mean() <= 1e-5, float(err.mean())


def test_attention_masks_future_positions(gpu_lib):
    """Cells whose position is past the query's (after a Self-Extend / seq_add shuffle) are
    masked (the kq_mask of llm_build_llama), in both attention modes."""
    rng = np.random.default_rng(5)
    for n_cells in (300, 700):
        q = rng.standard_normal((32, 128)).astype(np.float32) * 0.5
        k16 = (rng.standard_normal((n_cells, 8 * 128)) * 0.5).astype(np.float16)
        v16 = rng.standard_normal((n_cells, 8 * 128)).astype(np.float16)
        cp = rng.permutation(n_cells).astype(np.int32)
        pos = int(cp[-1])
        cp[-1] = pos                      # the query's own cell
        got = engine.op_attention(q, k16, v16, 8, cell_pos=cp, pos=pos)
        ref = _attn_ref(q, k16, v16, 8, cp, pos)
        assert np.abs(got - ref).max() <= 2.0 ** -10 * np.abs(v16.astype(np.float32)).max()
