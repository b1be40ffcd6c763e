"""Op-level parity of the prompt-batch kernels at the BASELINE models' real widths.

The decode kernels are pinned op by op in test_gpu_ops.py; these are the kernels of the
n_ubatch physical batches (Session.cpp:381-392, Instance.hpp:23-24) -- prompt ingestion and
batched verification:

  mmq2_t / mmqs_t (mmq.hip)  v_mfma_i32_32x32x32_i8 GEMMs of up to 512 token rows (mmqs: the
                             split-K streaming form of <= 64 rows), every weight row tile and
                             every padded token tile, through mi_op_gemm
  attn_mfma_kernel (attn_mfma.hip)  f16-MFMA causal attention over 512..2048 cells, through
                             mi_op_attention_batch

GEMM bar.  Each token row's activation is quantised to Q8_K (Q8_0 for Q8_0 weights) exactly as
the CPU graph does (quantize_row_q8_K / the x86 quantize_row_q8_0), and every per-block integer
dot the MFMA forms is the exact int32 of vec_dot_q*_q8_K / vec_dot_q8_0_q8_0; only the fp32 order
in which the blocks are added differs.  So every element must lie within
GEMM_TOL x sum_b |term_b| of the oracle (the 2e-5 of the decode GEMV tests), where term_b are
the per-block products d_w*d_x*isum (and the Q4_K -dmin*d_x*sum(m*bsum) terms) of
oracle/ggml_ref.block_sums, computed here in float64 for all tokens at once.
Attention bar: as test_gpu_ops.test_attention_matches_oracle (2^-10 max|V|: one f16 rounding
flip of a softmax weight moves the output by at most 2^-11 p|v|)."""
import numpy as np
import pytest

import ggml_ref as R
from blama_amd import engine
from util import rand_matrix, rand_x

pytestmark = pytest.mark.gpu

GEMM_TOL = 2e-5


def _act_blocks(t, X):
    """Dequantised activations per quant block: (blk_elems, A[T, nblk, blk_elems] f64)."""
    T, K = X.shape
    if t == R.Q8_0:
        a = [R.quantize_q8_0(x) for x in X]
        A = np.stack([q.d[:, None].astype(np.float64) * q.qs for q in a])          # (T, K/32, 32)
        return 32, A
    a = [R.quantize_q8_K(x) for x in X]
    A = np.stack([q.d[:, None].astype(np.float64) * q.qs for q in a])              # (T, K/256, 256)
    return 256, A


def _weight_blocks(t, raw, rows, K):
    """(Wp, Wm): the per-block weights split into the d*scale*q part and the -dmin*m part
    (Q4_K only; None otherwise), f64 (rows, nblk, blk_elems)."""
    if t in (R.Q4_K, R.Q5_K):
        d, dmin, sc, m, q = (R.unpack_q4_K if t == R.Q4_K else R.unpack_q5_K)(raw)
        nb = K // 256
        q = q.reshape(rows, nb, 8, 32).astype(np.float64)
        Wp = d.reshape(rows, nb, 1, 1).astype(np.float64) * sc.reshape(rows, nb, 8, 1) * q
        Wm = np.broadcast_to((dmin.reshape(rows, nb, 1, 1).astype(np.float64) * m.reshape(rows, nb, 8, 1)),
                             (rows, nb, 8, 32))
        return Wp.reshape(rows, nb, 256), -Wm.reshape(rows, nb, 256)
    if t == R.Q6_K:
        d, sc, q = R.unpack_q6_K(raw)
        nb = K // 256
        Wp = d.reshape(rows, nb, 1, 1).astype(np.float64) * sc.reshape(rows, nb, 16, 1) * \
            q.reshape(rows, nb, 16, 16).astype(np.float64)
        return Wp.reshape(rows, nb, 256), None
    d, q = R.unpack_q8_0(raw)
    nb = K // 32
    return d.reshape(rows, nb, 1).astype(np.float64) * q.reshape(rows, nb, 32), None


def gemm_ref(t, raw, rows, K, X):
    """y[T, rows] and the bound sum_b |term_b| (f64), all tokens at once."""
    _, A = _act_blocks(t, X)
    Wp, Wm = _weight_blocks(t, raw, rows, K)
    T = X.shape[0]
    y = np.zeros((T, rows))
    bound = np.zeros((T, rows))
    for b in range(A.shape[1]):
        yp = A[:, b] @ Wp[:, b].T
        y += yp
        bound += np.abs(yp)
        if Wm is not None:
            ym = A[:, b] @ Wm[:, b].T
            y += ym
            bound += np.abs(ym)
    return y, bound


def _check_gemm(t, rows, K, ntok, pair, seed):
    raw = rand_matrix(t, rows, K, seed=seed)
    X = np.stack([rand_x(K, seed=seed * 1000 + i) for i in range(ntok)])
    X[ntok // 2, :256] = 0.0                               # an all-zero activation block (d = 0)
    up = rand_matrix(t, rows, K, seed=seed + 1) if pair else None
    got = engine.op_gemm(t, raw, rows, K, X, raw_up=up).astype(np.float64)
    g, bg = gemm_ref(t, raw, rows, K, X)
    if not pair:
        err = np.abs(got - g)
        lim = GEMM_TOL * bg + 1e-30
    else:
        u, bu = gemm_ref(t, up, rows, K, X)
        s = g / (1.0 + np.exp(-g))
        ref = s * u
        err = np.abs(got - ref)
        # d(silu(g) u) <= |silu'(g)| |u| eg + |silu(g)| eu, |silu'| <= 1.1; plus the fp32 epilogue
        lim = GEMM_TOL * (1.1 * np.abs(u) * bg + np.abs(s) * bu) + 1e-6 * np.abs(ref) + 1e-30
    bad = np.argwhere(err > lim)
    assert bad.size == 0, (R.TYPE_NAME[t], rows, K, ntok, len(bad), bad[:5].tolist(), float((err / lim).max()))


# (type, rows, K, token counts, gate/up pair): the 7B / Llama-3-8B / Mixtral (Q5_K experts) /
# TinyLlama projection shapes,
# 33 tokens (one full 32-token tile + a 1-token padded tile), 128, and a whole 512-token batch
GEMM_CASES = [
    (R.Q4_K, 4096, 4096, (33, 128, 512), False),
    (R.Q4_K, 11008, 4096, (33, 512), True),
    (R.Q4_K, 4096, 11008, (128, 512), False),
    (R.Q4_K, 14336, 4096, (128,), False),
    (R.Q5_K, 4096, 4096, (33, 512), False),
    (R.Q5_K, 14336, 4096, (128,), True),
    (R.Q5_K, 4096, 14336, (128,), False),
    (R.Q6_K, 4096, 4096, (33, 512), False),
    (R.Q6_K, 4096, 11008, (512,), False),
    (R.Q6_K, 14336, 4096, (128,), True),
    (R.Q6_K, 4096, 14336, (128,), False),
    (R.Q6_K, 32000, 4096, (128,), False),
    (R.Q8_0, 2048, 2048, (33, 512), False),
    (R.Q8_0, 5632, 2048, (128,), True),
    (R.Q8_0, 2048, 5632, (512,), False),
    (R.Q8_0, 32000, 2048, (64,), False),
]


@pytest.mark.parametrize("t,rows,K,ntoks,pair", GEMM_CASES,
                         ids=[f"{R.TYPE_NAME[c[0]]}-{c[1]}x{c[2]}{'-pair' if c[4] else ''}" for c in GEMM_CASES])
def test_mmq32_matches_oracle(gpu_lib, monkeypatch, t, rows, K, ntoks, pair):
    # mi_op_gemm sends <= 64-token calls to the short-batch GEMM: pin the tiled one at these counts
    # too (the engine still runs it for MoE experts without the grouped form)
    monkeypatch.setenv("MI_MMQS_MAX", "0")
    for ntok in ntoks:
        _check_gemm(t, rows, K, ntok, pair, seed=rows + K + ntok)


# the short-batch GEMM (mmqs: <= 64 tokens, split over K; mi_op_gemm sums the K-parts as the
# engine's consumers do): every type at the widths whose K splits into 4, 11, 14 and 22 parts,
# one and two token tiles
MMQS_CASES = [
    (R.Q4_K, 4096, 4096, (2, 20, 64), False),
    (R.Q4_K, 11008, 4096, (20, 64), True),
    (R.Q4_K, 4096, 11008, (20, 64), False),
    (R.Q5_K, 4096, 14336, (24,), False),
    (R.Q5_K, 4096, 4096, (64,), False),     # Mixtral's Q / W_o at 64 tokens: two token tiles
    (R.Q5_K, 1000, 4096, (40,), True),
    (R.Q6_K, 4096, 11008, (20, 64), False),
    (R.Q6_K, 1000, 4096, (33,), True),
    (R.Q6_K, 32000, 4096, (20,), False),
    (R.Q8_0, 2048, 5632, (20, 64), False),
    (R.Q8_0, 5632, 2048, (24,), True),
]


@pytest.mark.parametrize("t,rows,K,ntoks,pair", MMQS_CASES,
                         ids=[f"{R.TYPE_NAME[c[0]]}-{c[1]}x{c[2]}{'-pair' if c[4] else ''}" for c in MMQS_CASES])
def test_mmqs_matches_oracle(gpu_lib, t, rows, K, ntoks, pair):
    for ntok in ntoks:
        _check_gemm(t, rows, K, ntok, pair, seed=3 * rows + K + ntok)


def test_mmq32_rows_not_multiple_of_tile(gpu_lib, monkeypatch):
    """Row counts that leave a partial 32-row (pair: 16-row) tile (the tiled GEMM at every count)."""
    monkeypatch.setenv("MI_MMQS_MAX", "0")
    _check_gemm(R.Q4_K, 1000, 2048, 40, False, seed=7)
    _check_gemm(R.Q4_K, 1000, 2048, 40, True, seed=8)
    _check_gemm(R.Q4_K, 1000, 2048, 5, True, seed=11)       # one token tile
    _check_gemm(R.Q4_K, 1000, 2048, 70, False, seed=12)     # three token tiles (no tile pair for the last)
    _check_gemm(R.Q5_K, 77, 1024, 200, True, seed=13)       # a second 128-token block of two tiles
    _check_gemm(R.Q6_K, 77, 1024, 5, False, seed=9)
    _check_gemm(R.Q5_K, 77, 1024, 5, True, seed=10)


def attn_batch_ref(q, k16, v16, n_head_kv, tok_cell, tok_pos, cell_pos):
    """KQ -> masked soft_max -> KQV per token and head, as R.attention_head (f16 q and p, f32
    softmax with a double sum), vectorised over the tokens and the q heads of each kv head."""
    T, n_head, hd = q.shape
    r = n_head // n_head_kv
    scale = np.float32(1.0) / np.sqrt(np.float32(hd), dtype=np.float32)
    n = k16.shape[0]
    cells = np.arange(n)
    vis = (cells[None, :] <= tok_cell[:, None]) & (cell_pos[None, :] <= tok_pos[:, None])   # (T, n)
    out = np.empty((T, n_head, hd), np.float32)
    q16 = R.f32_to_f16(q).astype(np.float64)
    for g in range(n_head_kv):
        K = k16[:, g * hd:(g + 1) * hd].astype(np.float64)
        V = v16[:, g * hd:(g + 1) * hd].astype(np.float64)
        s = (q16[:, g * r:(g + 1) * r] @ K.T).astype(np.float32)                 # (T, r, n)
        w = (s * scale).astype(np.float32)
        w = np.where(vis[:, None, :], w, np.float32(-np.inf))
        mx = w.max(axis=-1, keepdims=True)
        e = np.exp((w - mx).astype(np.float32)).astype(np.float32)
        tot = e.astype(np.float64).sum(axis=-1, keepdims=True)
        p = (e * (1.0 / tot).astype(np.float32)).astype(np.float32)
        p16 = R.f32_to_f16(p).astype(np.float64)
        out[:, g * r:(g + 1) * r] = (p16 @ V).astype(np.float32)
    return out


@pytest.mark.parametrize("n_head,n_head_kv,hd", [(32, 32, 128), (32, 8, 128), (32, 4, 64), (8, 8, 64)])
@pytest.mark.parametrize("n_cells,ntok", [(512, 512), (1536, 512), (2048, 512), (700, 33)])
def test_attn_mfma_matches_oracle(gpu_lib, n_head, n_head_kv, hd, n_cells, ntok):
    """The batch's tokens are the cache's last ntok cells (a prompt continuing a context)."""
    rng = np.random.default_rng(n_cells + ntok + hd + n_head_kv)
    q = (rng.standard_normal((ntok, n_head, hd)) * 0.6).astype(np.float32)
    k16 = (rng.standard_normal((n_cells, n_head_kv * hd)) * 0.6).astype(np.float16)
    v16 = rng.standard_normal((n_cells, n_head_kv * hd)).astype(np.float16)
    tc = np.arange(n_cells - ntok, n_cells, dtype=np.int32)
    cp = np.arange(n_cells, dtype=np.int32)
    got = engine.op_attention_batch(q, k16, v16, n_head_kv, tc, tc, cp)
    ref = attn_batch_ref(q, k16, v16, n_head_kv, tc, tc, cp)
    err = np.abs(got - ref)
    assert err.max() <= 2.0 ** -10 * np.abs(v16.astype(np.float32)).max(), float(err.max())
    assert err.mean() <= 1e-5, float(err.mean())


def test_attn_mfma_masks_by_position(gpu_lib):
    """Cells whose position is past a token's (a shuffled Self-Extend / seq_add layout) are
    masked in the batch kernel too."""
    rng = np.random.default_rng(11)
    n_cells, ntok = 900, 100
    q = (rng.standard_normal((ntok, 32, 128)) * 0.5).astype(np.float32)
    k16 = (rng.standard_normal((n_cells, 8 * 128)) * 0.5).astype(np.float16)
    v16 = rng.standard_normal((n_cells, 8 * 128)).astype(np.float16)
    cp = rng.permutation(n_cells).astype(np.int32)
    tc = np.arange(n_cells - ntok, n_cells, dtype=np.int32)
    tpos = cp[tc].copy()
    got = engine.op_attention_batch(q, k16, v16, 8, tc, tpos, cp)
    ref = attn_batch_ref(q, k16, v16, 8, tc, tpos, cp)
    assert np.abs(got - ref).max() <= 2.0 ** -10 * np.abs(v16.astype(np.float32)).max()
