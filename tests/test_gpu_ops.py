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
