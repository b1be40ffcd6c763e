"""Op-level parity of the decode step's streaming GEMV (blama_amd/csrc/dgemv.hip, mi_op_dgemv)
against the CPU restatement (oracle/ggml_ref.py): every instantiation the step's dispatcher
(dv_fn) can return -- role {Q/K/V, residual add, SwiGLU pair, store} x chunks per row
C in {1, 2, 3, 4, 6, 7} (K = 256 ... 14336) x weight type, and the mixed-type Q/K/V launches
(Q4_K + Q6_K, Q4_K + Q8_0, Q5_K + Q6_K) -- at the BASELINE models' real widths; and the residual
add whose workgroups quantise x themselves (DV_ADDQ, the small models' FFN down) bit-identical to
the one fed by dv_quant_kernel.

The activation is quantised on the device by dv_quant_kernel (bit-exact with quantize_row_q8_K /
the x86 quantize_row_q8_0, test_gpu_ops.py), so every per-block integer dot equals the CPU's; only
the fp32 order of the per-superblock partials differs: GEMV_TOL = 2e-5 relative to sum |terms|,
the bar of test_gpu_ops.py::test_gemv_matches_oracle."""
import numpy as np
import pytest

import ggml_ref as R
from blama_amd import engine
from util import rand_matrix, rand_x

pytestmark = pytest.mark.gpu

GEMV_TOL = 2e-5
ROLE_QKV, ROLE_ADD, ROLE_SWIGLU, ROLE_STORE, ROLE_ADDQ = 0, 1, 2, 3, 4


def _ref(t, w, K, x, sel=None):
    if sel is not None:
        w = w.reshape(-1, R.row_bytes(t, K))[sel].reshape(-1)
    return R.mul_mat_vec(w, t, K, x).astype(np.float64), R.mul_mat_vec_abs(w, t, K, x)


def _sel(rows):
    # the oracle on a row subset for the large matrices (every workgroup's range is still sampled)
    return None if rows <= 4096 else np.unique(np.r_[np.arange(0, rows, 5), np.arange(rows - 40, rows)])


def _check(got, ref, absb, what):
    err = np.abs(got.astype(np.float64) - ref)
    bound = absb * GEMV_TOL + 1e-30
    assert np.all(err <= bound), (what, float((err / bound).max()))


# K -> C = ceil(K / 2048) (5 -> 6): 256 -> 1, 4096 -> 2, 5632 -> 3, 8192 -> 4, 11008 -> 6, 14336 -> 7
@pytest.mark.parametrize("t", [R.Q4_K, R.Q5_K, R.Q6_K, R.Q8_0])
@pytest.mark.parametrize("rows,K", [(64, 256), (4096, 4096), (2048, 5632), (512, 8192), (4096, 11008), (4096, 14336)])
def test_dgemv_residual_add(gpu_lib, t, rows, K):
    w = rand_matrix(t, rows, K, seed=rows + K + t)
    x = rand_x(K, seed=K + 3)
    res = rand_x(rows, seed=rows + 1)
    y = engine.op_dgemv(ROLE_ADD, t, w, rows, K, x, resid=res)
    sel = _sel(rows)
    ref, absb = _ref(t, w, K, x, sel)
    r = (res if sel is None else res[sel]).astype(np.float64)
    got = (y if sel is None else y[sel]).astype(np.float64)
    # y = fl(dot + resid): the GEMV bound plus the rounding of the add
    bound = absb * GEMV_TOL + (np.abs(ref) + np.abs(r)) * 1.2e-7 + 1e-30
    err = np.abs(got - (ref + r))
    assert np.all(err <= bound), (R.TYPE_NAME[t], rows, K, float((err / bound).max()))


# DV_ADDQ runs dv_quant_kernel's no-norm arithmetic per 256-block in each workgroup: same bits
@pytest.mark.parametrize("t", [R.Q4_K, R.Q5_K, R.Q6_K, R.Q8_0])
@pytest.mark.parametrize("rows,K", [(64, 256), (2048, 5632), (512, 8192), (4096, 11008), (1024, 14336)])
def test_dgemv_residual_add_inlaunch_quant(gpu_lib, t, rows, K):
    w = rand_matrix(t, rows, K, seed=rows + K + t + 7)
    x = rand_x(K, seed=K + 5)
    res = rand_x(rows, seed=rows + 2)
    y1 = engine.op_dgemv(ROLE_ADD, t, w, rows, K, x, resid=res)
    y4 = engine.op_dgemv(ROLE_ADDQ, t, w, rows, K, x, resid=res)
    assert np.array_equal(y1.view(np.uint32), y4.view(np.uint32)), (R.TYPE_NAME[t], rows, K)


@pytest.mark.parametrize("t", [R.Q4_K, R.Q5_K, R.Q6_K, R.Q8_0])
@pytest.mark.parametrize("rows,K", [(32000, 4096), (96, 256), (256, 8192)])
def test_dgemv_store(gpu_lib, t, rows, K):
    w = rand_matrix(t, rows, K, seed=rows * 3 + K + t)
    x = rand_x(K, seed=K + 5)
    y = engine.op_dgemv(ROLE_STORE, t, w, rows, K, x)
    sel = _sel(rows)
    ref, absb = _ref(t, w, K, x, sel)
    _check(y if sel is None else y[sel], ref, absb, f"STORE {R.TYPE_NAME[t]} {rows}x{K}")


@pytest.mark.parametrize("t", [R.Q4_K, R.Q5_K, R.Q6_K, R.Q8_0])
@pytest.mark.parametrize("rows,K", [(11008, 4096), (14336, 4096), (128, 256), (512, 8192)])
def test_dgemv_swiglu_pair(gpu_lib, t, rows, K):
    wg = rand_matrix(t, rows, K, seed=rows + 11 + t)
    wu = rand_matrix(t, rows, K, seed=rows + 12 + t)
    x = rand_x(K, seed=K + 7)
    y = engine.op_dgemv(ROLE_SWIGLU, t, wg, rows, K, x, type2=t, raw2=wu, rows2=rows)
    sel = _sel(rows)
    g, ga = _ref(t, wg, K, x, sel)
    u, ua = _ref(t, wu, K, x, sel)
    # silu(g) * u in fp32 (ggml_vec_swiglu_f32 of b5187: silu then mul); the bound propagates
    # the GEMV bounds of g and u through the product
    g32, u32 = g.astype(np.float32), u.astype(np.float32)
    ref = (g32 / (np.float32(1) + np.exp(-g32))) * u32
    sg = 1.0 / (1.0 + np.exp(-g))
    dsilu = np.abs(sg * (1 + g * (1 - sg)))
    bound = (dsilu * np.abs(u) * ga + np.abs(g * sg) * ua) * GEMV_TOL + np.abs(ref) * 3e-7 + 1e-30
    got = (y if sel is None else y[sel]).astype(np.float64)
    err = np.abs(got - ref.astype(np.float64))
    assert np.all(err <= bound), (R.TYPE_NAME[t], rows, K, float((err / bound).max()))


# Q/K/V launches (no RoPE here: every row a Q row; RoPE and the KV append are checked end to end):
# one type, and the mixed launches of the Q4_K_M / Q5_K_M / Mixtral mixes
@pytest.mark.parametrize("t0,t1", [(R.Q4_K, None), (R.Q5_K, None), (R.Q6_K, None), (R.Q8_0, None),
                                   (R.Q4_K, R.Q6_K), (R.Q4_K, R.Q8_0), (R.Q5_K, R.Q6_K), (R.Q5_K, R.Q8_0),
                                   (R.Q6_K, R.Q8_0)])
@pytest.mark.parametrize("rows0,rows1,K", [(8192, 4096, 4096), (4096, 2048, 4096), (256, 128, 256)])
def test_dgemv_qkv_segments(gpu_lib, t0, t1, rows0, rows1, K):
    w0 = rand_matrix(t0, rows0, K, seed=rows0 + K + t0)
    x = rand_x(K, seed=K + 9)
    if t1 is None:
        y = engine.op_dgemv(ROLE_QKV, t0, w0, rows0, K, x)
        ref, absb = _ref(t0, w0, K, x)
        _check(y, ref, absb, f"QKV {R.TYPE_NAME[t0]}")
        return
    w1 = rand_matrix(t1, rows1, K, seed=rows1 + K + t1)
    y = engine.op_dgemv(ROLE_QKV, t0, w0, rows0, K, x, type2=t1, raw2=w1, rows2=rows1)
    r0, a0 = _ref(t0, w0, K, x)
    r1, a1 = _ref(t1, w1, K, x)
    _check(y[:rows0], r0, a0, f"QKV seg 0 {R.TYPE_NAME[t0]}")
    _check(y[rows0:], r1, a1, f"QKV seg 1 {R.TYPE_NAME[t1]}")
