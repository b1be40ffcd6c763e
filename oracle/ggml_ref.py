"""CPU restatement of the ggml CPU arithmetic that Blama's verifier path runs.

TEST INFRASTRUCTURE ONLY.  Nothing in ``blama_amd/`` imports this module; only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
use it, and only as the checker.

What it restates
----------------
Blama never does arithmetic itself: every FLOP of the hot path is inside the
third-party dependency **llama.cpp tag b5187** (pinned at
``/root/reference/inference/code/CMakeLists.txt:35``), which is *not present* in
this container.  The functions below restate the published
algorithms of that tag's CPU backend (``ggml/src/ggml-quants.c``,
``ggml/src/ggml-cpu/ggml-cpu-quants.c``, ``ggml/src/ggml-cpu/ops`` in
``ggml-cpu.c``) and of ``src/llama-graph.cpp`` / ``src/llama-model.cpp``
(``llm_build_llama``, and ``llm_build_gpt2`` for SURVEY.md §8 row f4) and are anchored
on the reference's call sites:

* ``Model::Params{.gpu=false}`` selects this CPU path
  (``inference/code/llama/Model.cpp:13-16,28``);
* ``llama_decode`` is called at ``inference/code/llama/Session.cpp:388``;
* logits are read at ``Session.cpp:24`` and top-10 extracted at
  ``Session.cpp:254-260`` (full sort, descending);
* the verify gather is ``Session.cpp:263-282``;
* LogitComparer / MetricsAggregator: ``LogitComparer.cpp:8-128``.

Pinning
-------
The only golden vector the reference holds that runs without model files is
the LogitComparer known-answer test ``inference/test/t-LogitComparer.cpp:13-39``
(pinned in ``tests/test_oracle.py``).  The quant formats, the integer
dot products and the llama graph are **parity unpinned**: no reference test
covers Q4_K/Q5_K/Q6_K/Q8_0 LLaMA arithmetic, and ggml itself cannot be built
here.  Parity for those rows rests on this restatement,
cross-checked against the independent C restatement in ``oracle/ggml_cpu.c``.

Floating point conventions mirrored from ggml's CPU build (C11, so
``-ffp-contract=off``: no FMA contraction in scalar code):

* fp16 <-> fp32 via round-to-nearest-even (``_cvtss_sh(x, 0)`` / F16C);
* activations are quantised to Q8_K for K-quant weights
  (``quantize_row_q8_K_ref``) and to Q8_0 for Q8_0 weights (the x86 SIMD form of
  ``quantize_row_q8_0``: ``id = 127/amax``, round-to-nearest-even);
* the block dot products are exact integer sums per (sub-)block combined in
  float; this restatement combines them in float64 ("the exact value"), ggml
  and the GPU both land within fp32 rounding of it;
* ``rms_norm`` and ``soft_max`` accumulate in double (``ggml_float``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

QK_K = 256
QK8_0 = 32

# ggml_type ids (ggml.h, b5187)
F32, F16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1 = 0, 1, 2, 3, 6, 7, 8, 9
Q2_K, Q3_K, Q4_K, Q5_K, Q6_K, Q8_K = 10, 11, 12, 13, 14, 15
BF16 = 30

TYPE_NAME = {F32: "F32", F16: "F16", Q8_0: "Q8_0", Q4_K: "Q4_K", Q5_K: "Q5_K",
             Q6_K: "Q6_K", Q8_K: "Q8_K", BF16: "BF16"}

# (elements per block, bytes per block) -- ggml-common.h block structs
BLOCK = {
    F32: (1, 4),
    F16: (1, 2),
    Q8_0: (32, 34),     # f16 d; i8 qs[32]
    Q4_K: (256, 144),   # f16 d; f16 dmin; u8 scales[12]; u8 qs[128]
    Q5_K: (256, 176),   # f16 d; f16 dmin; u8 scales[12]; u8 qh[32]; u8 qs[128]
    Q6_K: (256, 210),   # u8 ql[128]; u8 qh[64]; i8 scales[16]; f16 d
}


def row_bytes(t: int, k: int) -> int:
    n, b = BLOCK[t]
    assert k % n == 0, (t, k)
    return k // n * b


def f16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(b).view(np.float16).astype(np.float32)


def f32_to_f16(x) -> np.ndarray:
    """GGML_FP32_TO_FP16: round to nearest even (numpy's cast is RNE)."""
    return np.asarray(x, dtype=np.float32).astype(np.float16)


# --------------------------------------------------------------------------
# Block unpacking helpers
# --------------------------------------------------------------------------

def _blocks(raw: np.ndarray, t: int) -> np.ndarray:
    n, b = BLOCK[t]
    raw = np.ascontiguousarray(raw, dtype=np.uint8).reshape(-1)
    assert raw.size % b == 0
    return raw.reshape(-1, b)


def get_scale_min_k4(scales: np.ndarray):
    """ggml-quants.c get_scale_min_k4 for all j=0..7 at once.

    scales: (nb, 12) uint8 -> (sc, m) each (nb, 8) int32.
    j<4:  sc = s[j]&63, m = s[j+4]&63
    j>=4: sc = (s[j+4]&0xF) | ((s[j-4]>>6)<<4), m = (s[j+4]>>4) | ((s[j]>>6)<<4)
    """
    s = scales.astype(np.int32)
    sc = np.empty((s.shape[0], 8), np.int32)
    m = np.empty((s.shape[0], 8), np.int32)
    for j in range(4):
        sc[:, j] = s[:, j] & 63
        m[:, j] = s[:, j + 4] & 63
    for j in range(4, 8):
        sc[:, j] = (s[:, j + 4] & 0xF) | ((s[:, j - 4] >> 6) << 4)
        m[:, j] = (s[:, j + 4] >> 4) | ((s[:, j] >> 6) << 4)
    return sc, m


def unpack_q4_K(raw):
    """-> d (nb,) f32, dmin (nb,) f32, sc (nb,8), m (nb,8), q (nb,256) int32 in [0,15]."""
    bl = _blocks(raw, Q4_K)
    d = f16_bits_to_f32(bl[:, 0:2].copy()).reshape(-1)
    dmin = f16_bits_to_f32(bl[:, 2:4].copy()).reshape(-1)
    sc, m = get_scale_min_k4(bl[:, 4:16])
    qs = bl[:, 16:144].astype(np.int32).reshape(-1, 4, 32)  # 4 chunks of 64 elems
    q = np.empty((bl.shape[0], 4, 64), np.int32)
    q[:, :, :32] = qs & 0xF
    q[:, :, 32:] = qs >> 4
    return d, dmin, sc, m, q.reshape(-1, 256)


def unpack_q5_K(raw):
    bl = _blocks(raw, Q5_K)
    d = f16_bits_to_f32(bl[:, 0:2].copy()).reshape(-1)
    dmin = f16_bits_to_f32(bl[:, 2:4].copy()).reshape(-1)
    sc, m = get_scale_min_k4(bl[:, 4:16])
    qh = bl[:, 16:48].astype(np.int32)             # (nb, 32)
    qs = bl[:, 48:176].astype(np.int32).reshape(-1, 4, 32)
    q = np.empty((bl.shape[0], 4, 64), np.int32)
    for c in range(4):
        q[:, c, :32] = (qs[:, c] & 0xF) + (((qh >> (2 * c)) & 1) << 4)
        q[:, c, 32:] = (qs[:, c] >> 4) + (((qh >> (2 * c + 1)) & 1) << 4)
    return d, dmin, sc, m, q.reshape(-1, 256)


def unpack_q6_K(raw):
    """-> d (nb,), sc (nb,16) int32 signed, q (nb,256) int32 in [-32,31]."""
    bl = _blocks(raw, Q6_K)
    ql = bl[:, 0:128].astype(np.int32)
    qh = bl[:, 128:192].astype(np.int32)
    sc = bl[:, 192:208].view(np.int8).astype(np.int32)
    d = f16_bits_to_f32(bl[:, 208:210].copy()).reshape(-1)
    q = np.empty((bl.shape[0], 256), np.int32)
    for h in range(2):
        L = ql[:, 64 * h: 64 * h + 64]
        H = qh[:, 32 * h: 32 * h + 32]
        base = 128 * h
        q[:, base + 0: base + 32] = ((L[:, :32] & 0xF) | (((H >> 0) & 3) << 4)) - 32
        q[:, base + 32: base + 64] = ((L[:, 32:] & 0xF) | (((H >> 2) & 3) << 4)) - 32
        q[:, base + 64: base + 96] = ((L[:, :32] >> 4) | (((H >> 4) & 3) << 4)) - 32
        q[:, base + 96: base + 128] = ((L[:, 32:] >> 4) | (((H >> 6) & 3) << 4)) - 32
    return d, sc, q


def unpack_q8_0(raw):
    bl = _blocks(raw, Q8_0)
    d = f16_bits_to_f32(bl[:, 0:2].copy()).reshape(-1)
    q = bl[:, 2:34].view(np.int8).astype(np.int32)
    return d, q


# --------------------------------------------------------------------------
# dequantize_row_* (ggml-quants.c) -- used by get_rows (token embedding)
# --------------------------------------------------------------------------

def dequantize(raw: np.ndarray, t: int) -> np.ndarray:
    """Exact float32 restatement of dequantize_row_{q4_K,q5_K,q6_K,q8_0,f16,f32}.

    Operation order follows ggml-quants.c with no FMA contraction:
    q4_K/q5_K: y = (d*sc)*q - (dmin*m);  q6_K: y = (d*sc)*q;  q8_0: y = q*d.
    """
    if t == F32:
        return np.ascontiguousarray(raw).view(np.float32).reshape(-1).copy()
    if t == F16:
        return np.ascontiguousarray(raw).view(np.float16).astype(np.float32).reshape(-1)
    if t in (Q4_K, Q5_K):
        d, dmin, sc, m, q = (unpack_q4_K if t == Q4_K else unpack_q5_K)(raw)
        d1 = (d[:, None] * sc.astype(np.float32)).astype(np.float32)     # (nb,8)
        m1 = (dmin[:, None] * m.astype(np.float32)).astype(np.float32)
        d1 = np.repeat(d1, 32, axis=1)
        m1 = np.repeat(m1, 32, axis=1)
        y = (d1 * q.astype(np.float32)).astype(np.float32) - m1
        return y.astype(np.float32).reshape(-1)
    if t == Q6_K:
        d, sc, q = unpack_q6_K(raw)
        ds = (d[:, None] * sc.astype(np.float32)).astype(np.float32)      # (nb,16)
        ds = np.repeat(ds, 16, axis=1)
        return (ds * q.astype(np.float32)).astype(np.float32).reshape(-1)
    if t == Q8_0:
        d, q = unpack_q8_0(raw)
        return (q.astype(np.float32) * d[:, None]).astype(np.float32).reshape(-1)
    raise NotImplementedError(TYPE_NAME.get(t, t))


# --------------------------------------------------------------------------
# Activation quantisation (the CPU's vec_dot_type conversion)
# --------------------------------------------------------------------------

@dataclass
class Q8K:
    d: np.ndarray      # (nb,) f32
    qs: np.ndarray     # (nb,256) int32 (values in [-127,127])
    bsums: np.ndarray  # (nb,16) int32


def quantize_q8_K(x: np.ndarray) -> Q8K:
    """quantize_row_q8_K_ref (ggml-quants.c): per 256 block,
    max = signed value of largest |x| (first on ties), iscale = -127/max,
    q = min(127, nearest_int(iscale*x)), d = 1/iscale, bsums per 16."""
    x = np.asarray(x, np.float32).reshape(-1, QK_K)
    ax = np.abs(x)
    idx = np.argmax(ax, axis=1)
    rows = np.arange(x.shape[0])
    amax = ax[rows, idx]
    mx = x[rows, idx]
    zero = amax == 0
    with np.errstate(divide="ignore", invalid="ignore"):
        iscale = (np.float32(-127.0) / mx).astype(np.float32)
        q = np.rint((iscale[:, None] * x).astype(np.float32))
        q = np.minimum(q, 127).astype(np.int32)
        d = (np.float32(1.0) / iscale).astype(np.float32)
    q[zero] = 0
    d[zero] = 0
    bsums = q.reshape(-1, 16, 16).sum(axis=2).astype(np.int32)
    return Q8K(d=d.astype(np.float32), qs=q, bsums=bsums)


@dataclass
class Q80:
    d: np.ndarray   # (nb,) f32 (already rounded through fp16)
    qs: np.ndarray  # (nb,32) int32


def quantize_q8_0(x: np.ndarray) -> Q80:
    """x86 SIMD form of quantize_row_q8_0 (ggml-cpu-quants.c, AVX2 branch):
    amax over 32, d = fp16(amax/127), id = 127/amax (0 if amax==0),
    q = round_nearest_even(x*id)."""
    x = np.asarray(x, np.float32).reshape(-1, QK8_0)
    amax = np.abs(x).max(axis=1).astype(np.float32)
    d = f32_to_f16(amax / np.float32(127.0)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(amax != 0, np.float32(127.0) / amax, np.float32(0)).astype(np.float32)
    q = np.rint((x * idv[:, None]).astype(np.float32)).astype(np.int32)
    return Q80(d=d, qs=q)


# --------------------------------------------------------------------------
# vec_dot_*: exact per-block integer sums, combined in float64
# --------------------------------------------------------------------------

def block_sums(raw: np.ndarray, t: int, K: int, x: np.ndarray):
    """For a weight matrix raw (M rows, row-major GGUF blocks) and activation x
    return (coef, isum) with y[r] = sum_b coef[r,b] * isum[r,b] (float64).

    The integer parts are exactly what vec_dot_{q4_K,q5_K,q6_K}_q8_K /
    vec_dot_q8_0_q8_0 (ggml-cpu-quants.c) compute; coef are the float32
    products the CPU forms (y.d * fp16(x.d) etc.)."""
    M = np.asarray(raw).reshape(-1).size // row_bytes(t, K)
    if t in (Q4_K, Q5_K):
        a = quantize_q8_K(x)
        nb = K // QK_K
        d, dmin, sc, m, q = (unpack_q4_K if t == Q4_K else unpack_q5_K)(raw)
        q = q.reshape(M, nb, 8, 32).astype(np.int64)
        a8 = a.qs.reshape(1, nb, 8, 32).astype(np.int64)
        dots = (q * a8).sum(-1)                                     # (M,nb,8)
        S = (dots * sc.reshape(M, nb, 8)).sum(-1)                   # (M,nb)
        bs32 = a.bsums.reshape(nb, 8, 2).sum(-1).astype(np.int64)   # per 32-subblock
        Mi = (m.reshape(M, nb, 8).astype(np.int64) * bs32[None]).sum(-1)
        cd = (d.reshape(M, nb) * a.d[None]).astype(np.float32)
        cm = (dmin.reshape(M, nb) * a.d[None]).astype(np.float32)
        return [(cd, S), (-cm.astype(np.float64), Mi)]
    if t == Q6_K:
        a = quantize_q8_K(x)
        nb = K // QK_K
        d, sc, q = unpack_q6_K(raw)
        q = q.reshape(M, nb, 16, 16).astype(np.int64)
        a8 = a.qs.reshape(1, nb, 16, 16).astype(np.int64)
        S = ((q * a8).sum(-1) * sc.reshape(M, nb, 16)).sum(-1)
        cd = (d.reshape(M, nb) * a.d[None]).astype(np.float32)
        return [(cd, S)]
    if t == Q8_0:
        a = quantize_q8_0(x)
        nb = K // QK8_0
        d, q = unpack_q8_0(raw)
        S = (q.reshape(M, nb, 32).astype(np.int64) * a.qs.reshape(1, nb, 32)).sum(-1)
        cd = (d.reshape(M, nb) * a.d[None]).astype(np.float32)
        return [(cd, S)]
    raise NotImplementedError(TYPE_NAME.get(t, t))


def mul_mat_vec(raw: np.ndarray, t: int, K: int, x: np.ndarray) -> np.ndarray:
    """ggml_mul_mat(W, x) for one activation column on the CPU backend:
    y[M] = W[M x K] . x[K] with x quantised to W's vec_dot_type."""
    x = np.asarray(x, np.float32).reshape(-1)
    assert x.size == K
    if t == F32:
        W = np.ascontiguousarray(raw).view(np.float32).reshape(-1, K)
        return (W.astype(np.float64) @ x.astype(np.float64)).astype(np.float32)
    if t == F16:
        # vec_dot_type of F16 is F16: x is rounded to fp16 first
        W = np.ascontiguousarray(raw).view(np.float16).reshape(-1, K).astype(np.float64)
        return (W @ f32_to_f16(x).astype(np.float64)).astype(np.float32)
    acc = None
    for coef, isum in block_sums(raw, t, K, x):
        part = (coef.astype(np.float64) * isum.astype(np.float64)).sum(-1)
        acc = part if acc is None else acc + part
    return acc.astype(np.float32)


def mul_mat_vec_abs(raw: np.ndarray, t: int, K: int, x: np.ndarray) -> np.ndarray:
    """sum_b |coef*isum| per row: the scale of the fp32 rounding error budget."""
    x = np.asarray(x, np.float32).reshape(-1)
    if t in (F32, F16):
        W = np.ascontiguousarray(raw).view(np.float32 if t == F32 else np.float16)
        return (np.abs(W.reshape(-1, K).astype(np.float64)) @ np.abs(x.astype(np.float64)))
    acc = None
    for coef, isum in block_sums(raw, t, K, x):
        part = np.abs(coef.astype(np.float64) * isum.astype(np.float64)).sum(-1)
        acc = part if acc is None else acc + part
    return acc


# --------------------------------------------------------------------------
# Element-wise / normalisation ops (ggml-cpu.c)
# --------------------------------------------------------------------------

def rms_norm(x: np.ndarray, eps: float) -> np.ndarray:
    """ggml_compute_forward_rms_norm_f32: sum of float squares in double,
    mean = (float)(sum/n), scale = 1.0f/sqrtf(mean+eps), y = x*scale."""
    x = np.asarray(x, np.float32)
    sq = (x * x).astype(np.float32).astype(np.float64)
    s = float(np.sum(sq))          # order differs from a serial loop only in the double's last bits
    mean = np.float32(s / x.size)
    scale = np.float32(1.0) / np.sqrt(np.float32(mean + np.float32(eps)), dtype=np.float32)
    return (x * np.float32(scale)).astype(np.float32)


def layer_norm(x: np.ndarray, eps: float) -> np.ndarray:
    """ggml_compute_forward_norm_f32 (ggml-cpu.c, b5187): sum in double, mean = (float)(sum/n);
    v = x - mean (f32), y = v, sum2 += (double)(v*v) (the square rounded to f32 first);
    variance = (float)(sum2/n); y *= 1.0f/sqrtf(variance + eps).  build_norm (LLM_NORM) then
    multiplies by the weight and adds the bias as separate f32 ops (ggml_mul, ggml_add)."""
    x = np.asarray(x, np.float32)
    n = x.shape[-1]
    mean = np.float32(np.sum(x.astype(np.float64)) / n)
    v = (x - mean).astype(np.float32)
    sum2 = np.sum((v * v).astype(np.float32).astype(np.float64))
    var = np.float32(sum2 / n)
    scale = np.float32(1.0) / np.sqrt(np.float32(var + np.float32(eps)), dtype=np.float32)
    return (v * scale).astype(np.float32)


_GELU_TAB = None


def gelu_table() -> np.ndarray:
    """ggml_table_gelu_f16 (ggml-cpu.c init, GGML_GELU_FP16 is defined in b5187): for every f16
    bit pattern u, fp16(ggml_gelu_f32(fp32(u))) with ggml_gelu_f32(x) =
    0.5f*x*(1.0f + tanhf(SQRT_2_OVER_PI*x*(1.0f + GELU_COEF_A*x*x))), evaluated in f32 with the C
    library's tanhf (the same call the reference's x86 build makes).  Returns uint16[65536]."""
    global _GELU_TAB
    if _GELU_TAB is None:
        import ctypes
        libm = ctypes.CDLL("libm.so.6")
        libm.tanhf.restype = ctypes.c_float
        libm.tanhf.argtypes = [ctypes.c_float]
        xs = np.arange(65536, dtype=np.uint16).view(np.float16).astype(np.float32)
        xs = np.where(np.isfinite(xs), xs, np.float32(0.0)).astype(np.float32)   # inf/nan rows: unused
        a = np.float32(0.044715)
        k = np.float32(0.79788456080286535587989211986876)
        inner = (k * xs).astype(np.float32) * ((np.float32(1.0) + (a * xs).astype(np.float32) * xs)
                                               .astype(np.float32))
        inner = inner.astype(np.float32)
        th = np.array([libm.tanhf(float(v)) if np.isfinite(v) else (1.0 if v > 0 else -1.0) for v in inner],
                      np.float32)
        y = ((np.float32(0.5) * xs).astype(np.float32) * (np.float32(1.0) + th).astype(np.float32)).astype(np.float32)
        with np.errstate(invalid="ignore", over="ignore"):
            _GELU_TAB = y.astype(np.float16).view(np.uint16)
    return _GELU_TAB


def gelu(x: np.ndarray) -> np.ndarray:
    """ggml_vec_gelu_f32 with GGML_GELU_FP16: x <= -10 -> 0, x >= 10 -> x, else the f16 table at
    fp16(x)."""
    x = np.asarray(x, np.float32)
    t = gelu_table()[x.astype(np.float16).view(np.uint16)].view(np.float16).astype(np.float32)
    return np.where(x <= -10.0, np.float32(0.0), np.where(x >= 10.0, x, t)).astype(np.float32)


def silu(x: np.ndarray) -> np.ndarray:
    """ggml_silu_f32: x/(1+expf(-x)) (ggml's SIMD expf differs by <=1-2 ulp)."""
    x = np.asarray(x, np.float32)
    with np.errstate(over="ignore"):
        return (x / (np.float32(1.0) + np.exp(-x).astype(np.float32))).astype(np.float32)


def rope_theta_scale(freq_base: float, n_dims: int) -> np.float32:
    """theta_scale = powf(freq_base, -2.0f/n_dims) (ggml_compute_forward_rope_f32)."""
    return np.float32(np.power(np.float32(freq_base), np.float32(-2.0) / np.float32(n_dims),
                               dtype=np.float32))


def rope_cache(pos: int, n_dims: int, freq_base: float, freq_scale: float = 1.0,
               freq_factors=None):
    """ggml_rope_cache_init with ext_factor=0, mscale=1: theta starts at pos and
    is multiplied by theta_scale once per pair (iterated float multiply)."""
    ts = rope_theta_scale(freq_base, n_dims)
    theta = np.float32(pos)
    cos = np.empty(n_dims // 2, np.float32)
    sin = np.empty(n_dims // 2, np.float32)
    for i in range(n_dims // 2):
        ff = np.float32(1.0) if freq_factors is None else np.float32(freq_factors[i])
        th = np.float32(np.float32(freq_scale) * np.float32(theta / ff))
        cos[i] = np.float32(math.cos(float(th)))
        sin[i] = np.float32(math.sin(float(th)))
        theta = np.float32(theta * ts)
    return cos, sin


def rope_norm(x: np.ndarray, pos: int, n_dims: int, freq_base: float, freq_factors=None):
    """mode 0 (NORM): rotate adjacent pairs (x[2i], x[2i+1]) of each head.
    x: (n_heads, head_dim)."""
    x = np.asarray(x, np.float32)
    cos, sin = rope_cache(pos, n_dims, freq_base, freq_factors=freq_factors)
    y = x.copy()
    x0 = x[:, 0:n_dims:2]
    x1 = x[:, 1:n_dims:2]
    y[:, 0:n_dims:2] = (x0 * cos - x1 * sin).astype(np.float32)
    y[:, 1:n_dims:2] = (x0 * sin + x1 * cos).astype(np.float32)
    return y


def soft_max(s: np.ndarray, scale: float) -> np.ndarray:
    """ggml_compute_forward_soft_max_f32 (no mask/alibi needed for batch-1
    causal decode): w = s*scale; max; e = expf(w-max); sum in double;
    p = e * (float)(1.0/sum)."""
    w = (np.asarray(s, np.float32) * np.float32(scale)).astype(np.float32)
    mx = np.float32(w.max())
    e = np.exp((w - mx).astype(np.float32)).astype(np.float32)
    tot = float(np.sum(e.astype(np.float64)))
    return (e * np.float32(1.0 / tot)).astype(np.float32)


def attention_head(q: np.ndarray, K16: np.ndarray, V16: np.ndarray, scale: float) -> np.ndarray:
    """One head of KQ -> soft_max -> KQV on the CPU backend (flash_attn=false,
    Instance.hpp:25): K,V are the f16 cache rows; ggml_mul_mat converts the
    f32 operand to the f16 vec_dot_type, so q and the probabilities are
    rounded to fp16 before their dot products."""
    q16 = f32_to_f16(q).astype(np.float64)
    s = (K16.astype(np.float64) @ q16).astype(np.float32)
    p = soft_max(s, scale)
    p16 = f32_to_f16(p).astype(np.float64)
    return (p16 @ V16.astype(np.float64)).astype(np.float32)


# --------------------------------------------------------------------------
# Top-k / gather (Session.cpp:246-282) and LogitComparer (LogitComparer.cpp)
# --------------------------------------------------------------------------

def topk(logits: np.ndarray, k: int):
    """Session::getLogitsFromCtx(int topK) (Session.cpp:246-261): full sort by
    logit descending; ties (left unspecified by std::sort) are ordered by id
    ascending in this build."""
    logits = np.asarray(logits, np.float32)
    order = np.lexsort((np.arange(logits.size), -logits.astype(np.float64)))[:k]
    return [(int(i), float(logits[i])) for i in order]


def gather(logits: np.ndarray, ids):
    """Session::getLogitsFromCtx(TokenDataVector) (Session.cpp:263-282): the
    logits at the claimed ids (set semantics of the any_of scan), sorted desc."""
    idset = sorted(set(int(i) for i in ids))
    res = [(i, float(np.float32(logits[i]))) for i in idset]
    res.sort(key=lambda t: (-t[1], t[0]))
    return res


def _softmax_map(data):
    # LogitComparer.cpp:8-28 -- uses data[0] as the max (assumes sorted desc)
    mx = np.float32(data[0][1])
    res = {}
    tot = np.float32(0.0)
    for tok, logit in data:
        p = np.float32(np.exp(np.float32(np.float32(logit) - mx)))
        res[tok] = p
        tot = np.float32(tot + p)
    return {k: np.float32(v / tot) for k, v in res.items()}


def _euclid_sq(data):
    # LogitComparer.cpp:106-115
    d = np.float32(0.0)
    for _, logit in data:
        d = np.float32(d + np.float32(logit) * np.float32(logit))
    return d


def _jsd(p1, p2):
    # LogitComparer.cpp:82-104 (natural log, over the id intersection)
    avg = {t: np.float32((p + p2[t]) / np.float32(2.0)) for t, p in p1.items() if t in p2}

    def kl(P, Q):
        k = np.float32(0.0)
        for t, p in P.items():
            if p > 0 and t in Q and Q[t] > 0:
                k = np.float32(k + p * np.float32(np.log(np.float32(p / Q[t]))))
        return k
    return np.float32((kl(p1, avg) + kl(p2, avg)) / np.float32(2.0))


@dataclass
class ComparisonMetrics:
    top1Match: float
    distance: float
    jsd: float


def compare(data1, data2) -> ComparisonMetrics:
    """LogitComparer::compare (LogitComparer.cpp:39-55)."""
    top1 = 1.0 if data1[0][0] == data2[0][0] else 0.0
    n = min(len(data1), len(data2))
    d1 = _euclid_sq(data1[:n])
    d2 = _euclid_sq(data2[:n])
    with np.errstate(invalid="ignore", divide="ignore"):
        dist = np.float32(np.abs(np.float32(d1 - d2)) / max(d1, d2))
    return ComparisonMetrics(top1, float(dist), float(_jsd(_softmax_map(data1), _softmax_map(data2))))


def logit_similarity(data1, data2) -> float:
    """LogitComparer::logitSimilarity (LogitComparer.cpp:57-80)."""
    l2 = {t: np.float32(l) for t, l in data2}
    ws = np.float32(0.0)
    tw = np.float32(0.0)
    for t, l in data1:
        l = np.float32(l)
        w = np.float32(abs(l))
        sim = np.float32(0.0)
        if t in l2:
            sim = np.float32(1.0) - np.float32(abs(l - l2[t]) / abs(max(l, l2[t])))
        ws = np.float32(ws + w * sim)
        tw = np.float32(tw + w)
    return float(ws / tw) if tw > 0 else 0.0


class MetricsAggregator:
    """MetricsAggregator::pushAndVerify (LogitComparer.cpp:117-128)."""

    def __init__(self):
        self.metrics = []

    def push_and_verify(self, ms) -> float:
        self.metrics.extend(ms)
        total = 0.0
        for m in self.metrics:
            total += 0.5 * (1.0 - np.float32(m.distance)) + 0.5 * (1.0 - np.float32(m.jsd))
        return float(np.float32(total / len(self.metrics)))


# --------------------------------------------------------------------------
# The llama decode graph (llm_build_llama, llama.cpp b5187 src/llama-model.cpp)
# --------------------------------------------------------------------------

@dataclass
class Tensor:
    type: int
    shape: tuple          # ggml ne order: (ne0=K, ne1=rows, [ne2=experts])
    data: np.ndarray      # raw bytes (uint8) in GGUF layout


@dataclass
class HParams:
    n_vocab: int
    n_embd: int
    n_layer: int
    n_head: int
    n_head_kv: int
    n_ff: int
    n_ctx_train: int
    eps: float
    rope_base: float
    n_rot: int
    n_expert: int = 0
    n_expert_used: int = 0
    arch: str = "llama"      # "llama" (llm_build_llama) or "gpt2" (llm_build_gpt2)

    @property
    def head_dim(self):
        return self.n_embd // self.n_head


@dataclass
class LlamaOracle:
    """Batch-1 decode of the llama graph on the CPU restatement.

    tensors: name -> Tensor (GGUF names: token_embd.weight, blk.N.attn_q.weight, ...)."""
    hp: HParams
    tensors: dict
    n_ctx: int = 0
    kcache: list = field(default_factory=list)
    vcache: list = field(default_factory=list)
    n_past: int = 0          # cells in use
    cell_pos: list = field(default_factory=list)

    def __post_init__(self):
        if not self.n_ctx:
            self.n_ctx = self.hp.n_ctx_train
        kvd = self.hp.n_head_kv * self.hp.head_dim
        self.kcache = [np.zeros((self.n_ctx, kvd), np.float16) for _ in range(self.hp.n_layer)]
        self.vcache = [np.zeros((self.n_ctx, kvd), np.float16) for _ in range(self.hp.n_layer)]

    def _mm(self, name, x):
        t = self.tensors[name]
        return mul_mat_vec(t.data, t.type, t.shape[0], x)

    def _w(self, name):
        t = self.tensors[name]
        return dequantize(t.data, t.type)

    def _ffn(self, il, cur):
        hp = self.hp
        if hp.n_expert == 0:
            g = self._mm(f"blk.{il}.ffn_gate.weight", cur)
            u = self._mm(f"blk.{il}.ffn_up.weight", cur)
            h = (silu(g) * u).astype(np.float32)
            return self._mm(f"blk.{il}.ffn_down.weight", h)
        # build_moe_ffn (src/llama-graph.cpp): softmax gating, top-k, norm_w
        logits = self._mm(f"blk.{il}.ffn_gate_inp.weight", cur)
        probs = soft_max(logits, 1.0)
        sel = np.argsort(-probs, kind="stable")[: hp.n_expert_used]
        w = probs[sel].astype(np.float32)
        w = (w / np.float32(np.sum(w.astype(np.float32), dtype=np.float32))).astype(np.float32)
        out = None
        for slot, e in enumerate(sel):
            g = self._expert_mm(f"blk.{il}.ffn_gate_exps.weight", e, cur)
            u = self._expert_mm(f"blk.{il}.ffn_up_exps.weight", e, cur)
            h = (silu(g) * u).astype(np.float32)
            y = (self._expert_mm(f"blk.{il}.ffn_down_exps.weight", e, h) * w[slot]).astype(np.float32)
            out = y if out is None else (out + y).astype(np.float32)
        return out

    def _expert_mm(self, name, e, x):
        t = self.tensors[name]
        K, M = t.shape[0], t.shape[1]
        rb = row_bytes(t.type, K)
        raw = t.data.reshape(-1)[e * M * rb:(e + 1) * M * rb]
        return mul_mat_vec(raw, t.type, K, x)

    # ---- KV cache cell operations (llama_kv_self_seq_rm / seq_add / seq_div) ----
    def kv_seq_rm(self, p0, p1):
        p1 = 1 << 30 if p1 < 0 else p1
        keep = [c for c in range(self.n_past) if not (p0 <= self.cell_pos[c] < p1)]
        for il in range(self.hp.n_layer):
            self.kcache[il][: len(keep)] = self.kcache[il][keep]
            self.vcache[il][: len(keep)] = self.vcache[il][keep]
        self.cell_pos = [self.cell_pos[c] for c in keep]
        self.n_past = len(keep)

    def kv_seq_shift(self, p0, p1, delta=0, div=0):
        """seq_add (pos += delta) / seq_div (pos //= div) with the K-shift:
        cached f16 K re-rotated by the position delta (llama.cpp build_k_shift:
        ggml_rope_ext on the f16 cache view, result rounded back to f16)."""
        p1 = 1 << 30 if p1 < 0 else p1
        hd = self.hp.head_dim
        ff = self.tensors.get("rope_freqs.weight")
        ffv = None if ff is None else dequantize(ff.data, ff.type)
        for c in range(self.n_past):
            ps = self.cell_pos[c]
            if p0 <= ps < p1:
                npos = ps // div if div else ps + delta
                d = npos - ps
                self.cell_pos[c] = npos
                if d:
                    for il in range(self.hp.n_layer):
                        k = self.kcache[il][c].astype(np.float32).reshape(self.hp.n_head_kv, hd)
                        self.kcache[il][c] = f32_to_f16(rope_norm(k, d, self.hp.n_rot, self.hp.rope_base,
                                                                  ffv).reshape(-1))
        neg = [c for c in range(self.n_past) if self.cell_pos[c] < 0]
        if neg:
            self.kv_seq_rm(-(1 << 30), 0)

    def _row(self, name, r):
        t = self.tensors[name]
        rb = row_bytes(t.type, t.shape[0])
        return dequantize(t.data.reshape(-1)[r * rb:(r + 1) * rb], t.type)

    def _vec(self, name):
        return self._w(name).astype(np.float32)

    def _norm(self, x, name):
        """build_norm(LLM_NORM): layer_norm, * weight, + bias (separate f32 ops)."""
        y = (layer_norm(x, self.hp.eps) * self._vec(name + ".weight")).astype(np.float32)
        return (y + self._vec(name + ".bias")).astype(np.float32)

    def _decode_one_gpt2(self, token: int) -> np.ndarray:
        """llm_build_gpt2 (src/llama-model.cpp, b5187) for one token: token + learned position
        embedding; per layer LayerNorm -> fused QKV + bias -> attention (no RoPE) -> WO + bias
        -> residual; LayerNorm -> up + bias -> GELU -> down + bias -> residual; final LayerNorm
        and the output head (tied to token_embd when output.weight is absent)."""
        hp = self.hp
        hd = hp.head_dim
        d = hp.n_embd
        pos = (max(self.cell_pos) + 1) if self.n_past else 0
        cell = self.n_past
        assert cell < self.n_ctx and pos < hp.n_ctx_train
        x = (self._row("token_embd.weight", token) + self._row("position_embd.weight", pos)).astype(np.float32)
        scale = np.float32(1.0) / np.sqrt(np.float32(hd), dtype=np.float32)
        for il in range(hp.n_layer):
            b = f"blk.{il}."
            cur = self._norm(x, b + "attn_norm")
            qkv = (self._mm(b + "attn_qkv.weight", cur) + self._vec(b + "attn_qkv.bias")).astype(np.float32)
            q = qkv[:d].reshape(hp.n_head, hd)
            k = qkv[d:2 * d]
            v = qkv[2 * d:3 * d]
            self.kcache[il][cell] = f32_to_f16(k)
            self.vcache[il][cell] = f32_to_f16(v)
            vis = [c for c in range(cell + 1) if c == cell or self.cell_pos[c] <= pos]
            Kc = self.kcache[il][vis].reshape(len(vis), hp.n_head_kv, hd)
            Vc = self.vcache[il][vis].reshape(len(vis), hp.n_head_kv, hd)
            ratio = hp.n_head // hp.n_head_kv
            att = np.empty((hp.n_head, hd), np.float32)
            for h in range(hp.n_head):
                att[h] = attention_head(q[h], Kc[:, h // ratio], Vc[:, h // ratio], scale)
            cur = (self._mm(b + "attn_output.weight", att.reshape(-1)) + self._vec(b + "attn_output.bias")).astype(np.float32)
            x = (cur + x).astype(np.float32)
            cur = self._norm(x, b + "ffn_norm")
            u = (self._mm(b + "ffn_up.weight", cur) + self._vec(b + "ffn_up.bias")).astype(np.float32)
            hh = gelu(u)
            cur = (self._mm(b + "ffn_down.weight", hh) + self._vec(b + "ffn_down.bias")).astype(np.float32)
            x = (cur + x).astype(np.float32)
        cur = self._norm(x, "output_norm")
        out = self.tensors.get("output.weight", self.tensors["token_embd.weight"])
        logits = mul_mat_vec(out.data, out.type, out.shape[0], cur)
        self.cell_pos.append(pos)
        self.n_past += 1
        return logits

    def decode_one(self, token: int) -> np.ndarray:
        """One llama_decode of a single token at position max(pos)+1; returns logits f32[V]."""
        if self.hp.arch == "gpt2":
            return self._decode_one_gpt2(token)
        hp = self.hp
        hd = hp.head_dim
        pos = (max(self.cell_pos) + 1) if self.n_past else 0
        cell = self.n_past
        assert cell < self.n_ctx
        te = self.tensors["token_embd.weight"]
        rb = row_bytes(te.type, hp.n_embd)
        x = dequantize(te.data.reshape(-1)[token * rb:(token + 1) * rb], te.type)
        scale = np.float32(1.0) / np.sqrt(np.float32(hd), dtype=np.float32)
        ff = self.tensors.get("rope_freqs.weight")
        ffv = None if ff is None else dequantize(ff.data, ff.type)
        for il in range(hp.n_layer):
            cur = (rms_norm(x, hp.eps) * self._w(f"blk.{il}.attn_norm.weight")).astype(np.float32)
            q = self._mm(f"blk.{il}.attn_q.weight", cur).reshape(hp.n_head, hd)
            k = self._mm(f"blk.{il}.attn_k.weight", cur).reshape(hp.n_head_kv, hd)
            v = self._mm(f"blk.{il}.attn_v.weight", cur)
            q = rope_norm(q, pos, hp.n_rot, hp.rope_base, ffv)
            k = rope_norm(k, pos, hp.n_rot, hp.rope_base, ffv)
            self.kcache[il][cell] = f32_to_f16(k.reshape(-1))
            self.vcache[il][cell] = f32_to_f16(v)
            vis = [c for c in range(cell + 1) if c == cell or self.cell_pos[c] <= pos]
            Kc = self.kcache[il][vis].reshape(len(vis), hp.n_head_kv, hd)
            Vc = self.vcache[il][vis].reshape(len(vis), hp.n_head_kv, hd)
            ratio = hp.n_head // hp.n_head_kv
            att = np.empty((hp.n_head, hd), np.float32)
            for h in range(hp.n_head):
                g = h // ratio
                att[h] = attention_head(q[h], Kc[:, g], Vc[:, g], scale)
            cur = self._mm(f"blk.{il}.attn_output.weight", att.reshape(-1))
            x = (cur + x).astype(np.float32)
            cur = (rms_norm(x, hp.eps) * self._w(f"blk.{il}.ffn_norm.weight")).astype(np.float32)
            x = (self._ffn(il, cur) + x).astype(np.float32)
        cur = (rms_norm(x, hp.eps) * self._w("output_norm.weight")).astype(np.float32)
        out = self.tensors.get("output.weight", self.tensors["token_embd.weight"])
        logits = mul_mat_vec(out.data, out.type, out.shape[0], cur)
        self.cell_pos.append(pos)
        self.n_past += 1
        return logits

    def decode(self, tokens):
        logits = None
        for t in tokens:
            logits = self.decode_one(int(t))
        return logits
