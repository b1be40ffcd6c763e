"""Synthetic LLaMA-family GGUF images for the BASELINE.json configs.

No checkpoint can be downloaded here, so tests and the
bench use GGUF images with the *exact* tensor names, shapes and per-tensor
quant types of the named models, filled with seeded random -- but valid and
realistically scaled -- quant blocks.

Per-tensor type rules follow llama.cpp b5187 ``llama_tensor_get_type``
(src/llama-quant.cpp) as summarised in SURVEY.md §8 "Q4_K_M tensor mix":
Q4_K_M -> output Q6_K; attn_v / ffn_down Q6_K where use_more_bits(i, n);
everything else Q4_K; 8-expert models bump attn_k/attn_v to Q8_0 and
attn_output to Q5_K (Q4_K_M) ; norms F32.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, replace

import os

import numpy as np

from . import gguf

F32, F16, Q8_0, Q4_K, Q5_K, Q6_K = 0, 1, 8, 12, 13, 14


@dataclass(frozen=True)
class LlamaConfig:
    name: str
    n_vocab: int
    n_embd: int
    n_layer: int
    n_head: int
    n_head_kv: int
    n_ff: int
    n_ctx_train: int
    rope_base: float
    eps: float
    ftype: str            # "Q4_K_M", "Q5_K_M", "Q6_K", "Q8_0", "Q4_K"...
    n_expert: int = 0
    n_expert_used: int = 0
    arch: str = "llama"   # "llama" or "gpt2" (llm_build_gpt2)

    @property
    def head_dim(self):
        return self.n_embd // self.n_head


CONFIGS = {
    # BASELINE.json configs[0..4]
    "tinyllama-1.1b-q8_0": LlamaConfig("TinyLlama-1.1B", 32000, 2048, 22, 32, 4, 5632, 2048,
                                        10000.0, 1e-5, "Q8_0"),
    "llama2-7b-q4_k_m": LlamaConfig("Llama-2-7B", 32000, 4096, 32, 32, 32, 11008, 4096,
                                     10000.0, 1e-5, "Q4_K_M"),
    "llama3-8b-q6_k": LlamaConfig("Llama-3-8B", 128256, 4096, 32, 32, 8, 14336, 8192,
                                   500000.0, 1e-5, "Q6_K"),
    "mixtral-8x7b-q5_k_m": LlamaConfig("Mixtral-8x7B", 32000, 4096, 32, 32, 8, 14336, 32768,
                                        1e6, 1e-5, "Q5_K_M", n_expert=8, n_expert_used=2),
    # small shapes for parity tests (same code paths, seconds on the CPU oracle)
    "tiny-q4_k_m": LlamaConfig("tiny", 512, 256, 4, 4, 2, 512, 256, 10000.0, 1e-5, "Q4_K_M"),
    "tiny-q5_k_m": LlamaConfig("tiny", 512, 256, 2, 4, 2, 512, 256, 10000.0, 1e-5, "Q5_K_M"),
    "tiny-q6_k": LlamaConfig("tiny", 640, 256, 2, 4, 1, 768, 256, 500000.0, 1e-5, "Q6_K"),
    "tiny-q8_0": LlamaConfig("tiny", 384, 256, 2, 8, 4, 768, 256, 10000.0, 1e-6, "Q8_0"),
    "tiny1-q4_k_m": LlamaConfig("tiny1", 512, 256, 1, 4, 2, 512, 256, 10000.0, 1e-5, "Q4_K_M"),
    "tiny-moe-q5_k_m": LlamaConfig("tiny-moe", 512, 256, 2, 4, 2, 512, 256, 1e6, 1e-5,
                                    "Q5_K_M", n_expert=4, n_expert_used=2),
    # GQA ratio 2 with 16 kv heads of 64: the quantising decode attention has no
    # kernel for two kv heads per 256-block, so decode takes the gemv_kernel step and short
    # batches the plain fused attention + quant_act -- both must still run
    "tiny-gqa16-q4_k_m": LlamaConfig("tiny-gqa16", 512, 2048, 2, 32, 16, 512, 256, 10000.0, 1e-5, "Q4_K_M"),
    # the reference's own KAT model shape (gpt2-117m-q6_k, t-integration.cpp:25): 12 x 768,
    # 12 heads of 64, n_ff 3072, V 50257, 1024 positions, every matrix Q6_K, tied output head
    "gpt2-117m-q6_k": LlamaConfig("GPT-2-117M", 50257, 768, 12, 12, 12, 3072, 1024, 10000.0, 1e-5,
                                  "Q6_K", arch="gpt2"),
    "tiny-gpt2-q6_k": LlamaConfig("tiny-gpt2", 700, 256, 2, 4, 4, 768, 128, 10000.0, 1e-5, "Q6_K",
                                  arch="gpt2"),
    "tiny-gpt2-q8_0": LlamaConfig("tiny-gpt2", 600, 512, 2, 8, 8, 1024, 128, 10000.0, 1e-5, "Q8_0",
                                  arch="gpt2"),
}


def use_more_bits(i: int, n: int) -> bool:
    # llama-quant.cpp use_more_bits
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def _gpt2_types(cfg, base) -> dict:
    """llm_build_gpt2's tensors (LLM_ARCH_GPT2 in src/llama-arch.cpp): every matrix of the
    file type, LayerNorm weights / biases and the matrix biases F32, no output.weight (the
    head is token_embd, TENSOR_DUPLICATED in llama-model.cpp)."""
    t = {"token_embd.weight": base, "position_embd.weight": base,
         "output_norm.weight": F32, "output_norm.bias": F32}
    for i in range(cfg.n_layer):
        p = f"blk.{i}."
        for n in ("attn_norm", "ffn_norm"):
            t[p + n + ".weight"] = F32
            t[p + n + ".bias"] = F32
        for n in ("attn_qkv", "attn_output", "ffn_up", "ffn_down"):
            t[p + n + ".weight"] = base
            t[p + n + ".bias"] = F32
    return t


def _gpt2_shapes(cfg) -> dict:
    d = cfg.n_embd
    s = {"token_embd.weight": (d, cfg.n_vocab), "position_embd.weight": (d, cfg.n_ctx_train),
         "output_norm.weight": (d,), "output_norm.bias": (d,)}
    for i in range(cfg.n_layer):
        p = f"blk.{i}."
        for n in ("attn_norm", "ffn_norm"):
            s[p + n + ".weight"] = (d,)
            s[p + n + ".bias"] = (d,)
        s[p + "attn_qkv.weight"] = (d, 3 * d)
        s[p + "attn_qkv.bias"] = (3 * d,)
        s[p + "attn_output.weight"] = (d, d)
        s[p + "attn_output.bias"] = (d,)
        s[p + "ffn_up.weight"] = (d, cfg.n_ff)
        s[p + "ffn_up.bias"] = (cfg.n_ff,)
        s[p + "ffn_down.weight"] = (cfg.n_ff, d)
        s[p + "ffn_down.bias"] = (d,)
    return s


def tensor_types(cfg: LlamaConfig) -> dict:
    """name -> ggml type for every weight (the Q*_K_M mixes of llama_tensor_get_type)."""
    base = {"Q4_K_M": Q4_K, "Q5_K_M": Q5_K, "Q6_K": Q6_K, "Q8_0": Q8_0, "Q4_K": Q4_K,
            "Q5_K": Q5_K}[cfg.ftype]
    if cfg.arch == "gpt2":
        return _gpt2_types(cfg, base)
    mixed = cfg.ftype in ("Q4_K_M", "Q5_K_M")
    t = {"token_embd.weight": base, "output_norm.weight": F32,
         "output.weight": Q8_0 if base == Q8_0 else Q6_K}
    n = cfg.n_layer
    for i in range(n):
        p = f"blk.{i}."
        t[p + "attn_norm.weight"] = F32
        t[p + "ffn_norm.weight"] = F32
        t[p + "attn_q.weight"] = base
        t[p + "attn_k.weight"] = base
        t[p + "attn_v.weight"] = base
        t[p + "attn_output.weight"] = base
        if mixed and use_more_bits(i, n):
            t[p + "attn_v.weight"] = Q6_K
        if cfg.n_expert == 8 and base != Q8_0:
            t[p + "attn_k.weight"] = Q8_0
            t[p + "attn_v.weight"] = Q8_0
            if cfg.ftype == "Q4_K_M":
                t[p + "attn_output.weight"] = Q5_K
        down = Q6_K if (mixed and use_more_bits(i, n)) else base
        if cfg.n_expert:
            t[p + "ffn_gate_inp.weight"] = F32
            t[p + "ffn_gate_exps.weight"] = base
            t[p + "ffn_up_exps.weight"] = base
            t[p + "ffn_down_exps.weight"] = down
        else:
            t[p + "ffn_gate.weight"] = base
            t[p + "ffn_up.weight"] = base
            t[p + "ffn_down.weight"] = down
    return t


def tensor_shapes(cfg: LlamaConfig) -> dict:
    """name -> ggml ne shape (ne0 = input dim K)."""
    if cfg.arch == "gpt2":
        return _gpt2_shapes(cfg)
    d, kv = cfg.n_embd, cfg.n_head_kv * cfg.head_dim
    s = {"token_embd.weight": (d, cfg.n_vocab), "output_norm.weight": (d,),
         "output.weight": (d, cfg.n_vocab)}
    for i in range(cfg.n_layer):
        p = f"blk.{i}."
        s[p + "attn_norm.weight"] = (d,)
        s[p + "ffn_norm.weight"] = (d,)
        s[p + "attn_q.weight"] = (d, d)
        s[p + "attn_k.weight"] = (d, kv)
        s[p + "attn_v.weight"] = (d, kv)
        s[p + "attn_output.weight"] = (d, d)
        if cfg.n_expert:
            s[p + "ffn_gate_inp.weight"] = (d, cfg.n_expert)
            s[p + "ffn_gate_exps.weight"] = (d, cfg.n_ff, cfg.n_expert)
            s[p + "ffn_up_exps.weight"] = (d, cfg.n_ff, cfg.n_expert)
            s[p + "ffn_down_exps.weight"] = (cfg.n_ff, d, cfg.n_expert)
        else:
            s[p + "ffn_gate.weight"] = (d, cfg.n_ff)
            s[p + "ffn_up.weight"] = (d, cfg.n_ff)
            s[p + "ffn_down.weight"] = (cfg.n_ff, d)
    return s


def _rng(seed: int, name: str):
    h = hashlib.sha256(f"{seed}:{name}".encode()).digest()
    return np.random.default_rng(int.from_bytes(h[:8], "little"))


def _pack_scales_k4(sc: np.ndarray, m: np.ndarray) -> np.ndarray:
    """Inverse of get_scale_min_k4 (the packing of quantize_row_q4_K_ref)."""
    nb = sc.shape[0]
    s = np.zeros((nb, 12), np.uint8)
    for j in range(4):
        s[:, j] = sc[:, j]
        s[:, j + 4] = m[:, j]
    for j in range(4, 8):
        s[:, j + 4] = (sc[:, j] & 0xF) | ((m[:, j] & 0xF) << 4)
        s[:, j - 4] |= (sc[:, j] >> 4) << 6
        s[:, j] |= (m[:, j] >> 4) << 6
    return s


def fill_quant(view: np.ndarray, t: int, rng, std: float = 0.03):
    """Fill a tensor's bytes with valid random blocks whose dequantised values
    are roughly zero-mean with standard deviation ``std``."""
    be, bb = gguf.GGML_BLOCK[t]
    if t == F32:
        v = view.view(np.float32)
        v[:] = rng.standard_normal(v.size, dtype=np.float32) * np.float32(std)
        return
    if t == F16:
        v = view.view(np.float16)
        v[:] = (rng.standard_normal(v.size, dtype=np.float32) * np.float32(std)).astype(np.float16)
        return
    nb = view.size // bb
    bl = view.reshape(nb, bb)
    CH = 1 << 16   # blocks per chunk (bounded temporaries)
    for a in range(0, nb, CH):
        b = bl[a:a + CH]
        n = b.shape[0]
        b[:] = rng.integers(0, 256, size=b.shape, dtype=np.uint8)
        if t in (Q4_K, Q5_K):
            qmax = 15 if t == Q4_K else 31
            sc = rng.integers(24, 64, size=(n, 8), dtype=np.int32)
            d = (std / (40.0 * (qmax + 1) / np.sqrt(12.0))) * rng.uniform(0.8, 1.2, n)
            ratio = 16.0 if t == Q4_K else 32.0      # dmin = d*ratio
            dmin = d * ratio
            m = np.clip(np.rint(sc * (qmax / 2.0) / ratio), 0, 63).astype(np.int32)
            b[:, 0:2] = d.astype(np.float16).view(np.uint8).reshape(n, 2)
            b[:, 2:4] = dmin.astype(np.float16).view(np.uint8).reshape(n, 2)
            b[:, 4:16] = _pack_scales_k4(sc.astype(np.uint8), m.astype(np.uint8))
        elif t == Q6_K:
            sc = rng.integers(16, 48, size=(n, 16), dtype=np.int32)
            sgn = rng.integers(0, 2, size=(n, 16), dtype=np.int32) * 2 - 1
            b[:, 192:208] = (sc * sgn).astype(np.int8).view(np.uint8)
            d = (std / (32.0 * 64 / np.sqrt(12.0))) * rng.uniform(0.8, 1.2, n)
            b[:, 208:210] = d.astype(np.float16).view(np.uint8).reshape(n, 2)
        elif t == Q8_0:
            d = (std / (256 / np.sqrt(12.0))) * rng.uniform(0.8, 1.2, n)
            b[:, 0:2] = d.astype(np.float16).view(np.uint8).reshape(n, 2)
        else:
            raise NotImplementedError(t)


# ---------------------------------------------------------------------------
# Float -> block quantisers (simple, valid blocks; not ggml's rmse-searching
# quantize_row_*_ref -- any valid block is valid model data).  X: (n, 256)
# float32 superblocks (Q8_0: (n, 32) blocks); returns (n, block_bytes) uint8.
# ---------------------------------------------------------------------------
def _f16(a):
    return np.asarray(a, np.float32).astype(np.float16)


def quantize_q8_0_rows(X):
    X = X.reshape(-1, 32)
    amax = np.abs(X).max(1)
    d16 = _f16(amax / 127.0)
    d = d16.astype(np.float32)
    q = np.clip(np.rint(np.divide(X, d[:, None], out=np.zeros_like(X), where=d[:, None] > 0)), -127, 127)
    out = np.empty((X.shape[0], 34), np.uint8)
    out[:, 0:2] = d16.view(np.uint8).reshape(-1, 2)
    out[:, 2:] = q.astype(np.int8).view(np.uint8)
    return out


def quantize_q6_K_rows(X):
    X = X.reshape(-1, 256)
    n = X.shape[0]
    s = np.abs(X.reshape(n, 16, 16)).max(2) / 31.0            # per-16 scale
    d16 = _f16(s.max(1) / 127.0)
    d = d16.astype(np.float32)
    sc = np.clip(np.rint(np.divide(s, d[:, None], out=np.zeros_like(s), where=d[:, None] > 0)), 1, 127)
    eff = np.repeat(d[:, None] * sc, 16, axis=1)
    q = np.clip(np.rint(np.divide(X, eff, out=np.zeros_like(X), where=eff > 0)), -32, 31).astype(np.int32) + 32
    ql = np.zeros((n, 128), np.uint8)
    qh = np.zeros((n, 64), np.uint8)
    for h in range(2):
        e = q[:, 128 * h:128 * h + 128]
        a, b, c, dd = e[:, 0:32], e[:, 32:64], e[:, 64:96], e[:, 96:128]
        ql[:, 64 * h:64 * h + 32] = (a & 0xF) | ((c & 0xF) << 4)
        ql[:, 64 * h + 32:64 * h + 64] = (b & 0xF) | ((dd & 0xF) << 4)
        qh[:, 32 * h:32 * h + 32] = (a >> 4) | ((b >> 4) << 2) | ((c >> 4) << 4) | ((dd >> 4) << 6)
    out = np.empty((n, 210), np.uint8)
    out[:, 0:128] = ql
    out[:, 128:192] = qh
    out[:, 192:208] = sc.astype(np.int8).view(np.uint8)
    out[:, 208:210] = d16.view(np.uint8).reshape(n, 2)
    return out


def quantize_q45_K_rows(X, q5: bool):
    X = X.reshape(-1, 256)
    n = X.shape[0]
    qmax = 31 if q5 else 15
    sub = X.reshape(n, 8, 32)
    mn = np.maximum(0.0, -sub.min(2))
    s = (sub.max(2) + mn) / qmax
    d16 = _f16(s.max(1) / 63.0)
    m16 = _f16(mn.max(1) / 63.0)
    d, dm = d16.astype(np.float32), m16.astype(np.float32)
    sc = np.clip(np.rint(np.divide(s, d[:, None], out=np.zeros_like(s), where=d[:, None] > 0)), 0, 63)
    m = np.clip(np.rint(np.divide(mn, dm[:, None], out=np.zeros_like(mn), where=dm[:, None] > 0)), 0, 63)
    eff = d[:, None] * sc
    off = dm[:, None] * m
    q = np.clip(np.rint(np.divide(sub + off[:, :, None], eff[:, :, None], out=np.zeros_like(sub),
                                  where=eff[:, :, None] > 0)), 0, qmax).astype(np.int32).reshape(n, 256)
    qs = np.zeros((n, 128), np.uint8)
    qh = np.zeros((n, 32), np.uint8)
    for j in range(4):
        lo, hi = q[:, 64 * j:64 * j + 32], q[:, 64 * j + 32:64 * j + 64]
        qs[:, 32 * j:32 * j + 32] = (lo & 0xF) | ((hi & 0xF) << 4)
        if q5:
            qh |= (((lo >> 4) & 1) << (2 * j)).astype(np.uint8)
            qh |= (((hi >> 4) & 1) << (2 * j + 1)).astype(np.uint8)
    out = np.empty((n, 176 if q5 else 144), np.uint8)
    out[:, 0:2] = d16.view(np.uint8).reshape(n, 2)
    out[:, 2:4] = m16.view(np.uint8).reshape(n, 2)
    out[:, 4:16] = _pack_scales_k4(sc.astype(np.uint8), m.astype(np.uint8))
    if q5:
        out[:, 16:48] = qh
        out[:, 48:176] = qs
    else:
        out[:, 16:144] = qs
    return out


def quantize_rows(X, t: int) -> np.ndarray:
    X = np.ascontiguousarray(X, np.float32)
    if t == Q8_0:
        return quantize_q8_0_rows(X).reshape(-1)
    if t == Q6_K:
        return quantize_q6_K_rows(X).reshape(-1)
    if t in (Q4_K, Q5_K):
        return quantize_q45_K_rows(X, t == Q5_K).reshape(-1)
    if t == F32:
        return X.reshape(-1).view(np.uint8)
    if t == F16:
        return X.reshape(-1).astype(np.float16).view(np.uint8)
    raise NotImplementedError(t)


# ---------------------------------------------------------------------------
# Token structure.  A random-weight 32-layer quantised network is chaotic: two
# correct CPU implementations that differ only in fp32 summation order end up
# with LogitComparer similarity ~0.7 (measured; DESIGN.md "synthetic weights"),
# because its top-10 logits are tightly packed in a flat distribution.  Trained
# LMs have peaked next-token distributions.  The synthetic model gets one:
# a per-token direction B[t] (unit-variance Gaussian) is the embedding of t,
# and output row t' carries sum_k alpha/sqrt(k) * B[t'-k], k = 1..10, on top of
# the random part -- after token t the model "prefers" t+1 > t+2 > ... > t+10.
# ---------------------------------------------------------------------------
_BCHUNK = 1024


def _token_dirs(seed: int, lo: int, hi: int, V: int, d: int) -> np.ndarray:
    """B[t mod V] for t in [lo, hi) (lo may be negative); float32 (hi-lo, d)."""
    out = np.empty((hi - lo, d), np.float32)
    t = lo
    while t < hi:
        tm = t % V
        c = tm // _BCHUNK
        base = c * _BCHUNK
        rows = min(_BCHUNK, V - base)
        blk = _rng(seed, f"tokdir:{c}").standard_normal((rows, d), dtype=np.float32)
        take = min(hi - t, base + rows - tm)
        out[t - lo:t - lo + take] = blk[tm - base:tm - base + take]
        t += take
    return out


def _init_params(cfg):
    env = dict(kv.split("=") for kv in os.environ.get("BLAMA_SYNTH_INIT", "").split(",") if kv)
    p = {"base": 0.03, "qk": 0.01, "resid": 0.03 / np.sqrt(2.0 * cfg.n_layer), "embd": 8.0,
         "alpha": 0.01, "nsucc": 10}
    if cfg.arch == "gpt2":
        p["embd"] = 1.0   # the embedding is also the (tied) output head: logits O(sqrt(d))
    for k, v in env.items():
        p[k] = float(v)
    return p


def _fill_structured(cfg, seed, name, t, view, P):
    V, d = cfg.n_vocab, cfg.n_embd
    be, bb = gguf.GGML_BLOCK[t]
    row_b = d // be * bb
    rows = view.reshape(V, row_b)
    CH = 2048
    ns = int(P["nsucc"])

    def chunk(a):
        b = min(V, a + CH)
        if name == "token_embd.weight":
            X = _token_dirs(seed, a, b, V, d) * np.float32(P["embd"])
        else:
            # chunk 0 draws from the tensor's own stream (as every small-vocab model always
            # did); later chunks from streams of their own, so chunks fill in parallel
            rng = _rng(seed, name) if a == 0 else _rng(seed, f"{name}:{a}")
            X = rng.standard_normal((b - a, d), dtype=np.float32) * np.float32(P["base"])
            Bw = _token_dirs(seed, a - ns, b, V, d)
            for k in range(1, ns + 1):
                X += np.float32(P["alpha"] / np.sqrt(k)) * Bw[ns - k:ns - k + (b - a)]
        rows[a:b] = quantize_rows(X, t).reshape(b - a, row_b)

    starts = list(range(0, V, CH))
    if len(starts) == 1:
        chunk(0)
        return
    from concurrent.futures import ThreadPoolExecutor   # numpy releases the GIL in these ops
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        list(ex.map(chunk, starts))


def vocab_tokens(n_vocab: int):
    toks = ["<unk>", "<s>", "</s>"] + ["<0x%02X>" % i for i in range(256)]
    toks += ["▁t%d" % i for i in range(n_vocab - len(toks))]
    return toks[:n_vocab]


RESIDUAL_OUT = ("attn_output.weight", "ffn_down.weight", "ffn_down_exps.weight")


def _init_std(P, name):
    if name.endswith(("attn_q.weight", "attn_k.weight")):
        return P["qk"]      # attention scores O(1): softmax not saturated
    if name.endswith(RESIDUAL_OUT):
        return P["resid"]   # residual branches scaled by 1/sqrt(2 n_layer)
    return P["base"]


BPE_CORPUS = [
    "The quick brown fox jumps over the lazy dog. It's a test, isn't it? We'll see.",
    "Verification sessions run concurrently on every replica of the model.",
    "request number 0 1 2 3 4 5 6 7 8 9 10 11 12 13 14 15 and 3.14159 pies",
    "Hello world! Numbers 1 22 333 4444, naive cafe, resume -- quotes and text.",
]


def bpe_vocab(n_vocab: int, n_merges_vocab: int = 800) -> dict:
    """A Llama-3-shaped byte-level BPE vocabulary of exactly n_vocab entries ("gpt2" tokenizer,
    pre-tokenizer "llama-bpe"): a BPE model trained here with HuggingFace `tokenizers` (the
    byte alphabet and up to n_merges_vocab pieces with their merges), then
    <|begin_of_text|> / <|end_of_text|> / <|eot_id|> and <|reserved_special_token_i|> control
    tokens up to n_vocab, as Llama-3's 128256-entry vocabulary ends in 256 reserved specials.
    Returns tokens, token types, merges, bos/eos ids and the trained `tokenizers.Tokenizer`
    (which encodes prompts exactly as the host mirror does, tests/test_tokenizer_bpe.py)."""
    import json
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers
    llama3 = (r"(?:'[sS]|'[tT]|'[rR][eE]|'[vV][eE]|'[mM]|'[lL][lL]|'[dD])|[^\r\n\p{L}\p{N}]?\p{L}+|"
              r"\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
    tok = Tokenizer(models.BPE(ignore_merges=True))
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(llama3), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, trim_offsets=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=n_merges_vocab, min_frequency=1,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)
    tok.train_from_iterator(BPE_CORPUS * 20, trainer=trainer)
    model = json.loads(tok.to_str())["model"]
    toks = [None] * len(model["vocab"])
    for t, i in model["vocab"].items():
        toks[i] = t
    merges = [m if isinstance(m, str) else " ".join(m) for m in model["merges"]]
    types = [1] * len(toks)
    specials = ["<|begin_of_text|>", "<|end_of_text|>", "<|eot_id|>"]
    k = 0
    while len(toks) + len(specials) < n_vocab:
        specials.append("<|reserved_special_token_%d|>" % k)
        k += 1
    base = len(toks)
    toks += specials
    types += [3] * len(specials)
    assert len(toks) == n_vocab
    return dict(tokens=toks, types=types, merges=merges, pre="llama-bpe", bos=base, eos=base + 1,
                eot=base + 2, tokenizer=tok)


def build_gguf(cfg: LlamaConfig, seed: int = 0, header_only: bool = False, vocab: dict | None = None) -> np.ndarray:
    """The whole synthetic GGUF file as one uint8 array (header_only: just the
    metadata + tensor table, enough for a vocab-only or no_upload replica load).
    vocab: a byte-level BPE vocabulary from bpe_vocab() instead of the SPM one."""
    w = gguf.GGUFWriter()
    arch = cfg.arch
    w.add_str("general.architecture", arch)
    w.add_str("general.name", f"synthetic {cfg.name} {cfg.ftype}")
    w.add_u32("general.file_type", {"Q8_0": 7, "Q4_K_M": 15, "Q5_K_M": 17, "Q6_K": 18,
                                    "Q4_K": 15, "Q5_K": 17}[cfg.ftype])
    w.add_u32(f"{arch}.context_length", cfg.n_ctx_train)
    w.add_u32(f"{arch}.embedding_length", cfg.n_embd)
    w.add_u32(f"{arch}.block_count", cfg.n_layer)
    w.add_u32(f"{arch}.feed_forward_length", cfg.n_ff)
    w.add_u32(f"{arch}.attention.head_count", cfg.n_head)
    if arch == "gpt2":   # LLM_KV_ATTENTION_LAYERNORM_EPS; no RoPE keys
        w.add_f32(f"{arch}.attention.layer_norm_epsilon", cfg.eps)
    else:
        w.add_u32(f"{arch}.attention.head_count_kv", cfg.n_head_kv)
        w.add_f32(f"{arch}.attention.layer_norm_rms_epsilon", cfg.eps)
        w.add_f32(f"{arch}.rope.freq_base", cfg.rope_base)
        w.add_u32(f"{arch}.rope.dimension_count", cfg.head_dim)
    w.add_u32(f"{arch}.vocab_size", cfg.n_vocab)
    if cfg.n_expert:
        w.add_u32(f"{arch}.expert_count", cfg.n_expert)
        w.add_u32(f"{arch}.expert_used_count", cfg.n_expert_used)
    if vocab is None:
        w.add_str("tokenizer.ggml.model", "llama")
        toks = vocab_tokens(cfg.n_vocab)
        w.add_array("tokenizer.ggml.tokens", gguf.T_STRING, toks)
        w.add_array("tokenizer.ggml.scores", gguf.T_FLOAT32, [-float(i) for i in range(len(toks))])
        ttype = [2, 3, 3] + [6] * 256 + [1] * (len(toks) - 259)
        w.add_array("tokenizer.ggml.token_type", gguf.T_INT32, ttype[:len(toks)])
        w.add_u32("tokenizer.ggml.bos_token_id", 1)
        w.add_u32("tokenizer.ggml.eos_token_id", 2)
        w.add_u32("tokenizer.ggml.unknown_token_id", 0)
    else:
        assert len(vocab["tokens"]) == cfg.n_vocab
        w.add_str("tokenizer.ggml.model", "gpt2")
        w.add_str("tokenizer.ggml.pre", vocab["pre"])
        w.add_array("tokenizer.ggml.tokens", gguf.T_STRING, vocab["tokens"])
        w.add_array("tokenizer.ggml.token_type", gguf.T_INT32, vocab["types"])
        w.add_array("tokenizer.ggml.merges", gguf.T_STRING, vocab["merges"])
        w.add_u32("tokenizer.ggml.bos_token_id", vocab["bos"])
        w.add_u32("tokenizer.ggml.eos_token_id", vocab["eos"])
        w.add_u32("tokenizer.ggml.eot_token_id", vocab["eot"])
    w.add_bool("tokenizer.ggml.add_bos_token", arch != "gpt2")
    types = tensor_types(cfg)
    shapes = tensor_shapes(cfg)
    for name in types:
        w.add_tensor(name, types[name], shapes[name])

    if header_only:
        return np.frombuffer(w.header_bytes()[0], np.uint8).copy()
    P = _init_params(cfg)

    def fill(name, t, shape, view):
        rng = _rng(seed, name)
        if name in ("token_embd.weight", "output.weight"):
            _fill_structured(cfg, seed, name, t, view, P)
            return
        if name.endswith("norm.weight"):
            v = view.view(np.float32)
            v[:] = rng.uniform(0.8, 1.2, v.size).astype(np.float32)
        elif name.endswith(".bias"):
            v = view.view(np.float32)
            v[:] = (rng.standard_normal(v.size) * 0.02).astype(np.float32)
        elif name == "position_embd.weight":
            fill_quant(view, t, rng, std=0.1)
        elif name.endswith("ffn_gate_inp.weight"):
            fill_quant(view, t, rng, std=0.05)
        else:
            fill_quant(view, t, rng, std=_init_std(P, name))

    return w.to_bytes(fill=fill)


def small_config(name: str, **kw) -> LlamaConfig:
    return replace(CONFIGS[name], **kw)
