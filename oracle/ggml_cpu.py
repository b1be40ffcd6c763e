"""ctypes driver for oracle/ggml_cpu.c -- the C restatement of the ggml CPU path.

TEST INFRASTRUCTURE ONLY (checker + the bench's cpu_baseline); the product
(blama_amd/) never imports it.  Build: `make -C oracle` (done by
__graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "libggml_oracle.so")
_lib = None


class HParams(C.Structure):
    _fields_ = [("n_vocab", C.c_int), ("n_embd", C.c_int), ("n_layer", C.c_int), ("n_head", C.c_int),
                ("n_head_kv", C.c_int), ("n_ff", C.c_int), ("n_rot", C.c_int), ("n_expert", C.c_int),
                ("n_expert_used", C.c_int), ("eps", C.c_float), ("rope_base", C.c_float)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run `make -C oracle`")
        L = C.CDLL(LIB)
        L.orc_gemv.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.orc_create.restype = C.c_void_p
        L.orc_create.argtypes = [C.POINTER(HParams), C.c_int]
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_set_tensor.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_void_p, C.c_int64, C.c_int64, C.c_int64]
        L.orc_decode.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.orc_kv_clear.argtypes = [C.c_void_p]
        L.orc_n_threads.restype = C.c_int
        L.orc_set_alt.argtypes = [C.c_int]
        L.orc_set_simd.argtypes = [C.c_int]
        L.orc_last_moe_margin.restype = C.c_float
        _lib = L
    return _lib


def set_simd(on: bool) -> None:
    """The AVX2 dot kernels (ggml's x86 technique; the bench's CPU-baseline timing) instead of the
    generic loops (the parity order, default)."""
    lib().orc_set_simd(1 if on else 0)


def gemv(t: int, raw: np.ndarray, rows: int, K: int, x: np.ndarray) -> np.ndarray:
    raw = np.ascontiguousarray(raw, np.uint8)
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty(rows, np.float32)
    if lib().orc_gemv(t, raw.ctypes.data, rows, K, x.ctypes.data, y.ctypes.data) != 0:
        raise RuntimeError("orc_gemv: unsupported type")
    return y


class Model:
    """Batch-1 llama decode on the C restatement; tensors are views into a GGUF image."""

    def __init__(self, gguf_image, n_ctx: int = 0):
        import sys
        sys.path.insert(0, os.path.dirname(_HERE))
        from blama_amd import gguf
        self._buf = gguf_image
        rd = gguf.GGUFReader(gguf_image)
        kv = rd.kv
        a = kv["general.architecture"]
        n_embd = int(kv[f"{a}.embedding_length"])
        n_head = int(kv[f"{a}.attention.head_count"])
        hp = HParams(int(rd.tensors["token_embd.weight"].shape[1]), n_embd, int(kv[f"{a}.block_count"]),
                     n_head, int(kv.get(f"{a}.attention.head_count_kv", n_head)),
                     int(kv[f"{a}.feed_forward_length"]),
                     int(kv.get(f"{a}.rope.dimension_count", n_embd // n_head)),
                     int(kv.get(f"{a}.expert_count", 0)), int(kv.get(f"{a}.expert_used_count", 0)),
                     float(kv[f"{a}.attention.layer_norm_rms_epsilon"]),
                     float(kv.get(f"{a}.rope.freq_base", 10000.0)))
        self.hp = hp
        self.n_ctx = n_ctx or int(kv[f"{a}.context_length"])
        self.h = lib().orc_create(C.byref(hp), self.n_ctx)
        self._keep = []
        for name, t in rd.tensors.items():
            data = np.ascontiguousarray(t.data)
            self._keep.append(data)
            ne = list(t.shape) + [1, 1]
            lib().orc_set_tensor(self.h, name.encode(), t.type, data.ctypes.data, ne[0], ne[1], ne[2])

    def decode_one(self, token: int, alt: bool = False) -> np.ndarray:
        """alt: the same algorithm with the 8 float lanes of every k-quant dot (the blocks of a
        Q8_0 row) summed in the reverse order -- an equally valid fp32 order (measures the CPU
        path's own noise floor)."""
        out = np.empty(self.hp.n_vocab, np.float32)
        lib().orc_set_alt(1 if alt else 0)
        try:
            rc = lib().orc_decode(self.h, int(token), out.ctypes.data)
        finally:
            lib().orc_set_alt(0)
        if rc != 0:
            raise RuntimeError("orc_decode: no KV space")
        # the smallest router gap (last pick vs first left out) over this token's MoE layers
        self.last_moe_margin = float(lib().orc_last_moe_margin())
        return out

    def reset(self):
        """llama_kv_self_clear: an empty cache (a new session)."""
        lib().orc_kv_clear(self.h)

    def decode(self, tokens):
        out = None
        for t in tokens:
            out = self.decode_one(t)
        return out

    def close(self):
        if self.h:
            lib().orc_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def time_decode(cfg_name: str, seconds: float, gguf_image=None):
    """Decode tokens on the host cores until ~`seconds` have elapsed (bounded sample)."""
    import sys
    sys.path.insert(0, os.path.dirname(_HERE))
    from blama_amd import synthetic
    cfg = synthetic.CONFIGS[cfg_name]
    buf = gguf_image if gguf_image is not None else synthetic.build_gguf(cfg, seed=0)
    m = Model(buf, n_ctx=256)
    toks = np.random.default_rng(1234).integers(0, cfg.n_vocab, 64)
    m.decode_one(int(toks[0]))   # warm
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and n + 1 < len(toks):
        m.decode_one(int(toks[n + 1]))
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 3), "unit": "tokens/s", "cores": lib().orc_n_threads(), "kind": "port",
            "sample": f"{n} batch-1 decode steps of synthetic {cfg.name} {cfg.ftype} (C restatement of the "
                      f"ggml b5187 CPU path, OpenMP over rows/heads), {dt:.1f}s wall"}
