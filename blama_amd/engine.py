"""ctypes binding of the C ABI in include/mi_engine.h.

This is the Python-side view of the drop-in boundary (the same entry points a
cgo/JNI/ctypes binding in a host application would declare).  It loads the
in-tree ``blama_amd/libmi_engine.so`` and fails loudly if it is missing: there
is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MI_ENGINE_LIB=<name> loads libmi_engine_<name>.so instead: "stamps" is the diagnostic build
# (per-workgroup timestamps), other names are A/B builds of an earlier revision (scripts/ab_build.sh)
_VARIANT = os.environ.get("MI_ENGINE_LIB")
LIB_PATH = os.path.join(_HERE, f"libmi_engine_{_VARIANT}.so" if _VARIANT else "libmi_engine.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "mi_engine.h")

_lib = None


class EngineError(RuntimeError):
    pass


class ModelParams(C.Structure):
    _fields_ = [("device_ordinal", C.c_int32), ("cpu_only", C.c_int32),
                ("vocab_only", C.c_int32), ("no_upload", C.c_int32)]


_P = C.c_void_p
_SIGS = {
    "mi_last_error": (C.c_char_p, []),
    "mi_model_load": (_P, [C.c_char_p, C.POINTER(ModelParams)]),
    "mi_model_load_from_memory": (_P, [_P, C.c_size_t, C.POINTER(ModelParams)]),
    "mi_model_free": (None, [_P]),
    "mi_model_n_vocab": (C.c_int32, [_P]),
    "mi_model_n_ctx_train": (C.c_int32, [_P]),
    "mi_model_n_embd": (C.c_int32, [_P]),
    "mi_model_n_layer": (C.c_int32, [_P]),
    "mi_model_n_head": (C.c_int32, [_P]),
    "mi_model_n_head_kv": (C.c_int32, [_P]),
    "mi_model_n_ff": (C.c_int32, [_P]),
    "mi_model_n_expert": (C.c_int32, [_P]),
    "mi_model_token_bos": (C.c_int32, [_P]),
    "mi_model_token_eos": (C.c_int32, [_P]),
    "mi_model_add_bos": (C.c_int32, [_P]),
    "mi_model_token_is_eog": (C.c_int32, [_P, C.c_int32]),
    "mi_model_token_text": (C.c_int32, [_P, C.c_int32, C.c_char_p, C.c_int32]),
    "mi_model_n_tokens": (C.c_int32, [_P]),
    "mi_model_token_score": (C.c_float, [_P, C.c_int32]),
    "mi_model_token_type": (C.c_int32, [_P, C.c_int32]),
    "mi_model_tokenizer": (C.c_int32, [_P, C.c_char_p, C.c_int32]),
    "mi_model_meta_str": (C.c_int32, [_P, C.c_char_p, C.c_char_p, C.c_int32]),
    "mi_model_n_merges": (C.c_int32, [_P]),
    "mi_model_merge": (C.c_int32, [_P, C.c_int32, C.c_char_p, C.c_int32]),
    "mi_model_weight_bytes": (C.c_int64, [_P]),
    "mi_model_arena": (C.c_int32, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    "mi_model_type_histogram": (C.c_int32, [_P, C.POINTER(C.c_int64), C.c_int32]),
    "mi_model_replicate": (C.c_int32, [C.POINTER(_P), C.c_int32]),
    "mi_ctx_create": (_P, [_P, C.c_uint32, C.c_uint32, C.c_uint32]),
    "mi_ctx_free": (None, [_P]),
    "mi_n_ctx": (C.c_uint32, [_P]),
    "mi_n_batch": (C.c_uint32, [_P]),
    "mi_decode": (C.c_int32, [_P, C.POINTER(C.c_int32), C.c_int32, C.c_int32]),
    "mi_topk": (C.c_int32, [_P, C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_float)]),
    "mi_gather": (C.c_int32, [_P, C.c_int32, C.POINTER(C.c_int32), C.c_int32, C.POINTER(C.c_float)]),
    "mi_logits": (C.POINTER(C.c_float), [_P, C.c_int32]),
    "mi_gather_rows": (C.c_int32, [_P, C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.c_int32, C.POINTER(C.c_float)]),
    "mi_synchronize": (None, [_P]),
    "mi_kv_clear": (None, [_P]),
    "mi_kv_seq_rm": (C.c_int32, [_P, C.c_int32, C.c_int32]),
    "mi_kv_seq_add": (C.c_int32, [_P, C.c_int32, C.c_int32, C.c_int32]),
    "mi_kv_seq_div": (C.c_int32, [_P, C.c_int32, C.c_int32, C.c_int32]),
    "mi_kv_pos_max": (C.c_int32, [_P]),
    "mi_kv_n_cells": (C.c_int32, [_P]),
    "mi_state_size": (C.c_size_t, [_P]),
    "mi_state_get": (C.c_size_t, [_P, _P, C.c_size_t]),
    "mi_state_set": (C.c_size_t, [_P, _P, C.c_size_t]),
    "mi_prof_enable": (C.c_int32, [_P, C.c_int32]),
    "mi_prof_read": (C.c_int32, [_P, C.POINTER(C.c_float), C.c_int32]),
    "mi_prof_ffn_bytes": (C.c_int64, [_P]),
    "mi_decode_path": (C.c_int32, [_P]),
    "mi_op_dgemv": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mi_prof_bytes": (C.c_int64, [_P]),
    "mi_debug_stamps": (C.c_int32, [_P, _P, C.c_int32]),
    "mi_op_gemv": (C.c_int32, [C.c_int32, C.c_int32, _P, C.c_int32, C.c_int32, _P, _P]),
    "mi_op_dequant": (C.c_int32, [C.c_int32, C.c_int32, _P, C.c_int32, C.c_int32, _P]),
    "mi_op_quantize_q8_K": (C.c_int32, [C.c_int32, _P, C.c_int32, _P, _P, _P]),
    "mi_op_topk": (C.c_int32, [C.c_int32, _P, C.c_int32, C.c_int32, _P, _P]),
    "mi_op_attention": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, _P,
                                    C.c_int32, _P]),
    "mi_op_gemv_bench": (C.c_int32, [C.c_int32, C.c_int32, _P, C.c_int32, C.c_int32, C.c_int32,
                                     C.POINTER(C.c_float)]),
    "mi_op_gemm": (C.c_int32, [C.c_int32, C.c_int32, _P, _P, C.c_int32, C.c_int32, C.c_int32, _P, _P]),
    "mi_op_attention_batch": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                          _P, _P, _P, _P, _P, _P, _P]),
}


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Names of the functions include/mi_engine.h declares."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mi_[A-Za-z0-9_]+)\s*\(", txt)))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EngineError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return (lib().mi_last_error() or b"").decode()


def _check(rc, what):
    if rc is None or (isinstance(rc, int) and rc < 0):
        raise EngineError(f"{what}: {last_error()}")
    return rc


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Model:
    """Owns an mi_model (llama_model_load_from_file + llama_model_free)."""

    def __init__(self, source, device: int = 0, vocab_only: bool = False, no_upload: bool = False):
        L = lib()
        p = ModelParams(device, 0, int(vocab_only), int(no_upload))
        if isinstance(source, (str, os.PathLike)):
            h = L.mi_model_load(os.fspath(source).encode(), C.byref(p))
        else:
            if isinstance(source, (bytes, bytearray, memoryview)):
                buf = np.frombuffer(source, np.uint8)
            else:
                buf = np.ascontiguousarray(source, dtype=np.uint8)
            h = L.mi_model_load_from_memory(_ptr(buf), buf.size, C.byref(p))
        if not h:
            raise EngineError(f"model load failed: {last_error()}")
        self.h = h
        self.n_vocab = L.mi_model_n_vocab(h)
        self.n_embd = L.mi_model_n_embd(h)
        self.n_layer = L.mi_model_n_layer(h)
        self.n_ctx_train = L.mi_model_n_ctx_train(h)
        self.n_head = L.mi_model_n_head(h)
        self.n_head_kv = L.mi_model_n_head_kv(h)
        self.n_ff = L.mi_model_n_ff(h)
        self.n_expert = L.mi_model_n_expert(h)

    def close(self):
        if getattr(self, "h", None):
            lib().mi_model_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def weight_bytes(self) -> int:
        return lib().mi_model_weight_bytes(self.h)

    @property
    def arena(self):
        """(device pointer, bytes) of the weight arena (replica broadcast)."""
        p = C.c_void_p()
        n = C.c_size_t()
        _check(lib().mi_model_arena(self.h, C.byref(p), C.byref(n)), "arena")
        return p.value, n.value

    def type_histogram(self) -> dict:
        a = (C.c_int64 * 32)()
        lib().mi_model_type_histogram(self.h, a, 32)
        return {i: int(a[i]) for i in range(32) if a[i]}

    def token_text(self, tok: int) -> str:
        n = lib().mi_model_token_text(self.h, tok, None, 0)
        _check(n, "token_text")
        b = C.create_string_buffer(n + 1)
        lib().mi_model_token_text(self.h, tok, b, n + 1)
        return b.raw[:n].decode("utf-8", errors="replace")

    @property
    def bos(self):
        return lib().mi_model_token_bos(self.h)

    @property
    def eos(self):
        return lib().mi_model_token_eos(self.h)

    def is_eog(self, tok: int) -> bool:
        return lib().mi_model_token_is_eog(self.h, tok) == 1


class Context:
    """Owns an mi_ctx (llama_init_from_model + llama_free)."""

    def __init__(self, model: Model, n_ctx: int = 0, n_batch: int = 2048, n_ubatch: int = 512):
        h = lib().mi_ctx_create(model.h, n_ctx, n_batch, n_ubatch)
        if not h:
            raise EngineError(f"context creation failed: {last_error()}")
        self.h = h
        self.model = model
        self.n_ctx = lib().mi_n_ctx(h)
        self.n_batch = lib().mi_n_batch(h)

    def close(self):
        if getattr(self, "h", None):
            lib().mi_ctx_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decode(self, tokens, all_logits: bool = False) -> int:
        """mi_decode; all_logits=True is MI_OUT_ALL (output row i = the distribution after token i)."""
        t = np.ascontiguousarray(tokens, dtype=np.int32)
        rc = lib().mi_decode(self.h, t.ctypes.data_as(C.POINTER(C.c_int32)), t.size, 1 if all_logits else 0)
        _check(rc, "decode")
        return rc

    def topk(self, k: int = 10, row: int = -1):
        ids = np.empty(k, np.int32)
        vals = np.empty(k, np.float32)
        _check(lib().mi_topk(self.h, row, k, ids.ctypes.data_as(C.POINTER(C.c_int32)),
                             vals.ctypes.data_as(C.POINTER(C.c_float))), "topk")
        return ids, vals

    def gather(self, ids, row: int = -1):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        out = np.empty(ids.size, np.float32)
        _check(lib().mi_gather(self.h, row, ids.ctypes.data_as(C.POINTER(C.c_int32)), ids.size,
                               out.ctypes.data_as(C.POINTER(C.c_float))), "gather")
        return out

    def gather_rows(self, row0: int, ids) -> np.ndarray:
        """ids [n_rows][k] -> logits of rows row0.. at those ids (mi_gather_rows)."""
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        out = np.empty(ids.shape, np.float32)
        _check(lib().mi_gather_rows(self.h, row0, ids.shape[0], ids.ctypes.data_as(C.POINTER(C.c_int32)),
                                    ids.shape[1], out.ctypes.data_as(C.POINTER(C.c_float))), "gather_rows")
        return out

    def logits(self, row: int = -1) -> np.ndarray:
        p = lib().mi_logits(self.h, row)
        if not p:
            raise EngineError(f"logits: {last_error()}")
        return np.ctypeslib.as_array(p, shape=(self.model.n_vocab,)).copy()

    def synchronize(self):
        lib().mi_synchronize(self.h)

    def kv_clear(self):
        lib().mi_kv_clear(self.h)

    def kv_seq_rm(self, p0, p1):
        return _check(lib().mi_kv_seq_rm(self.h, p0, p1), "kv_seq_rm")

    def kv_seq_add(self, p0, p1, delta):
        return _check(lib().mi_kv_seq_add(self.h, p0, p1, delta), "kv_seq_add")

    def kv_seq_div(self, p0, p1, d):
        return _check(lib().mi_kv_seq_div(self.h, p0, p1, d), "kv_seq_div")

    @property
    def pos_max(self):
        return lib().mi_kv_pos_max(self.h)

    @property
    def n_cells(self):
        return lib().mi_kv_n_cells(self.h)

    def state_get(self) -> bytes:
        n = lib().mi_state_size(self.h)
        buf = np.empty(n, np.uint8)
        got = lib().mi_state_get(self.h, _ptr(buf), n)
        if got != n:
            raise EngineError(f"state_get: {last_error()}")
        return buf.tobytes()

    def state_set(self, data: bytes):
        buf = np.frombuffer(data, np.uint8).copy()
        got = lib().mi_state_set(self.h, _ptr(buf), buf.size)
        if got == 0:
            raise EngineError(f"state_set: {last_error()}")

    def prof_enable(self, stride: int):
        lib().mi_prof_enable(self.h, stride)

    def prof_read(self, n: int = 64) -> np.ndarray:
        a = np.zeros(n, np.float32)
        k = _check(lib().mi_prof_read(self.h, a.ctypes.data_as(C.POINTER(C.c_float)), n), "prof_read")
        return a[:k]

    @property
    def ffn_bytes(self) -> int:
        return lib().mi_prof_ffn_bytes(self.h)

    def decode_path(self) -> int:
        """1: decode steps within 512 cells run on the streaming GEMV (dgemv.hip); 0: gemv_kernel."""
        return int(lib().mi_decode_path(self.h))

    @property
    def prof_bytes(self) -> int:
        """Algorithmic bytes of the launch prof_read last timed (the FFN gate/up GEMV)."""
        return lib().mi_prof_bytes(self.h)

# ---- op-level entry points (parity tests / micro-benchmarks) ----

def op_gemv(type_: int, raw: np.ndarray, rows: int, K: int, x: np.ndarray, device: int = 0) -> np.ndarray:
    raw = np.ascontiguousarray(raw, np.uint8)
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty(rows, np.float32)
    _check(lib().mi_op_gemv(device, type_, _ptr(raw), rows, K, _ptr(x), _ptr(y)), "op_gemv")
    return y


def op_dgemv(role: int, type_: int, raw: np.ndarray, rows: int, K: int, x: np.ndarray, type2: int = -1,
             raw2=None, rows2: int = 0, resid=None, device: int = 0) -> np.ndarray:
    """mi_op_dgemv: the decode step's streaming GEMV launch of `role` (0 Q/K/V without RoPE, 1 residual
    add, 2 SwiGLU pair, 3 store, 4 residual add with x quantised inside the launch)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out_rows = rows + (rows2 if role == 0 and raw2 is not None else 0)
    y = np.empty(out_rows, np.float32)
    r = None if resid is None else np.ascontiguousarray(resid, dtype=np.float32)
    raw = np.ascontiguousarray(raw)
    raw2 = None if raw2 is None else np.ascontiguousarray(raw2)
    rc = lib().mi_op_dgemv(device, role, type_, raw.ctypes.data, rows, K, type2,
                           raw2.ctypes.data if raw2 is not None else None, rows2 if raw2 is not None else 0,
                           _ptr(x), _ptr(r) if r is not None else None, _ptr(y))
    _check(rc, "op_dgemv")
    return y


def op_gemv_bench(type_: int, raw: np.ndarray, rows: int, K: int, iters: int = 100, device: int = 0) -> float:
    raw = np.ascontiguousarray(raw, np.uint8)
    us = C.c_float()
    _check(lib().mi_op_gemv_bench(device, type_, _ptr(raw), rows, K, iters, C.byref(us)), "op_gemv_bench")
    return us.value


def op_dequant(type_: int, raw: np.ndarray, rows: int, K: int, device: int = 0) -> np.ndarray:
    raw = np.ascontiguousarray(raw, np.uint8)
    out = np.empty(rows * K, np.float32)
    _check(lib().mi_op_dequant(device, type_, _ptr(raw), rows, K, _ptr(out)), "op_dequant")
    return out


def op_quantize_q8_K(x: np.ndarray, device: int = 0):
    x = np.ascontiguousarray(x, np.float32)
    K = x.size
    qs = np.empty(K, np.int8)
    d = np.empty(K // 256, np.float32)
    bs = np.empty((K // 256) * 16, np.int32)
    _check(lib().mi_op_quantize_q8_K(device, _ptr(x), K, _ptr(qs), _ptr(d), _ptr(bs)), "op_quantize_q8_K")
    return qs, d, bs


def op_topk(logits: np.ndarray, k: int, device: int = 0):
    logits = np.ascontiguousarray(logits, np.float32)
    ids = np.empty(k, np.int32)
    vals = np.empty(k, np.float32)
    _check(lib().mi_op_topk(device, _ptr(logits), logits.size, k, _ptr(ids), _ptr(vals)), "op_topk")
    return ids, vals


def op_attention(q: np.ndarray, k16: np.ndarray, v16: np.ndarray, n_head_kv: int, cell_pos=None, pos=None,
                 device: int = 0) -> np.ndarray:
    """q: (n_head, hd) f32; k16/v16: (n_cells, n_head_kv*hd) f16 -> (n_head, hd) f32."""
    q = np.ascontiguousarray(q, np.float32)
    n_head, hd = q.shape
    k16 = np.ascontiguousarray(k16, np.float16)
    v16 = np.ascontiguousarray(v16, np.float16)
    n = k16.shape[0]
    cp = np.ascontiguousarray(np.arange(n) if cell_pos is None else cell_pos, np.int32)
    pos = n - 1 if pos is None else pos
    out = np.empty(n_head * hd, np.float32)
    _check(lib().mi_op_attention(device, n_head, n_head_kv, hd, n, _ptr(q), _ptr(k16), _ptr(v16), _ptr(cp), pos,
                                 _ptr(out)), "op_attention")
    return out.reshape(n_head, hd)


def op_gemm(type_: int, raw: np.ndarray, rows: int, K: int, x: np.ndarray, raw_up=None,
            device: int = 0) -> np.ndarray:
    """Prompt-batch GEMM (mmqs up to MI_MMQS_MAX tokens, mmq32 above) of x (ntok, K) f32 ->
    (ntok, rows); with raw_up the gate/up
    SwiGLU pair silu(gate . x) * (up . x)."""
    raw = np.ascontiguousarray(raw, np.uint8)
    x = np.ascontiguousarray(x, np.float32)
    ntok = x.shape[0]
    up = None if raw_up is None else np.ascontiguousarray(raw_up, np.uint8)
    y = np.empty((ntok, rows), np.float32)
    _check(lib().mi_op_gemm(device, type_, _ptr(raw), None if up is None else _ptr(up), rows, K, ntok, _ptr(x),
                            _ptr(y)), "op_gemm")
    return y


def op_attention_batch(q: np.ndarray, k16: np.ndarray, v16: np.ndarray, n_head_kv: int, tok_cell, tok_pos=None,
                       cell_pos=None, device: int = 0) -> np.ndarray:
    """q: (ntok, n_head, hd) f32; k16/v16: (n_cells, n_head_kv*hd) f16; token t in cell tok_cell[t] at
    position tok_pos[t] (default: its cell) -> (ntok, n_head, hd) f32 (attn_mfma)."""
    q = np.ascontiguousarray(q, np.float32)
    ntok, n_head, hd = q.shape
    k16 = np.ascontiguousarray(k16, np.float16)
    v16 = np.ascontiguousarray(v16, np.float16)
    n = k16.shape[0]
    cp = np.ascontiguousarray(np.arange(n) if cell_pos is None else cell_pos, np.int32)
    tc = np.ascontiguousarray(tok_cell, np.int32)
    tpos = np.ascontiguousarray(tc if tok_pos is None else tok_pos, np.int32)
    out = np.empty((ntok, n_head, hd), np.float32)
    _check(lib().mi_op_attention_batch(device, n_head, n_head_kv, hd, n, ntok, _ptr(q), _ptr(k16), _ptr(v16),
                                       _ptr(cp), _ptr(tc), _ptr(tpos), _ptr(out)), "op_attention_batch")
    return out
