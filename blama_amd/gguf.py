"""Minimal GGUF v3 reader/writer (host tooling).

The engine parses GGUF itself in C++ (``blama_amd/csrc/gguf.cpp``); this Python
module exists to *write* synthetic models with the exact tensor names, shapes
and per-tensor quant types of the BASELINE.json configs (no model files can be
downloaded here), and to read a GGUF back for the CPU oracle in tests.

Format: magic "GGUF", u32 version=3, u64 n_tensors, u64 n_kv, KV pairs,
tensor infos (name, n_dims, ne[], type, offset), pad to general.alignment,
tensor data.  This mirrors what ``llama_model_load_from_file``
(called at /root/reference/inference/code/llama/Model.cpp:52) consumes.
"""
from __future__ import annotations

import io
import os
import struct
from dataclasses import dataclass

import numpy as np

GGUF_MAGIC = b"GGUF"
GGUF_VERSION = 3
DEFAULT_ALIGNMENT = 32

# gguf_type
T_UINT8, T_INT8, T_UINT16, T_INT16, T_UINT32, T_INT32, T_FLOAT32, T_BOOL, T_STRING, \
    T_ARRAY, T_UINT64, T_INT64, T_FLOAT64 = range(13)

_SCALAR_FMT = {T_UINT8: "<B", T_INT8: "<b", T_UINT16: "<H", T_INT16: "<h", T_UINT32: "<I",
               T_INT32: "<i", T_FLOAT32: "<f", T_BOOL: "<?", T_UINT64: "<Q", T_INT64: "<q",
               T_FLOAT64: "<d"}

# ggml type -> (block elems, block bytes)
GGML_BLOCK = {0: (1, 4), 1: (1, 2), 8: (32, 34), 12: (256, 144), 13: (256, 176),
              14: (256, 210), 30: (1, 2)}


def tensor_nbytes(ggml_type: int, shape) -> int:
    n = 1
    for s in shape:
        n *= int(s)
    be, bb = GGML_BLOCK[ggml_type]
    assert n % be == 0
    return n // be * bb


@dataclass
class GGUFTensor:
    name: str
    type: int
    shape: tuple   # ne order (ne0 innermost)
    offset: int    # relative to the data section
    data: np.ndarray | None = None  # uint8 view


class GGUFWriter:
    def __init__(self, alignment: int = DEFAULT_ALIGNMENT):
        self.kv: list[tuple[str, int, object]] = []
        self.tensors: list[tuple[str, int, tuple, np.ndarray]] = []
        self.alignment = alignment

    def add(self, key: str, vtype: int, value):
        self.kv.append((key, vtype, value))

    def add_str(self, key, v): self.add(key, T_STRING, v)
    def add_u32(self, key, v): self.add(key, T_UINT32, int(v))
    def add_i32(self, key, v): self.add(key, T_INT32, int(v))
    def add_f32(self, key, v): self.add(key, T_FLOAT32, float(v))
    def add_bool(self, key, v): self.add(key, T_BOOL, bool(v))

    def add_array(self, key, etype, values):
        self.add(key, T_ARRAY, (etype, list(values)))

    def add_tensor(self, name: str, ggml_type: int, shape, data: np.ndarray | None = None):
        """data=None declares the tensor only; fill it in place via to_bytes(fill=...)."""
        n = tensor_nbytes(ggml_type, shape)
        if data is not None:
            data = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
            assert data.size == n, (name, data.size, shape)
        self.tensors.append((name, ggml_type, tuple(int(s) for s in shape), data))

    @staticmethod
    def _str(b: io.BytesIO, s: str):
        e = s.encode("utf-8")
        b.write(struct.pack("<Q", len(e)))
        b.write(e)

    def _val(self, b, vtype, v):
        if vtype == T_STRING:
            self._str(b, v)
        elif vtype == T_ARRAY:
            et, vals = v
            b.write(struct.pack("<IQ", et, len(vals)))
            if et == T_STRING:
                for s in vals:
                    self._str(b, s)
            else:
                b.write(np.asarray(vals, dtype=np.dtype(_SCALAR_FMT[et])).tobytes())
        else:
            b.write(struct.pack(_SCALAR_FMT[vtype], v))

    def header_bytes(self) -> tuple[bytes, list[int]]:
        b = io.BytesIO()
        b.write(GGUF_MAGIC)
        b.write(struct.pack("<IQQ", GGUF_VERSION, len(self.tensors), len(self.kv) + 1))
        self._str(b, "general.alignment")
        b.write(struct.pack("<I", T_UINT32))
        b.write(struct.pack("<I", self.alignment))
        for k, t, v in self.kv:
            self._str(b, k)
            b.write(struct.pack("<I", t))
            self._val(b, t, v)
        offs = []
        off = 0
        for name, gt, shape, data in self.tensors:
            self._str(b, name)
            b.write(struct.pack("<I", len(shape)))
            b.write(struct.pack("<%dQ" % len(shape), *shape))
            b.write(struct.pack("<IQ", gt, off))
            offs.append(off)
            n = tensor_nbytes(gt, shape)
            off += (n + self.alignment - 1) // self.alignment * self.alignment
        hdr = b.getvalue()
        pad = (-len(hdr)) % self.alignment
        return hdr + b"\0" * pad, offs

    def to_bytes(self, fill=None) -> np.ndarray:
        """The whole file as one uint8 array (no disk round trip needed).

        fill(name, ggml_type, shape, view) is called for declared-only tensors
        and writes the tensor bytes into ``view`` in place (no second copy)."""
        hdr, offs = self.header_bytes()
        total = len(hdr)
        if self.tensors:
            name, gt, shape, _ = self.tensors[-1]
            total += offs[-1] + tensor_nbytes(gt, shape)
        buf = np.empty(total, np.uint8)
        buf[: len(hdr)] = np.frombuffer(hdr, np.uint8)
        prev_end = len(hdr)
        jobs = []
        for (name, gt, shape, data), off in zip(self.tensors, offs):
            a = len(hdr) + off
            n = tensor_nbytes(gt, shape)
            buf[prev_end:a] = 0
            view = buf[a:a + n]
            if data is not None:
                view[:] = data
            else:
                jobs.append((name, gt, shape, view))
            prev_end = a + n
        # each declared tensor is filled from its own generator (synthetic._rng keys it by name),
        # so the bytes do not depend on the order or the thread that fills them
        workers = min(16, os.cpu_count() or 1)
        if workers > 1 and len(jobs) > 1:
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(workers) as ex:
                for f in [ex.submit(fill, *j) for j in jobs]:
                    f.result()
        else:
            for j in jobs:
                fill(*j)
        return buf

    def write(self, path: str):
        hdr, offs = self.header_bytes()
        with open(path, "wb") as f:
            f.write(hdr)
            pos = 0
            for (name, gt, shape, data), off in zip(self.tensors, offs):
                assert data is not None, "write() needs tensor data; use to_bytes(fill=...)"
                if off > pos:
                    f.write(b"\0" * (off - pos))
                    pos = off
                f.write(data.tobytes())
                pos += data.size


class GGUFReader:
    """Parse a GGUF image (bytes / uint8 array / path). Tensor data are views."""

    def __init__(self, src):
        if isinstance(src, (str, bytes)) and not isinstance(src, bytes):
            self.buf = np.memmap(src, dtype=np.uint8, mode="r")
        else:
            self.buf = np.frombuffer(src, np.uint8) if isinstance(src, (bytes, bytearray)) else src
        self.pos = 0
        self.kv: dict[str, object] = {}
        self.tensors: dict[str, GGUFTensor] = {}
        self._parse()

    def _read(self, n):
        b = self.buf[self.pos:self.pos + n].tobytes()
        self.pos += n
        return b

    def _u(self, fmt):
        sz = struct.calcsize(fmt)
        return struct.unpack(fmt, self._read(sz))[0]

    def _s(self):
        n = self._u("<Q")
        return self._read(n).decode("utf-8", errors="replace")

    def _val(self, t):
        if t == T_STRING:
            return self._s()
        if t == T_ARRAY:
            et = self._u("<I")
            n = self._u("<Q")
            if et == T_STRING:
                return [self._s() for _ in range(n)]
            dt = np.dtype(_SCALAR_FMT[et])
            arr = np.frombuffer(self._read(n * dt.itemsize), dtype=dt)
            return arr
        return self._u(_SCALAR_FMT[t])

    def _parse(self):
        if self._read(4) != GGUF_MAGIC:
            raise ValueError("not a GGUF file")
        ver = self._u("<I")
        if ver not in (2, 3):
            raise ValueError(f"unsupported GGUF version {ver}")
        nt = self._u("<Q")
        nkv = self._u("<Q")
        for _ in range(nkv):
            k = self._s()
            t = self._u("<I")
            self.kv[k] = self._val(t)
        infos = []
        for _ in range(nt):
            name = self._s()
            nd = self._u("<I")
            shape = tuple(self._u("<Q") for _ in range(nd))
            gt = self._u("<I")
            off = self._u("<Q")
            infos.append(GGUFTensor(name, gt, shape, off))
        align = int(self.kv.get("general.alignment", DEFAULT_ALIGNMENT))
        data_start = (self.pos + align - 1) // align * align
        for ti in infos:
            n = tensor_nbytes(ti.type, ti.shape)
            a = data_start + ti.offset
            ti.data = self.buf[a:a + n]
            self.tensors[ti.name] = ti
