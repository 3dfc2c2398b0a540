"""Minimal pure-Python GGUF v2/v3 reader (test infrastructure).

Independent of both C/C++ readers (csrc/gguf_io.cpp, oracle/bert_oracle.c) so
the numpy restatement in tests/numpy_ref.py checks the oracle with a third
implementation of the container format.
"""
from __future__ import annotations

import struct

import numpy as np

_SCALAR = {0: "<B", 1: "<b", 2: "<H", 3: "<h", 4: "<I", 5: "<i", 6: "<f", 7: "<?", 10: "<Q", 11: "<q", 12: "<d"}
TYPE_ROW = {0: (1, 4), 1: (1, 2), 2: (32, 18), 3: (32, 20)}  # ggml type -> (block elems, block bytes)


class GGUF:
    def __init__(self, path: str):
        self.buf = np.memmap(path, dtype=np.uint8, mode="r")
        self.p = 0
        magic, self.version = struct.unpack_from("<II", self.buf, 0)
        assert magic == 0x46554747 and self.version in (2, 3)
        n_t, n_kv = struct.unpack_from("<QQ", self.buf, 8)
        self.p = 24
        self.kv = {}
        for _ in range(n_kv):
            k = self._str()
            t = self._u32()
            self.kv[k] = self._val(t)
        self.tensors = {}
        for _ in range(n_t):
            name = self._str()
            nd = self._u32()
            ne = [struct.unpack_from("<Q", self.buf, self.p + 8 * i)[0] for i in range(nd)]
            self.p += 8 * nd
            typ = self._u32()
            off = struct.unpack_from("<Q", self.buf, self.p)[0]
            self.p += 8
            self.tensors[name] = (ne, typ, off)
        align = int(self.kv.get("general.alignment", 32))
        self.data = (self.p + align - 1) // align * align

    def _u32(self):
        v = struct.unpack_from("<I", self.buf, self.p)[0]
        self.p += 4
        return v

    def _str(self):
        n = struct.unpack_from("<Q", self.buf, self.p)[0]
        s = bytes(self.buf[self.p + 8: self.p + 8 + n]).decode("utf-8", "replace")
        self.p += 8 + n
        return s

    def _val(self, t):
        if t == 8:
            return self._str()
        if t == 9:
            at = self._u32()
            n = struct.unpack_from("<Q", self.buf, self.p)[0]
            self.p += 8
            if at == 8:
                return [self._str() for _ in range(n)]
            fmt = _SCALAR[at]
            sz = struct.calcsize(fmt)
            arr = np.frombuffer(bytes(self.buf[self.p: self.p + n * sz]), dtype=np.dtype(fmt))
            self.p += n * sz
            return arr
        fmt = _SCALAR[t]
        v = struct.unpack_from(fmt, self.buf, self.p)[0]
        self.p += struct.calcsize(fmt)
        return v

    def raw(self, name: str):
        ne, typ, off = self.tensors[name]
        be, bb = TYPE_ROW[typ]
        nrows = int(np.prod(ne[1:])) if len(ne) > 1 else 1
        nbytes = nrows * (ne[0] // be) * bb
        start = self.data + off
        return ne, typ, np.asarray(self.buf[start: start + nbytes])

    def f32(self, name: str) -> np.ndarray:
        """Dequantise a tensor to float32 with shape [rows, ne0] (ggml get_rows semantics)."""
        ne, typ, b = self.raw(name)
        nrows = int(np.prod(ne[1:])) if len(ne) > 1 else 1
        if typ == 0:
            out = b.view(np.float32).copy()
        elif typ == 1:
            out = b.view(np.float16).astype(np.float32)
        elif typ == 2:
            blk = b.reshape(-1, 18)
            d = blk[:, :2].copy().view(np.float16).astype(np.float32)
            qs = blk[:, 2:]
            q = np.concatenate([(qs & 15).astype(np.int32) - 8, (qs >> 4).astype(np.int32) - 8], axis=1)
            out = (q.astype(np.float32) * d).ravel()
        elif typ == 3:
            blk = b.reshape(-1, 20)
            d = blk[:, :2].copy().view(np.float16).astype(np.float32)
            m = blk[:, 2:4].copy().view(np.float16).astype(np.float32)
            qs = blk[:, 4:]
            q = np.concatenate([(qs & 15), (qs >> 4)], axis=1).astype(np.float32)
            # ggml's x*d + m is contracted to an fma by gcc -mfma: emulate with float64 then round
            out = (q.astype(np.float64) * d + m).astype(np.float32).ravel()
        else:
            raise ValueError(typ)
        return out.reshape(nrows, ne[0]) if len(ne) > 1 else out
