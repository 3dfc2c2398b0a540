"""ctypes binding of the CPU oracle (oracle/bert_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product path.  Builds
oracle/_build/liboracle.so on first use if it is missing (gcc is in the image
on both the dev container and the GPU box).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "liboracle.so")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return SO


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        L = ctypes.CDLL(SO)
        L.oracle_load.restype = ctypes.c_void_p
        L.oracle_load.argtypes = [ctypes.c_char_p]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_hparams.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]
        L.oracle_eval.restype = ctypes.c_int
        L.oracle_eval.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_float)]
        L.oracle_eval_batch.restype = ctypes.c_int
        L.oracle_eval_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                        ctypes.POINTER(ctypes.c_int32), ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_float), ctypes.c_int]
        L.oracle_f32_to_f16.restype = ctypes.c_uint16
        L.oracle_f32_to_f16.argtypes = [ctypes.c_float]
        L.oracle_f16_to_f32.restype = ctypes.c_float
        L.oracle_f16_to_f32.argtypes = [ctypes.c_uint16]
        L.oracle_tab_gelu.restype = ctypes.c_uint16
        L.oracle_tab_gelu.argtypes = [ctypes.c_uint16]
        L.oracle_tab_exp.restype = ctypes.c_uint16
        L.oracle_tab_exp.argtypes = [ctypes.c_uint16]
        L.oracle_quantize_q8.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_int64, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                         ctypes.POINTER(ctypes.c_int8)]
        L.oracle_max_threads.restype = ctypes.c_int
        L.oracle_set_dot_variant.argtypes = [ctypes.c_int]
        L.oracle_set_attn_form.argtypes = [ctypes.c_int]
        L.oracle_set_simd.argtypes = [ctypes.c_int]
        L.oracle_simd_available.restype = ctypes.c_int
        L.oracle_embed_ln.restype = ctypes.c_int
        L.oracle_embed_ln.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_float)]
        L.oracle_eval_layers.restype = ctypes.c_int
        L.oracle_eval_layers.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_float)]
        L.oracle_layer.restype = ctypes.c_int
        L.oracle_layer.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_float)]
        _lib = L
    return _lib


# dot-kernel summation orders of the ggml builds the oracle can replay
# (bert_oracle.c oracle_set_dot_variant): the checker uses "avx2"
DOT_VARIANTS = {"avx2": 0, "generic": 1, "lanes16": 2}


# attention arithmetic (bert_oracle.c oracle_set_attn_form): "ggml" (the
# checker), or "gpu_operands" — a diagnostic, not a ggml build
ATTN_FORMS = {"ggml": 0, "gpu_operands": 1}


def set_attn_form(name: str) -> None:
    lib().oracle_set_attn_form(ATTN_FORMS[name])


def set_dot_variant(name: str) -> None:
    lib().oracle_set_dot_variant(DOT_VARIANTS[name])


def simd_available() -> bool:
    """The host CPU runs the AVX2 / FMA / F16C intrinsics form (bert_oracle.c oracle_set_simd)."""
    return bool(lib().oracle_simd_available())


def set_simd(on: bool) -> None:
    """The AVX2-order checker written with AVX2 intrinsics (bitwise the scalar
    form; only the CPU baseline's speed changes).  Off by default."""
    if on and not simd_available():
        raise RuntimeError("host CPU lacks AVX2/FMA/F16C")
    lib().oracle_set_simd(1 if on else 0)


class Oracle:
    def __init__(self, path: str):
        self.L = lib()
        self.m = self.L.oracle_load(path.encode())
        if not self.m:
            raise RuntimeError(f"oracle failed to load {path}")
        hp = (ctypes.c_int32 * 7)()
        self.L.oracle_hparams(self.m, hp)
        self.n_vocab, self.n_max, self.n_embd, self.n_inter, self.n_head, self.n_layer, self.wtype = list(hp)

    def __del__(self):
        if getattr(self, "m", None):
            self.L.oracle_free(self.m)
            self.m = None

    def embed_ln(self, tokens) -> np.ndarray:
        """The embeddings + LayerNorm stage of one sentence (reference bert.cpp:865-898): [N, E] f32."""
        t = np.ascontiguousarray(np.asarray(tokens, np.int32))
        out = np.zeros((len(t), self.n_embd), np.float32)
        rc = self.L.oracle_embed_ln(self.m, t.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(t),
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        if rc != 0:
            raise RuntimeError(f"oracle_embed_ln failed ({rc})")
        return out

    def eval_layers(self, tokens) -> np.ndarray:
        """The residual stream of one sentence after every stage: [n_layer + 1, N, E]
        (stage 0 the embedding LayerNorm, stage l + 1 encoder layer l; reference
        bert.cpp:865-993)."""
        t = np.ascontiguousarray(np.asarray(tokens, np.int32))
        out = np.zeros((self.n_layer + 1, len(t), self.n_embd), np.float32)
        rc = self.L.oracle_eval_layers(self.m, t.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(t),
                                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        if rc != 0:
            raise RuntimeError(f"oracle_eval_layers failed ({rc})")
        return out

    def layer(self, il: int, x: np.ndarray) -> np.ndarray:
        """Encoder layer il (reference bert.cpp:900-993) of one sentence applied to a
        given input stream x [N, E] (e.g. the GPU's own previous stage)."""
        x = np.ascontiguousarray(x, np.float32)
        out = np.zeros_like(x)
        rc = self.L.oracle_layer(self.m, il, x.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), x.shape[0],
                                 out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        if rc != 0:
            raise RuntimeError(f"oracle_layer failed ({rc})")
        return out

    def eval_batch(self, token_lists, n_threads: int = 0) -> np.ndarray:
        lens = [len(t) for t in token_lists]
        offs = np.zeros(len(lens) + 1, dtype=np.int32)
        offs[1:] = np.cumsum(lens)
        toks = np.ascontiguousarray(np.concatenate([np.asarray(t, dtype=np.int32) for t in token_lists]))
        out = np.zeros((len(lens), self.n_embd), dtype=np.float32)
        rc = self.L.oracle_eval_batch(self.m, toks.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                      offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(lens),
                                      out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n_threads)
        if rc != 0:
            raise RuntimeError(f"oracle_eval_batch failed ({rc})")
        return out


def quantize_q8(x: np.ndarray, q8_1: bool = False):
    """Row-block Q8 quantisation exactly as the oracle (ggml AVX2 quantize_row_q8_x)."""
    x = np.ascontiguousarray(x, dtype=np.float32).ravel()
    nb = x.size // 32
    d = np.zeros(nb, np.float32)
    s = np.zeros(nb, np.float32)
    q = np.zeros(x.size, np.int8)
    lib().oracle_quantize_q8(x.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), x.size, int(q8_1),
                             d.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                             s.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                             q.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)))
    return d, s, q
