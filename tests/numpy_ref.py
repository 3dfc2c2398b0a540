"""Independent numpy restatement of the reference embedding path (test infrastructure).

Same op order as reference bert.cpp:845-1012 and the same ggml rounding points
as oracle/bert_oracle.c (fp16 GELU/exp tables, Q8_0/Q8_1 activation
quantisation, fp16 activation rounding for F16 weights, f32 element-wise ops),
but every dot product / sum is evaluated in float64 instead of ggml's SIMD f32
accumulation order.  Used only to pin the C oracle (tests/test_oracle.py): the
two must agree to far tighter than the GPU tolerance.
"""
from __future__ import annotations

import numpy as np

from gguf_reader import GGUF

F32, F16, Q4_0, Q4_1 = 0, 1, 2, 3


def fp16(x):
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


_TABLES = None


def tables():
    """ggml_init's 64K-entry fp16 tables, restated with numpy float32 math."""
    global _TABLES
    if _TABLES is None:
        h = np.arange(65536, dtype=np.uint32).astype(np.uint16).view(np.float16).astype(np.float32)
        with np.errstate(all="ignore"):
            A, S = np.float32(0.044715), np.float32(0.79788456080286535587989211986876)
            inner = (A * h).astype(np.float64) * h + 1.0  # fma(A*x, x, 1)
            inner = inner.astype(np.float32)
            g = np.float32(0.5) * h * (np.float32(1.0) + np.tanh(S * h * inner))
            e = np.exp(h)
        _TABLES = (fp16(g), fp16(e))
    return _TABLES


def table_lookup(tab, x):
    idx = np.asarray(x, np.float32).astype(np.float16).view(np.uint16)
    return tab[idx]


def quant_q8(x, q8_1: bool):
    """ggml quantize_row_q8_0/q8_1 (AVX2): d = amax/127, q = rint(x*(127/amax))."""
    x = np.asarray(x, np.float32)
    b = x.reshape(x.shape[0], -1, 32)
    amax = np.abs(b).max(axis=2)
    d = (amax / np.float32(127)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(amax != 0, np.float32(127) / np.where(amax != 0, amax, 1), 0).astype(np.float32)
    q = np.rint(b * idv[..., None]).astype(np.int32)
    if not q8_1:
        d = fp16(d)
    s = (d * q.sum(axis=2).astype(np.float32)).astype(np.float32)
    return d, s, q


def layer_norm(x, w, b, eps):
    x = np.asarray(x, np.float32)
    mean = (x.astype(np.float64).sum(axis=1) / x.shape[1]).astype(np.float32)
    v = (x - mean[:, None]).astype(np.float32)
    var = ((v * v).astype(np.float64).sum(axis=1) / x.shape[1]).astype(np.float32)
    scale = (np.float32(1.0) / np.sqrt(var + np.float32(eps))).astype(np.float32)
    y = (v * scale[:, None]).astype(np.float32)
    y = (w[None, :] * y).astype(np.float32)
    return (y + b[None, :]).astype(np.float32)


class Model:
    def __init__(self, path: str):
        g = GGUF(path)
        self.g = g
        self.E = int(g.kv["bert.embedding_length"])
        self.I = int(g.kv["bert.feed_forward_length"])
        self.H = int(g.kv["bert.attention.head_count"])
        self.L = int(g.kv["bert.block_count"])
        self.eps = float(np.float32(g.kv["bert.attention.layer_norm_epsilon"]))
        self.word = g.f32("embeddings.word_embeddings.weight")
        self.pos = g.f32("embeddings.position_embeddings.weight")
        self.type = g.f32("embeddings.token_type_embeddings.weight")
        self.ln_e = (g.f32("embeddings.LayerNorm.weight"), g.f32("embeddings.LayerNorm.bias"))
        self.layers = []
        for il in range(self.L):
            p = f"encoder.layer.{il}."
            self.layers.append({k: self._mat(p + n) if n.endswith("dense.weight") or ".self." in n and n.endswith(
                "weight") else g.f32(p + n) for k, n in [
                ("q_w", "attention.self.query.weight"), ("q_b", "attention.self.query.bias"),
                ("k_w", "attention.self.key.weight"), ("k_b", "attention.self.key.bias"),
                ("v_w", "attention.self.value.weight"), ("v_b", "attention.self.value.bias"),
                ("o_w", "attention.output.dense.weight"), ("o_b", "attention.output.dense.bias"),
                ("ln1_w", "attention.output.LayerNorm.weight"), ("ln1_b", "attention.output.LayerNorm.bias"),
                ("i_w", "intermediate.dense.weight"), ("i_b", "intermediate.dense.bias"),
                ("o2_w", "output.dense.weight"), ("o2_b", "output.dense.bias"),
                ("ln2_w", "output.LayerNorm.weight"), ("ln2_b", "output.LayerNorm.bias")]})
        self.wtype = self.layers[0]["q_w"][0]

    def _mat(self, name):
        """Weight matrix in the form its ggml vec_dot needs: (type, payload)."""
        ne, typ, raw = self.g.raw(name)
        n, k = ne[1], ne[0]
        if typ in (F32, F16):
            return typ, self.g.f32(name).astype(np.float64)
        bs = 18 if typ == Q4_0 else 20
        blk = raw.reshape(n, k // 32, bs)
        d = blk[..., :2].copy().view(np.float16).astype(np.float64)[..., 0]
        qo = 2 if typ == Q4_0 else 4
        qs = blk[..., qo:]
        q = np.concatenate([qs & 15, qs >> 4], axis=2).astype(np.float64)
        if typ == Q4_0:
            return typ, ((q - 8) * d[..., None]).reshape(n, k)
        m = blk[..., 2:4].copy().view(np.float16).astype(np.float64)[..., 0]
        return typ, ((q * d[..., None]).reshape(n, k), m)

    def mul_mat_bias(self, mat, bias, x):
        typ, W = mat
        x = np.asarray(x, np.float32)
        if typ == F32:
            mm = x.astype(np.float64) @ W.T
        elif typ == F16:
            mm = fp16(x).astype(np.float64) @ W.T
        elif typ == Q4_0:
            d, _, q = quant_q8(x, False)
            a = (q * d[..., None].astype(np.float64)).reshape(x.shape)
            mm = a @ W.T
        else:
            Wq, m = W
            d, s, q = quant_q8(x, True)
            a = (q * d[..., None].astype(np.float64)).reshape(x.shape)
            mm = a @ Wq.T + s.astype(np.float64) @ m.T
        return (bias[None, :] + mm.astype(np.float32)).astype(np.float32)

    def eval(self, toks) -> np.ndarray:
        toks = np.asarray(toks)
        N, E, H = len(toks), self.E, self.H
        D = E // H
        gelu_t, exp_t = tables()
        x = (self.pos[:N] + (self.type[0][None, :] + self.word[toks])).astype(np.float32)
        x = layer_norm(x, *self.ln_e, self.eps)
        scale = np.float32(1.0) / np.sqrt(np.float32(D))
        for Lw in self.layers:
            Q = self.mul_mat_bias(Lw["q_w"], Lw["q_b"], x)
            K = self.mul_mat_bias(Lw["k_w"], Lw["k_b"], x)
            V = self.mul_mat_bias(Lw["v_w"], Lw["v_b"], x)
            ctx = np.zeros((N, E), np.float32)
            for h in range(H):
                sl = slice(h * D, (h + 1) * D)
                S = (Q[:, sl].astype(np.float64) @ K[:, sl].astype(np.float64).T).astype(np.float32) * scale
                mx = S.max(axis=1, keepdims=True)
                P = table_lookup(exp_t, (S - mx).astype(np.float32))
                r = (1.0 / P.astype(np.float64).sum(axis=1)).astype(np.float32)
                P = (P * r[:, None]).astype(np.float32)
                ctx[:, sl] = (P.astype(np.float64) @ V[:, sl].astype(np.float64)).astype(np.float32)
            o = self.mul_mat_bias(Lw["o_w"], Lw["o_b"], ctx)
            x1 = layer_norm((o + x).astype(np.float32), Lw["ln1_w"], Lw["ln1_b"], self.eps)
            u = self.mul_mat_bias(Lw["i_w"], Lw["i_b"], x1)
            u = table_lookup(gelu_t, u)
            f = self.mul_mat_bias(Lw["o2_w"], Lw["o2_b"], u)
            x = layer_norm((x1 + f).astype(np.float32), Lw["ln2_w"], Lw["ln2_b"], self.eps)
        inv = np.float32(1.0) / np.float32(N)
        m = (x.astype(np.float64) * np.float64(inv)).sum(axis=0).astype(np.float32)
        ss = (m * m).astype(np.float64).sum()
        length = np.sqrt(np.float32(ss))
        return (m * (np.float32(1.0) / length)).astype(np.float32)
