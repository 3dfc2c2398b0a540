"""Python host-side mirror of the drop-in C ABI (include/bert.h + bert_amd.h).

`BertModel` behaves like the class in the reference's examples/sample_dylib.py
(reference examples/sample_dylib.py:15-60): same constructor argument, same
`encode(sentences, batch_size)` contract, same ctypes signatures — only the
library path points at this repo's build/libbert.so.  The extra methods expose
the bert_amd.h extensions used by bench.py and the GPU tests (device-resident
evaluation on a caller stream, per-kernel timing, the synthetic-model
generator).

There is no CPU fallback: constructing a model on a host without a visible
MI355X raises, because the library itself refuses to load (runtime.cpp).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence, Union

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# BERT_AMD_LIB: another build of the library (development A/B runs only)
LIB_PATH = os.environ.get("BERT_AMD_LIB") or os.path.join(REPO, "build", "libbert.so")

F_P = ctypes.POINTER(ctypes.c_float)
I_P = ctypes.POINTER(ctypes.c_int32)

# every symbol include/bert.h and include/bert_amd.h declare
ABI_SYMBOLS = [
    "bert_params_parse", "bert_load_from_file", "bert_free", "bert_encode", "bert_encode_batch",
    "bert_tokenize", "bert_eval", "bert_eval_batch", "bert_n_embd", "bert_n_max_tokens",
    "bert_vocab_id_to_token", "bert_model_quantize",
]
EXT_SYMBOLS = [
    "bert_amd_load", "bert_amd_n_devices", "bert_amd_hparams", "bert_amd_eval_device",
    "bert_amd_profile_enable", "bert_amd_profile_read", "bert_amd_synth_model", "bert_amd_tokenize_json",
    "bert_amd_debug_embed", "bert_amd_workspace_rows", "bert_amd_last_error", "bert_amd_load_opts",
    "bert_amd_debug_layers", "bert_amd_set_option", "bert_amd_get_option", "bert_amd_shard_cuts",
]

# model shapes of BASELINE.json's configs
SHAPES = {
    "minilm": dict(n_vocab=30522, n_max_tokens=512, n_embd=384, n_intermediate=1536, n_head=12, n_layer=6),
    "e5-base": dict(n_vocab=250002, n_max_tokens=512, n_embd=768, n_intermediate=3072, n_head=12, n_layer=12),
    "bge-large": dict(n_vocab=30522, n_max_tokens=512, n_embd=1024, n_intermediate=4096, n_head=16, n_layer=24),
}
FTYPES = {"f32": 0, "f16": 1, "q4_0": 2, "q4_1": 3}

_lib = None


def lib() -> ctypes.CDLL:
    """Load build/libbert.so and declare every exported signature."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run `make` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    L.bert_load_from_file.restype = ctypes.c_void_p
    L.bert_load_from_file.argtypes = [ctypes.c_char_p]
    L.bert_free.argtypes = [ctypes.c_void_p]
    L.bert_n_embd.restype = ctypes.c_int32
    L.bert_n_embd.argtypes = [ctypes.c_void_p]
    L.bert_n_max_tokens.restype = ctypes.c_int32
    L.bert_n_max_tokens.argtypes = [ctypes.c_void_p]
    L.bert_encode_batch.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(F_P)]
    L.bert_encode.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_char_p, F_P]
    L.bert_tokenize.argtypes = [ctypes.c_void_p, ctypes.c_char_p, I_P, I_P, ctypes.c_int32]
    L.bert_eval.argtypes = [ctypes.c_void_p, ctypes.c_int32, I_P, ctypes.c_int32, F_P]
    L.bert_eval_batch.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(I_P), I_P,
                                  ctypes.POINTER(F_P)]
    L.bert_vocab_id_to_token.restype = ctypes.c_char_p
    L.bert_vocab_id_to_token.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.bert_model_quantize.restype = ctypes.c_bool
    L.bert_model_quantize.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    L.bert_amd_load.restype = ctypes.c_void_p
    L.bert_amd_load.argtypes = [ctypes.c_char_p, I_P, ctypes.c_int32]
    L.bert_amd_load_opts.restype = ctypes.c_void_p
    L.bert_amd_load_opts.argtypes = [ctypes.c_char_p, I_P, ctypes.c_int32, ctypes.c_char_p]
    L.bert_amd_n_devices.restype = ctypes.c_int32
    L.bert_amd_n_devices.argtypes = [ctypes.c_void_p]
    L.bert_amd_hparams.restype = ctypes.c_int32
    L.bert_amd_hparams.argtypes = [ctypes.c_void_p, I_P]
    L.bert_amd_eval_device.restype = ctypes.c_int32
    L.bert_amd_eval_device.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, I_P,
                                       ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
    L.bert_amd_profile_enable.restype = ctypes.c_int32
    L.bert_amd_profile_enable.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.bert_amd_profile_read.restype = ctypes.c_int32
    L.bert_amd_profile_read.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32, F_P, I_P, ctypes.c_int32]
    L.bert_amd_synth_model.restype = ctypes.c_int
    L.bert_amd_synth_model.argtypes = [ctypes.c_char_p] + [ctypes.c_int32] * 7 + [ctypes.c_uint64, ctypes.c_float]
    L.bert_amd_tokenize_json.restype = ctypes.c_int32
    L.bert_amd_tokenize_json.argtypes = [ctypes.c_char_p, ctypes.c_char_p, I_P, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
    L.bert_amd_debug_embed.restype = ctypes.c_int32
    L.bert_amd_debug_embed.argtypes = [ctypes.c_void_p, I_P, I_P, ctypes.c_int32, F_P, ctypes.c_void_p, ctypes.c_void_p]
    L.bert_amd_debug_layers.restype = ctypes.c_int32
    L.bert_amd_debug_layers.argtypes = [ctypes.c_void_p, I_P, I_P, ctypes.c_int32, F_P, ctypes.c_void_p, ctypes.c_void_p]
    L.bert_amd_set_option.restype = ctypes.c_int32
    L.bert_amd_set_option.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32]
    L.bert_amd_get_option.restype = ctypes.c_int32
    L.bert_amd_get_option.argtypes = [ctypes.c_void_p, ctypes.c_char_p, I_P]
    L.bert_amd_shard_cuts.restype = ctypes.c_int32
    L.bert_amd_shard_cuts.argtypes = [ctypes.c_int32, I_P, ctypes.c_int32, I_P]
    L.bert_amd_workspace_rows.restype = ctypes.c_int64
    L.bert_amd_workspace_rows.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.bert_amd_last_error.restype = ctypes.c_char_p
    _lib = L
    return L


def last_error() -> str:
    return lib().bert_amd_last_error().decode("utf-8", "replace")


def synth_model(path: str, shape: Union[str, dict] = "minilm", ftype: str = "q4_0", seed: int = 20250117,
                w_std: float = 0.05, **over) -> str:
    """Write a deterministic synthetic GGUF (csrc/synth.cpp) and return its path."""
    hp = dict(SHAPES[shape]) if isinstance(shape, str) else dict(shape)
    hp.update(over)
    rc = lib().bert_amd_synth_model(path.encode(), hp["n_vocab"], hp["n_max_tokens"], hp["n_embd"],
                                    hp["n_intermediate"], hp["n_head"], hp["n_layer"], FTYPES[ftype], seed, w_std)
    if rc != 0:
        raise RuntimeError(f"bert_amd_synth_model failed ({rc})")
    return path


def tokenize_json(tokenizer_json: str, text: str, n_max: int = 512, frame: bool = False,
                  cls_id: int = 101, sep_id: int = 102, pad_id: int = 0) -> List[int]:
    """Native tokenizer on a tokenizer.json string (no model, no GPU)."""
    buf = (ctypes.c_int32 * n_max)()
    n = lib().bert_amd_tokenize_json(tokenizer_json.encode("utf-8"), text.encode("utf-8"), buf, n_max,
                                     1 if frame else 0, cls_id, sep_id, pad_id)
    if n < 0:
        raise RuntimeError(last_error())
    return list(buf[:n])


def shard_cuts(n_tokens: Sequence[int], n_replicas: int) -> List[int]:
    """bert_eval_batch's split of a batch over n_replicas devices (no GPU needed)."""
    nt = np.ascontiguousarray(np.asarray(n_tokens, np.int32))
    cut = np.zeros(n_replicas + 1, np.int32)
    if lib().bert_amd_shard_cuts(len(nt), nt.ctypes.data_as(I_P), n_replicas, cut.ctypes.data_as(I_P)) != 0:
        raise ValueError(last_error())
    return cut.tolist()


def quantize(src: str, dst: str, ftype: str) -> bool:
    return bool(lib().bert_model_quantize(src.encode(), dst.encode(), FTYPES[ftype]))


class BertModel:
    """Mirror of examples/sample_dylib.py's BertModel, on the GPU library."""

    def __init__(self, fname: str, devices: Sequence[int] | None = None, options: str | dict | None = None):
        """devices: replica devices (None: bert_load_from_file, every visible one);
        options: bert_amd_load_opts' "key=value;..." string or a dict of them."""
        L = lib()
        self.lib = L
        if isinstance(options, dict):
            options = ";".join(f"{k}={v}" for k, v in options.items())
        if devices is None and options is None:
            self.ctx = L.bert_load_from_file(fname.encode("utf-8"))
        else:
            arr = (ctypes.c_int32 * len(devices))(*devices) if devices else None
            self.ctx = L.bert_amd_load_opts(fname.encode("utf-8"), arr, len(devices) if devices else 0,
                                            options.encode() if options else None)
        if not self.ctx:
            raise RuntimeError(f"failed to load {fname}: {last_error()}")
        self.n_embd = L.bert_n_embd(self.ctx)
        self.n_max_tokens = L.bert_n_max_tokens(self.ctx)
        hp = (ctypes.c_int32 * 7)()
        L.bert_amd_hparams(self.ctx, hp)
        self.hparams = list(hp)
        self.n_devices = L.bert_amd_n_devices(self.ctx)

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.bert_free(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- reference API
    def encode(self, sentences: Union[str, List[str]], batch_size: int = 16, n_threads: int = 6) -> np.ndarray:
        single = isinstance(sentences, str)
        if single:
            sentences = [sentences]
        n = len(sentences)
        emb = np.zeros((n, self.n_embd), dtype=np.float32)
        ptrs = (F_P * n)(*[e.ctypes.data_as(F_P) for e in emb])
        texts = (ctypes.c_char_p * n)(*[s.encode("utf-8") for s in sentences])
        self.lib.bert_encode_batch(self.ctx, n_threads, batch_size, n, texts, ptrs)
        return emb[0] if single else emb

    def tokenize(self, text: str, n_max: int | None = None) -> List[int]:
        n_max = n_max or self.n_max_tokens
        buf = (ctypes.c_int32 * n_max)()
        n = ctypes.c_int32(0)
        self.lib.bert_tokenize(self.ctx, text.encode("utf-8"), buf, ctypes.byref(n), n_max)
        return list(buf[: n.value])

    def eval_batch(self, token_lists: Union[Sequence[Sequence[int]], np.ndarray]) -> np.ndarray:
        """bert_eval_batch over host token lists (or a 2-D int32 array of equal-length
        sentences) -> [n, n_embd] float32."""
        n = len(token_lists)
        emb = np.full((n, self.n_embd), np.nan, dtype=np.float32)
        if isinstance(token_lists, np.ndarray) and token_lists.ndim == 2:
            # fixed-length batch: the pointer arrays are address arithmetic (no per-row objects)
            a = np.ascontiguousarray(token_lists, dtype=np.int32)
            tptr = (a.ctypes.data + np.arange(n, dtype=np.uint64) * np.uint64(a.strides[0])).astype(np.uint64)
            optr = (emb.ctypes.data + np.arange(n, dtype=np.uint64) * np.uint64(emb.strides[0])).astype(np.uint64)
            ntok = np.full(n, a.shape[1], np.int32)
            self.lib.bert_eval_batch(self.ctx, 1, n, ctypes.cast(tptr.ctypes.data, ctypes.POINTER(I_P)),
                                     ntok.ctypes.data_as(I_P), ctypes.cast(optr.ctypes.data, ctypes.POINTER(F_P)))
            return emb
        arrs = [np.ascontiguousarray(np.asarray(t, dtype=np.int32)) for t in token_lists]
        tok_p = (I_P * n)(*[a.ctypes.data_as(I_P) for a in arrs])
        ntok = (ctypes.c_int32 * n)(*[len(a) for a in arrs])
        out_p = (F_P * n)(*[e.ctypes.data_as(F_P) for e in emb])
        self.lib.bert_eval_batch(self.ctx, 1, n, tok_p, ntok, out_p)
        return emb

    def prepared_batch(self, token_lists: Sequence[Sequence[int]]):
        """(run, emb): run() calls bert_eval_batch on pointer arrays built once here
        (timing loops measure the C call, not the Python marshalling)."""
        n = len(token_lists)
        emb = np.full((n, self.n_embd), np.nan, dtype=np.float32)
        arrs = [np.ascontiguousarray(np.asarray(t, dtype=np.int32)) for t in token_lists]
        tok_p = (I_P * n)(*[a.ctypes.data_as(I_P) for a in arrs])
        ntok = (ctypes.c_int32 * n)(*[len(a) for a in arrs])
        out_p = (F_P * n)(*[e.ctypes.data_as(F_P) for e in emb])

        keep = (arrs, emb)  # the pointer arrays address these buffers

        def run():
            self.lib.bert_eval_batch(self.ctx, 1, n, tok_p, ntok, out_p)
            return keep[1]

        return run, emb

    def eval(self, tokens: Sequence[int]) -> np.ndarray:
        a = np.ascontiguousarray(np.asarray(tokens, dtype=np.int32))
        out = np.full(self.n_embd, np.nan, dtype=np.float32)
        self.lib.bert_eval(self.ctx, 1, a.ctypes.data_as(I_P), len(a), out.ctypes.data_as(F_P))
        return out

    # ---- extensions
    def eval_device(self, d_tokens_ptr: int, d_offsets_ptr: int, h_offsets: np.ndarray, n_seqs: int,
                    d_out_ptr: int, stream: int = 0, slot: int = 0) -> None:
        h = np.ascontiguousarray(h_offsets, dtype=np.int32)
        rc = self.lib.bert_amd_eval_device(self.ctx, slot, ctypes.c_void_p(d_tokens_ptr),
                                           ctypes.c_void_p(d_offsets_ptr), h.ctypes.data_as(I_P), n_seqs,
                                           ctypes.c_void_p(d_out_ptr), ctypes.c_void_p(stream or None))
        if rc != 0:
            raise RuntimeError(f"bert_amd_eval_device failed ({rc}): {last_error()}")

    def debug_embed(self, token_lists):
        """The embeddings + LayerNorm stage alone: (X f32 [M, E], q [M, E], d [M, E/32] or None)."""
        ids = np.ascontiguousarray(np.concatenate([np.asarray(t, np.int32) for t in token_lists]))
        offs = np.zeros(len(token_lists) + 1, np.int32)
        offs[1:] = np.cumsum([len(t) for t in token_lists])
        M, E, wt = len(ids), self.n_embd, self.hparams[6]
        X = np.zeros((M, E), np.float32)
        q = np.zeros((M, E), {0: np.float32, 1: np.float16, 2: np.int8, 3: np.int8}[wt])
        d = np.zeros((M, E // 32), np.float16 if wt == 2 else np.float32) if wt in (2, 3) else None
        rc = self.lib.bert_amd_debug_embed(self.ctx, ids.ctypes.data_as(I_P), offs.ctypes.data_as(I_P), len(token_lists),
                                           X.ctypes.data_as(F_P), q.ctypes.data_as(ctypes.c_void_p),
                                           d.ctypes.data_as(ctypes.c_void_p) if d is not None else None)
        if rc != 0:
            raise RuntimeError(f"bert_amd_debug_embed failed ({rc}): {last_error()}")
        return X, q, d

    def debug_layers(self, token_lists):
        """The residual stream after every stage (bert_amd_debug_layers): X f32
        [n_layer + 1, M, E], q [n_layer + 1, M, E] and d [n_layer + 1, M, E/32]
        (None for F16 / F32) — stage 0 the embeddings + LN, stage l + 1 layer l."""
        ids = np.ascontiguousarray(np.concatenate([np.asarray(t, np.int32) for t in token_lists]))
        offs = np.zeros(len(token_lists) + 1, np.int32)
        offs[1:] = np.cumsum([len(t) for t in token_lists])
        M, E, wt, S = len(ids), self.n_embd, self.hparams[6], self.hparams[5] + 1
        X = np.zeros((S, M, E), np.float32)
        q = np.zeros((S, M, E), {0: np.float32, 1: np.float16, 2: np.int8, 3: np.int8}[wt])
        d = np.zeros((S, M, E // 32), np.float16 if wt == 2 else np.float32) if wt in (2, 3) else None
        rc = self.lib.bert_amd_debug_layers(self.ctx, ids.ctypes.data_as(I_P), offs.ctypes.data_as(I_P),
                                            len(token_lists), X.ctypes.data_as(F_P), q.ctypes.data_as(ctypes.c_void_p),
                                            d.ctypes.data_as(ctypes.c_void_p) if d is not None else None)
        if rc != 0:
            raise RuntimeError(f"bert_amd_debug_layers failed ({rc}): {last_error()}")
        return X, q, d

    def set_option(self, key: str, value: int) -> None:
        """bert_amd_set_option (include/bert_amd.h); results are identical under every setting."""
        if self.lib.bert_amd_set_option(self.ctx, key.encode(), int(value)) != 0:
            raise ValueError(f"bert_amd_set_option({key}, {value}) failed: {last_error()}")

    def get_option(self, key: str) -> int:
        """bert_amd_get_option: a pipeline option, or a resolved load-time choice
        ("qkva_ntw", "i8_qkv", "i8_up", "i8_o", "i8_down", "q41bf", "q41bf_qkv",
        "q41bf_o", "q41bf_up", "q41bf_down", "emb_raw")."""
        v = ctypes.c_int32(0)
        if self.lib.bert_amd_get_option(self.ctx, key.encode(), ctypes.byref(v)) != 0:
            raise ValueError(f"bert_amd_get_option({key}) failed: {last_error()}")
        return int(v.value)

    def workspace_rows(self, slot: int = 0) -> int:
        return int(self.lib.bert_amd_workspace_rows(self.ctx, slot))

    def profile(self, enable: bool) -> None:
        self.lib.bert_amd_profile_enable(self.ctx, 1 if enable else 0)

    def profile_read(self) -> dict:
        names = ctypes.create_string_buffer(4096)
        ms = (ctypes.c_float * 64)()
        cnt = (ctypes.c_int32 * 64)()
        n = self.lib.bert_amd_profile_read(self.ctx, names, 4096, ms, cnt, 64)
        keys = names.raw.split(b"\0")[:n]
        return {k.decode(): (float(ms[i]), int(cnt[i])) for i, k in enumerate(keys)}
