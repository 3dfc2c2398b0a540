"""bert_encode_batch through bert.h only (ctypes, as the reference's
examples/sample_dylib.py binds it), for A/B of library builds across rounds
(a build without this round's bert_amd_* extensions loads too).

    python3 tools/consumer_ab.py <libbert.so> <model.gguf> [n_texts]

Prints one JSON line: embeddings/s at n_batch_size 16 / 256 / all (median of 5
after a warm-up), the same synthetic texts as bench.py's consumer line.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

lib_path, model = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
L = ctypes.CDLL(os.path.abspath(lib_path))
L.bert_load_from_file.restype = ctypes.c_void_p
L.bert_load_from_file.argtypes = [ctypes.c_char_p]
L.bert_vocab_id_to_token.restype = ctypes.c_char_p
L.bert_vocab_id_to_token.argtypes = [ctypes.c_void_p, ctypes.c_int32]
L.bert_n_embd.restype = ctypes.c_int32
L.bert_n_embd.argtypes = [ctypes.c_void_p]
F_P = ctypes.POINTER(ctypes.c_float)
L.bert_encode_batch.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(F_P)]
L.bert_free.argtypes = [ctypes.c_void_p]
saved = os.dup(1)
os.dup2(2, 1)
ctx = L.bert_load_from_file(model.encode())
os.dup2(saved, 1)
assert ctx, "load failed"
words = []
for i in range(1000, 30522):
    w = L.bert_vocab_id_to_token(ctx, i).decode("utf-8", "replace")
    if w.isalpha() and w.islower() and not w.startswith("##"):
        words.append(w)
rng = np.random.default_rng(20250117 + 7)
lens = rng.integers(8, 129, n)
texts = [" ".join(rng.choice(words, k - 2)) for k in lens]
c_texts = (ctypes.c_char_p * n)(*[t.encode("utf-8") for t in texts])
E = L.bert_n_embd(ctx)
emb = np.zeros((n, E), np.float32)
ptrs = (F_P * n)(*[emb[i].ctypes.data_as(F_P) for i in range(n)])
threads = int(os.environ.get("OMP_NUM_THREADS", 0) or 8)
res = {"lib": lib_path}
for bs in (16, 256, n):
    L.bert_encode_batch(ctx, threads, bs, n, c_texts, ptrs)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        L.bert_encode_batch(ctx, threads, bs, n, c_texts, ptrs)
        ts.append(time.perf_counter() - t0)
    res[f"bs{'all' if bs == n else bs}"] = round(n / float(np.median(ts)), 1)
L.bert_free(ctx)
print(json.dumps(res), flush=True)
