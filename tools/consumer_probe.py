"""Where bert_encode_batch's time goes (development probe): the same 4096
synthetic texts as bench.py's consumer line —
  tok16     bert_tokenize on 16 Python threads (ctypes releases the GIL)
  eval_all  bert_eval_batch on the pre-tokenised sentences (length-sorted)
  enc_all   bert_encode_batch, n_batch_size = all
  enc_16    bert_encode_batch, n_batch_size = 16
medians of 5 after a warm-up, ms.

    python3 tools/consumer_probe.py [model.gguf]
"""
import ctypes
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedding.cpp_amd"))
import bertlib  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/bert_amd_models/minilm_q4_0_s20250117_w0.05.gguf"
if not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    bertlib.synth_model(path, "minilm", "q4_0", seed=20250117, w_std=0.05)
m = bertlib.BertModel(path, devices=[0])
L, ctx = m.lib, m.ctx
words = []
for i in range(1000, 30522):
    w = L.bert_vocab_id_to_token(ctx, i).decode("utf-8", "replace")
    if w.isalpha() and w.islower() and not w.startswith("##"):
        words.append(w)
rng = np.random.default_rng(20250117 + 7)
n = 4096
lens = rng.integers(8, 129, n)
texts = [" ".join(rng.choice(words, k - 2)) for k in lens]
c_texts = (ctypes.c_char_p * n)(*[t.encode("utf-8") for t in texts])
threads = int(os.environ.get("OMP_NUM_THREADS", 0) or 16)


def tok_one(i):
    buf = (ctypes.c_int32 * 512)()
    nt = ctypes.c_int32(0)
    L.bert_tokenize(ctx, c_texts[i], buf, ctypes.byref(nt), 512)
    return np.frombuffer(buf, np.int32, nt.value).copy()


def med(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e3, 3)


res = {}
if os.environ.get("PROBE_ENC_ONLY"):  # (under a tracer: one warm-up and one timed bert_encode_batch, all at once)
    emb = np.zeros((n, 384), np.float32)
    ptrs = (bertlib.F_P * n)(*[emb[i].ctypes.data_as(bertlib.F_P) for i in range(n)])
    bs = int(os.environ["PROBE_ENC_ONLY"])
    L.bert_encode_batch(ctx, threads, bs, n, c_texts, ptrs)
    t0 = time.perf_counter()
    L.bert_encode_batch(ctx, threads, bs, n, c_texts, ptrs)
    print(json.dumps({"enc_ms": round((time.perf_counter() - t0) * 1e3, 3), "bs": bs}), flush=True)
    m.close()
    sys.exit(0)
pool = ThreadPoolExecutor(16)
res["tok16"] = med(lambda: list(pool.map(tok_one, range(n))))
toks = list(pool.map(tok_one, range(n)))
order = np.argsort([len(t) for t in toks], kind="stable")
stoks = [toks[i] for i in order]
# bert_eval_batch on the same sentences, length-sorted, ctypes arrays built once
# (what bert_encode_batch does after tokenising): enc_all - eval_all_c = the
# tokenisation and sorting inside the library
I_P = ctypes.POINTER(ctypes.c_int32)
tok_arrs = [np.ascontiguousarray(t, dtype=np.int32) for t in stoks]
tp = (I_P * n)(*[a.ctypes.data_as(I_P) for a in tok_arrs])
tn = (ctypes.c_int32 * n)(*[len(a) for a in tok_arrs])
embs_sorted = np.zeros((n, 384), np.float32)
eo = [int(i) for i in order]
ep = (bertlib.F_P * n)(*[embs_sorted[eo[i]].ctypes.data_as(bertlib.F_P) for i in range(n)])
res["eval_all_c"] = med(lambda: L.bert_eval_batch(ctx, threads, n, tp, tn, ep))
emb = np.zeros((n, 384), np.float32)
ptrs = (bertlib.F_P * n)(*[emb[i].ctypes.data_as(bertlib.F_P) for i in range(n)])
res["enc_all"] = med(lambda: L.bert_encode_batch(ctx, threads, n, n, c_texts, ptrs))
res["enc_16"] = med(lambda: L.bert_encode_batch(ctx, threads, 16, n, c_texts, ptrs))
res["enc_256"] = med(lambda: L.bert_encode_batch(ctx, threads, 256, n, c_texts, ptrs))
print(json.dumps(res), flush=True)
m.close()
