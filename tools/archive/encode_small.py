"""Development: bert_encode_batch on synthetic texts at a small n_batch_size
(the reference consumers' 16), for rocprofv3 kernel traces of small slices.
    python tools/encode_small.py [batch_size] [n_texts] [lanes]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "embedding.cpp_amd"))
import bertlib  # noqa: E402

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 16
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
lanes = int(sys.argv[3]) if len(sys.argv) > 3 else 4
merge = int(sys.argv[4]) if len(sys.argv) > 4 else 1
d = os.environ.get("BERT_AMD_MODEL_DIR", "/tmp/bert_amd_models")
os.makedirs(d, exist_ok=True)
path = os.path.join(d, "minilm_q4_0_s20250117_w0.05.gguf")
if not os.path.exists(path):
    bertlib.synth_model(path, "minilm", "q4_0", seed=20250117, w_std=0.05)
m = bertlib.BertModel(path)
m.set_option("encode_lanes", lanes)
m.set_option("encode_merge", merge)
rng = np.random.default_rng(1)
words = [f"w{i}" for i in range(500)]
texts = [" ".join(rng.choice(words, int(k))) for k in rng.integers(3, 60, n)]
m.encode(texts, batch_size=bs)
t0 = time.perf_counter()
for _ in range(3):
    m.encode(texts, batch_size=bs)
dt = (time.perf_counter() - t0) / 3
print(f"batch {bs} lanes {lanes} merge {merge}: {n / dt:.1f} emb/s ({dt * 1e3:.2f} ms)", flush=True)
m.close()
