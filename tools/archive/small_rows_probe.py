"""Where the 32-row small-batch GEMM tiles stop paying (option small_rows):
bert_eval_batch on B sentences of 128 tokens (host buffers), median of 50,
with small_rows 0 (batch kernels only) and large enough for B.  One JSON line
per batch size.

    python3 tools/small_rows_probe.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedding.cpp_amd"))
import bertlib  # noqa: E402

path = "/tmp/bert_amd_models/minilm_q4_0_s20250117_w0.05.gguf"
if not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    bertlib.synth_model(path, "minilm", "q4_0", seed=20250117, w_std=0.05)
m = bertlib.BertModel(path, devices=[0])
rng = np.random.default_rng(5)
for B in (1, 2, 4, 8, 16, 32, 64):
    toks = [[101] + rng.integers(1000, 30000, 126).tolist() + [102] for _ in range(B)]
    res = {"sentences": B, "rows": 128 * B}
    for sr in (0, 1 << 20):
        m.set_option("small_rows", sr)
        for _ in range(5):
            m.eval_batch(toks)
        ts = []
        for _ in range(50):
            t0 = time.perf_counter()
            m.eval_batch(toks)
            ts.append(time.perf_counter() - t0)
        res[f"us_small_rows_{'off' if sr == 0 else 'on'}"] = round(float(np.median(ts)) * 1e6, 1)
    print(json.dumps(res), flush=True)
m.close()
