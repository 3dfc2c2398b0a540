"""Small batches of short sentences with and without the fused small QKV +
attention kernel (option small_qkva): bert_eval_batch on B sentences of L
tokens (host buffers), median of 50, alternating the option.  One JSON line per
batch size.

    python3 tools/qkva_batch_probe.py [L]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedding.cpp_amd"))
import bertlib  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 48
path = "/tmp/bert_amd_models/minilm_q4_0_s20250117_w0.05.gguf"
if not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    bertlib.synth_model(path, "minilm", "q4_0", seed=20250117, w_std=0.05)
m = bertlib.BertModel(path, devices=[0])
rng = np.random.default_rng(5)
for B in (1, 4, 8, 16, 32, 47):
    toks = [[101] + rng.integers(1000, 30000, L - 2).tolist() + [102] for _ in range(B)]
    res = {"sentences": B, "tokens": L, "rows": B * L}
    outs = {}
    for rep in range(2):
        for v in (1, 0):
            m.set_option("small_qkva", v)
            for _ in range(5):
                outs[v] = m.eval_batch(toks)
            ts = []
            for _ in range(50):
                t0 = time.perf_counter()
                m.eval_batch(toks)
                ts.append(time.perf_counter() - t0)
            res.setdefault(f"us_small_qkva_{v}", []).append(round(float(np.median(ts)) * 1e6, 1))
    res["bitwise"] = bool(np.array_equal(outs[0], outs[1]))
    print(json.dumps(res), flush=True)
m.close()
