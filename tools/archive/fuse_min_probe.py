"""fuse_min A/B on small batches of short sentences: bert_eval_batch medians with
the producer/consumer kernel (fuse_min 48) and without (fuse_min 100000: the
small fused QKV + attention kernel).  python3 tools/fuse_min_probe.py"""
import json, os, sys, time
import numpy as np
sys.path.insert(0, "embedding.cpp_amd")
import bertlib
path = "/tmp/bert_amd_models/minilm_q4_0_s20250117_w0.05.gguf"
if not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    bertlib.synth_model(path, "minilm", "q4_0", seed=20250117, w_std=0.05)
m = bertlib.BertModel(path, devices=[0])
rng = np.random.default_rng(5)
for L in (16, 32, 48):
    for B in (48, 64, 96, 128):
        if B * L > 2048: continue
        toks = [[101] + rng.integers(1000, 30000, L - 2).tolist() + [102] for _ in range(B)]
        res = {"B": B, "L": L}
        outs = {}
        for rep in range(2):
            for fm in (48, 100000):
                m.set_option("fuse_min", fm)
                for _ in range(5): outs[fm] = m.eval_batch(toks)
                ts = []
                for _ in range(50):
                    t0 = time.perf_counter(); m.eval_batch(toks); ts.append(time.perf_counter() - t0)
                res.setdefault(f"fuse_min_{fm}", []).append(round(float(np.median(ts)) * 1e6, 1))
        res["bitwise"] = bool(np.array_equal(outs[48], outs[100000]))
        print(json.dumps(res), flush=True)
m.close()
